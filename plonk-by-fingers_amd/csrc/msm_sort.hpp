// Hand-written stable LSD radix sort of (key, value) u32 pairs for the MSM's bucket sort
// (gfx950; round 3, replacing hipcub::DeviceRadixSort). Keys are bucket ids of at most 20
// bits (the fixed-base form: 16 bits, the windowed form: 20), so 2-3 passes of 8-bit digits.
// Each pass is three kernels and touches no global atomics:
//   rs_hist     per tile of RS_TILE entries: its digit histogram (LDS atomics) -> hist[d][tile]
//   rs_scan     per digit: exclusive prefix over the tiles, in place, and the digit's total
//   rs_scatter  per tile: stable ranks (each wave ranks a contiguous quarter of the tile: wave
//               ballots match equal digits, a wave-private LDS counter per digit orders its
//               rounds; the per-wave counts, scanned, order the waves), a locally sorted copy
//               of the tile in LDS, then every digit's run written to its global position
//               (consecutive lanes write consecutive addresses of a run)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbf {

constexpr int RS_T = 256, RS_ITEMS = 16, RS_TILE = RS_T * RS_ITEMS;

__global__ void __launch_bounds__(RS_T) rs_hist(const uint32_t* keys, uint32_t m, uint32_t shift, uint32_t ntiles,
                                                uint32_t* hist) {
  __shared__ uint32_t h[RS_T / 64][256];  // one histogram per wave (less atomic contention)
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int w = 0; w < RS_T / 64; ++w) h[w][threadIdx.x] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * RS_TILE;
  uint32_t k[RS_ITEMS];
#pragma unroll
  for (int u = 0; u < RS_ITEMS; ++u) {
    const uint32_t e = base + u * RS_T + threadIdx.x;
    k[u] = e < m ? keys[e] : 0xFFFFFFFFu;
  }
#pragma unroll
  for (int u = 0; u < RS_ITEMS; ++u)
    if (k[u] != 0xFFFFFFFFu) atomicAdd(&h[wave][(k[u] >> shift) & 255], 1u);
  __syncthreads();
  uint32_t c = 0;
#pragma unroll
  for (int w = 0; w < RS_T / 64; ++w) c += h[w][threadIdx.x];
  hist[threadIdx.x * ntiles + blockIdx.x] = c;
}

// inclusive scan of one value per thread over the workgroup (RS_T threads)
__device__ __forceinline__ uint32_t rs_block_scan(uint32_t v, uint32_t* s) {
  s[threadIdx.x] = v;
  __syncthreads();
  for (int off = 1; off < RS_T; off <<= 1) {
    const uint32_t x = (int)threadIdx.x >= off ? s[threadIdx.x - off] : 0;
    __syncthreads();
    s[threadIdx.x] += x;
    __syncthreads();
  }
  return s[threadIdx.x];
}

// workgroup d: hist[d][*] -> exclusive prefix over the tiles; total[d] = the digit's count
__global__ void __launch_bounds__(RS_T) rs_scan(uint32_t* hist, uint32_t ntiles, uint32_t* total) {
  __shared__ uint32_t s[RS_T];
  uint32_t* row = hist + (uint64_t)blockIdx.x * ntiles;
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < ntiles; c0 += RS_T * 4) {
    uint32_t v[4], sum = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = c0 + threadIdx.x * 4 + j;
      v[j] = i < ntiles ? row[i] : 0;
      sum += v[j];
    }
    const uint32_t inc = rs_block_scan(sum, s);
    uint32_t ex = carry + inc - sum;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = c0 + threadIdx.x * 4 + j;
      if (i < ntiles) row[i] = ex;
      ex += v[j];
    }
    carry += s[RS_T - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) total[blockIdx.x] = carry;
}

// Wave w ranks the contiguous quarter [w*1024, (w+1)*1024) of the tile in 16 rounds of 64
// entries: ballots find the lanes holding the same digit, a wave-private LDS counter per
// digit orders the rounds (one wave's LDS accesses are ordered: no barrier between rounds).
// Then the per-wave counts are scanned across the waves, every entry goes to its slot of a
// locally sorted copy of the tile in LDS, and each digit's run is written to its global
// position.
constexpr int RS_WAVES = RS_T / 64, RS_WQ = RS_TILE / RS_WAVES;  // entries per wave
__global__ void __launch_bounds__(RS_T) rs_scatter(const uint32_t* keys, const uint32_t* vals, uint32_t* okeys,
                                                   uint32_t* ovals, uint32_t m, uint32_t shift, uint32_t ntiles,
                                                   const uint32_t* hist, const uint32_t* total) {
  __shared__ uint32_t s[RS_T];
  __shared__ uint32_t gbase[256], lstart[256];
  __shared__ uint32_t wc[RS_WAVES][256];
  __shared__ uint32_t lk[RS_TILE], lv[RS_TILE];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const uint32_t tile = blockIdx.x, base = tile * RS_TILE;
  // this wave's entries (all loads first: their latency overlaps the setup below)
  uint32_t key[RS_ITEMS], val[RS_ITEMS];
#pragma unroll
  for (int r = 0; r < RS_ITEMS; ++r) {
    const uint32_t e = base + wave * RS_WQ + r * 64 + lane;
    key[r] = e < m ? keys[e] : 0;
    val[r] = e < m ? vals[e] : 0;
  }
  // global start of digit t's run of this tile; this tile's count of digit t (from the
  // prefixes of this tile and the next); the local start of digit t (exclusive scan)
  const uint32_t tot = total[t];
  const uint32_t gtot_ex = rs_block_scan(tot, s) - tot;
  const uint32_t pre = hist[(uint64_t)t * ntiles + tile];
  const uint32_t nxt = tile + 1 < ntiles ? hist[(uint64_t)t * ntiles + tile + 1] : tot;
  const uint32_t mine = nxt - pre;
  __syncthreads();
  const uint32_t lex = rs_block_scan(mine, s) - mine;
  gbase[t] = gtot_ex + pre;
  lstart[t] = lex;
#pragma unroll
  for (int w = 0; w < RS_WAVES; ++w) wc[w][t] = 0;
  __syncthreads();
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t rank[RS_ITEMS];
#pragma unroll
  for (int r = 0; r < RS_ITEMS; ++r) {
    const bool valid = base + wave * RS_WQ + r * 64 + lane < m;
    const uint32_t d = (key[r] >> shift) & 255;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? bal : ~bal;
    }
    const uint32_t before = __popcll(peers & below);
    rank[r] = wc[wave][d] + before;  // this wave's earlier entries of digit d, then this round's
    if (valid && before == 0) wc[wave][d] += __popcll(peers);
  }
  __syncthreads();
  // wc[w][d] -> exclusive prefix over the waves (thread t owns digit t)
  {
    uint32_t acc = 0;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) {
      const uint32_t c = wc[w][t];
      wc[w][t] = acc;
      acc += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RS_ITEMS; ++r) {
    if (base + wave * RS_WQ + r * 64 + lane < m) {
      const uint32_t d = (key[r] >> shift) & 255;
      const uint32_t pos = lstart[d] + wc[wave][d] + rank[r];
      lk[pos] = key[r];
      lv[pos] = val[r];
    }
  }
  __syncthreads();
  const uint32_t count = m - base < (uint32_t)RS_TILE ? m - base : (uint32_t)RS_TILE;
#pragma unroll
  for (int r = 0; r < RS_ITEMS; ++r) {
    const uint32_t i = r * RS_T + t;
    if (i < count) {
      const uint32_t k = lk[i];
      const uint32_t d = (k >> shift) & 255;
      const uint32_t o = gbase[d] + (i - lstart[d]);
      okeys[o] = k;
      ovals[o] = lv[i];
    }
  }
}

// Sort m pairs by key bits [0, bits): keys/vals -> keys2/vals2 (inputs unchanged; tmpk / tmpv:
// m u32 each of ping-pong scratch). hist: 256 * ntiles + 256 u32 of scratch.
inline int rs_sort(const uint32_t* keys, const uint32_t* vals, uint32_t* keys2, uint32_t* vals2, uint32_t* tmpk,
                   uint32_t* tmpv, uint32_t m, int bits, uint32_t* hist, hipStream_t s) {
  if (m == 0) return 0;
  const uint32_t ntiles = (m + RS_TILE - 1) / RS_TILE;
  uint32_t* total = hist + 256ull * ntiles;
  const int passes = (bits + 7) / 8;
  // pass p reads (k_in, v_in) and writes (k_out, v_out); the last pass writes keys2 / vals2
  const uint32_t* kin = keys;
  const uint32_t* vin = vals;
  for (int p = 0; p < passes; ++p) {
    const bool last = p + 1 == passes;
    // an even number of passes left after this one writes tmp, else keys2 (so the last lands there)
    uint32_t* kout = ((passes - 1 - p) % 2 == 0) ? keys2 : tmpk;
    uint32_t* vout = ((passes - 1 - p) % 2 == 0) ? vals2 : tmpv;
    (void)last;
    hipLaunchKernelGGL(rs_hist, dim3(ntiles), dim3(RS_T), 0, s, kin, m, (uint32_t)(8 * p), ntiles, hist);
    hipLaunchKernelGGL(rs_scan, dim3(256), dim3(RS_T), 0, s, hist, ntiles, total);
    hipLaunchKernelGGL(rs_scatter, dim3(ntiles), dim3(RS_T), 0, s, kin, vin, kout, vout, m, (uint32_t)(8 * p), ntiles,
                       (const uint32_t*)hist, (const uint32_t*)total);
    kin = kout;
    vin = vout;
  }
  return 0;
}

}  // namespace pbf
