// Hand-written stable LSD radix sort of (key, value) u32 pairs for the MSM's bucket sort
// (gfx950; round 3, replacing hipcub::DeviceRadixSort). Keys are bucket ids of at most 24
// bits (the fixed-base form: 16, 20 or 22 bits, the windowed form: 20), so 2-3 passes of
// digits of at most 8 bits.
// Each pass is three kernels and touches no global atomics:
//   rs_hist     per tile of RS_TILE entries: its digit histogram (LDS atomics) -> hist[d][tile]
//   rs_scan     per digit: exclusive prefix over the tiles, in place, and the digit's total
//   rs_scatter  per tile: stable ranks (each wave ranks a contiguous quarter of the tile: wave
//               ballots match equal digits, a wave-private LDS counter per digit orders its
//               rounds; the per-wave counts, scanned, order the waves), a locally sorted copy
//               of the tile in LDS, then every digit's run written to its global position
//               (consecutive lanes write consecutive addresses of a run)
// A pass may read its input from RsDigitsT instead of (keys, vals): the fixed-base MSM's first
// pass takes planar 16-bit (32-bit for windows wider than 16 bits) signed digits and derives
// each entry's key and value from the digit and the entry index, so the digit kernel writes
// 2 (4) B per entry instead of 8 and the first pass reads 2 (4) B instead of 4 (histogram)
// and 8 (scatter).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbf {

#ifndef PBF_RS_ITEMS
#define PBF_RS_ITEMS 32
#endif
// RS_ITEMS entries per thread (a tile of 8192 entries: 64 KiB of LDS for the locally sorted
// copy, two workgroups per CU; runs of ~32 entries per digit and tile on the store side; 2^28
// pairs: 5.1 ms with 4096-entry tiles, 4.0 ms with 8192, scripts/ubench/sort_bench.hip).
// RS_TILE: the smallest tile any caller may pick (it sizes the histogram scratch); RS_TILE_MAX
// the largest (it bounds m).
constexpr int RS_T = 256, RS_ITEMS = PBF_RS_ITEMS, RS_TILE = RS_T * 16, RS_TILE_MAX = RS_T * 64;

// Signed digit code of C = uint16_t (windows of up to 16 bits) or uint32_t (wider fixed-base
// windows): |d| - 1 for d > 0, the top bit | (|d| - 1) for d < 0, all ones (rs_none<C>) for
// no entry (a zero digit or an identity point)
constexpr uint16_t RS_DIG_NONE = 0xFFFF;
template <typename C>
__host__ __device__ constexpr uint32_t rs_none() { return (uint32_t)(C)~(C)0; }
template <typename C>
__host__ __device__ constexpr uint32_t rs_sign() { return (uint32_t)1 << (8 * sizeof(C) - 1); }
template <typename C>
struct RsDigitsT {
  const C* dig;       // dig[w * n + i]: window w's digit code of scalar i
  uint32_t n;         // scalars
  uint32_t n_table;   // value of entry (w, i) = w * n_table + first + i, | neg if d < 0
  uint32_t first;
  uint32_t kw;    // key of entry (w, i) = w * kw + (|d| - 1) (fixed base: 0; windowed: 2^15)
  uint32_t zkey;  // key of a no-entry code (sorts last)
  uint32_t neg;   // sign flag of the value
};
using RsDigits = RsDigitsT<uint16_t>;
template <typename C>
__device__ __forceinline__ uint32_t rs_dig_key(uint32_t c, uint32_t w, const RsDigitsT<C>& dg) {
  return c == rs_none<C>() ? dg.zkey : w * dg.kw + (c & (rs_sign<C>() - 1));
}

template <int ITEMS, bool DIG = false, typename C = uint16_t>
__global__ void __launch_bounds__(RS_T) rs_hist(const uint32_t* keys, uint32_t m, uint32_t shift, uint32_t mask,
                                                uint32_t ntiles, uint32_t* hist, RsDigitsT<C> dg) {
  __shared__ uint32_t h[RS_T / 64][256];  // one histogram per wave (less atomic contention)
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int w = 0; w < RS_T / 64; ++w) h[w][threadIdx.x] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * (RS_T * ITEMS);
  uint32_t k[ITEMS];
  // four consecutive entries per load (round 6: 16-B key / 8-B code loads; the histogram does
  // not care which thread counts an entry); the tile's ragged end entry by entry
  static_assert(ITEMS % 4 == 0, "four entries per load");
#pragma unroll
  for (int u = 0; u < ITEMS / 4; ++u) {
    const uint32_t e = base + 4 * (u * RS_T + threadIdx.x);
    uint32_t raw[4];
    if constexpr (DIG) {
      if (e + 4 <= m) {
        if constexpr (sizeof(C) == 4) {
          const uint4 v = *reinterpret_cast<const uint4*>(dg.dig + e);
          raw[0] = v.x; raw[1] = v.y; raw[2] = v.z; raw[3] = v.w;
        } else {
          const uint2 v = *reinterpret_cast<const uint2*>(dg.dig + e);
          raw[0] = v.x & 0xFFFFu; raw[1] = v.x >> 16; raw[2] = v.y & 0xFFFFu; raw[3] = v.y >> 16;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) raw[q] = e + q < m ? (uint32_t)dg.dig[e + q] : 0u;
      }
      // pass 1 (shift 0, kw a multiple of 256): the digit follows from the code alone
#pragma unroll
      for (int q = 0; q < 4; ++q)
        k[4 * u + q] = e + q < m ? (raw[q] == rs_none<C>() ? dg.zkey : raw[q] & (rs_sign<C>() - 1)) : 0xFFFFFFFFu;
    } else {
      if (e + 4 <= m) {
        const uint4 v = *reinterpret_cast<const uint4*>(keys + e);
        raw[0] = v.x; raw[1] = v.y; raw[2] = v.z; raw[3] = v.w;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) raw[q] = e + q < m ? keys[e + q] : 0xFFFFFFFFu;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) k[4 * u + q] = raw[q];
    }
  }
#pragma unroll
  for (int u = 0; u < ITEMS; ++u)
    if (k[u] != 0xFFFFFFFFu) atomicAdd(&h[wave][(k[u] >> shift) & mask], 1u);
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
constexpr int RS_WAVES = RS_T / 64;
template <int ITEMS, bool DIG = false, typename C = uint16_t>
__global__ void __launch_bounds__(RS_T) __attribute__((amdgpu_waves_per_eu(2))) rs_scatter(const uint32_t* keys, const uint32_t* vals, uint32_t* okeys,
                                                   uint32_t* ovals, uint32_t m, uint32_t shift, uint32_t mask,
                                                   uint32_t ntiles, const uint32_t* hist, const uint32_t* total,
                                                   RsDigitsT<C> dg) {
  __shared__ uint32_t s[RS_T];
  __shared__ uint32_t gbase[256], lstart[256];
  __shared__ uint32_t wc[RS_WAVES][256];
  constexpr int TILE = RS_T * ITEMS, RS_WQ = TILE / RS_WAVES;  // entries per tile / per wave
  __shared__ uint32_t lk[TILE], lv[TILE];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const uint32_t tile = blockIdx.x, base = tile * TILE;
  // this wave's entries (all loads first: their latency overlaps the setup below)
  // DIG: key[r] holds the raw 16-bit code, no value registers: the digit of pass 1 (shift 0,
  // kw a multiple of 256) follows from the code alone; key and value from the code and the
  // entry index when the entry is placed in LDS
  uint32_t key[ITEMS], val[DIG ? 1 : ITEMS];
  const uint32_t e0 = base + wave * RS_WQ + lane;  // this lane's entries are 64 apart
  if constexpr (DIG) {
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t e = e0 + r * 64;
      key[r] = e < m ? (uint32_t)dg.dig[e] : rs_none<C>();
    }
  } else {
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t e = base + wave * RS_WQ + r * 64 + lane;
      key[r] = e < m ? keys[e] : 0;
      val[r] = e < m ? vals[e] : 0;
    }
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
  uint32_t rank[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const bool valid = base + wave * RS_WQ + r * 64 + lane < m;
    const uint32_t d =
        DIG ? (key[r] == rs_none<C>() ? dg.zkey : key[r] & (rs_sign<C>() - 1)) & mask : (key[r] >> shift) & mask;
    // match-any over the digit's bits (round 6): per bit one ballot, then per 32-bit half
    // peers &= ~(ballot ^ m) with m = 0 or ~0 the lane's bit: two 3-input logic operations
    // instead of a 64-bit select (a uniform skip of the bits above the pass's width measured
    // slower: profiles/r06/sort_match_ab.log)
    const uint64_t pv = __ballot(valid);
    uint32_t plo = (uint32_t)pv, phi = (uint32_t)(pv >> 32);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      // (bits above the width: every lane 0, the ballot 0, peers unchanged)
      const uint32_t mk = (uint32_t)__builtin_amdgcn_sbfe((int32_t)d, b, 1);  // 0 or ~0
      const uint64_t bal = __ballot(mk);
      plo &= ~((uint32_t)bal ^ mk);
      phi &= ~((uint32_t)(bal >> 32) ^ mk);
    }
    const uint64_t peers = ((uint64_t)phi << 32) | plo;
    const uint32_t before = __popcll(peers & below);
    rank[r] = wc[wave][d] + before;  // this wave's earlier entries of digit d, then this round's
    if (valid && before == 0) wc[wave][d] += __popcll(peers);
    // the next round's lanes read counters this round's leader lanes wrote: order the LDS
    // accesses across lanes explicitly (wavefront-scope fence + scheduling barrier)
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
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
  if constexpr (DIG) {
    uint32_t w = e0 / dg.n, i = e0 - w * dg.n;
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      if (e0 + r * 64 < m) {
        const uint32_t c = key[r], k = rs_dig_key(c, w, dg);
        const uint32_t d = k & mask;
        const uint32_t pos = lstart[d] + wc[wave][d] + rank[r];
        lk[pos] = k;
        lv[pos] = (w * dg.n_table + dg.first + i) | (c != rs_none<C>() && (c & rs_sign<C>()) ? dg.neg : 0u);
      }
      i += 64;
      const bool wrap = i >= dg.n;
      i -= wrap ? dg.n : 0u;
      w += wrap ? 1u : 0u;
    }
  } else {
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      if (e0 + r * 64 < m) {
        const uint32_t d = (key[r] >> shift) & mask;
        const uint32_t pos = lstart[d] + wc[wave][d] + rank[r];
        lk[pos] = key[r];
        lv[pos] = val[r];
      }
    }
  }
  __syncthreads();
  const uint32_t count = m - base < (uint32_t)TILE ? m - base : (uint32_t)TILE;
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t i = r * RS_T + t;
    if (i < count) {
      const uint32_t k = lk[i];
      const uint32_t d = (k >> shift) & mask;
      const uint32_t o = gbase[d] + (i - lstart[d]);
      okeys[o] = k;
      ovals[o] = lv[i];
    }
  }
}


// One pass: (kin, vin) (or dg) -> (kout, vout) stably sorted by key bits [shift, shift + dbits),
// dbits <= 8 (narrower digits: longer runs per digit and tile on the store side).
// hist: 256 * ntiles + 256 u32 of scratch.
// DIG (pass 1 only, shift 0) requires dg.n >= RS_T (rs_dig_ok) and dg.kw % 2^dbits == 0.
inline bool rs_dig_ok(uint64_t n) { return n >= (uint64_t)RS_T; }
template <int ITEMS = RS_ITEMS, bool DIG = false, typename C = uint16_t>
inline void rs_pass(const uint32_t* kin, const uint32_t* vin, uint32_t* kout, uint32_t* vout, uint32_t m,
                    uint32_t shift, uint32_t* hist, hipStream_t s, RsDigitsT<C> dg = {}, int dbits = 8) {
  constexpr uint32_t TILE = RS_T * ITEMS;
  static_assert(ITEMS >= 16 && TILE <= RS_TILE_MAX, "the scratch is sized for RS_TILE .. RS_TILE_MAX");
  const uint32_t ntiles = (m + TILE - 1) / TILE, mask = (1u << dbits) - 1;
  uint32_t* total = hist + 256ull * ntiles;
  hipLaunchKernelGGL((rs_hist<ITEMS, DIG, C>), dim3(ntiles), dim3(RS_T), 0, s, kin, m, shift, mask, ntiles, hist, dg);
  hipLaunchKernelGGL(rs_scan, dim3(256), dim3(RS_T), 0, s, hist, ntiles, total);
  hipLaunchKernelGGL((rs_scatter<ITEMS, DIG, C>), dim3(ntiles), dim3(RS_T), 0, s, kin, vin, kout, vout, m, shift, mask,
                     ntiles, (const uint32_t*)hist, (const uint32_t*)total, dg);
}

// digit widths of a `bits`-bit sort: ceil(bits / 8) passes, widths as equal as possible (the
// wider ones first): 16 -> 8, 8; 20 -> 7, 7, 6; 22 -> 8, 7, 7
inline int rs_passes(int bits) { return (bits + 7) / 8; }
inline int rs_width(int bits, int p) {
  const int np = rs_passes(bits), base = bits / np;
  return base + (p < bits % np ? 1 : 0);
}

// Sort m pairs by key bits [0, bits): keys/vals -> keys2/vals2 (inputs unchanged; tmpk / tmpv:
// m u32 each of ping-pong scratch). hist: 256 * ntiles + 256 u32 of scratch.
template <int ITEMS = RS_ITEMS>
inline int rs_sort(const uint32_t* keys, const uint32_t* vals, uint32_t* keys2, uint32_t* vals2, uint32_t* tmpk,
                   uint32_t* tmpv, uint32_t m, int bits, uint32_t* hist, hipStream_t s) {
  if (m == 0) return 0;
  const int passes = rs_passes(bits);
  // pass p reads (k_in, v_in) and writes (k_out, v_out); the last pass writes keys2 / vals2
  const uint32_t* kin = keys;
  const uint32_t* vin = vals;
  int shift = 0;
  for (int p = 0; p < passes; ++p) {
    // an even number of passes left after this one writes tmp, else keys2 (so the last lands there)
    uint32_t* kout = ((passes - 1 - p) % 2 == 0) ? keys2 : tmpk;
    uint32_t* vout = ((passes - 1 - p) % 2 == 0) ? vals2 : tmpv;
    rs_pass<ITEMS>(kin, vin, kout, vout, m, (uint32_t)shift, hist, s, RsDigits{}, rs_width(bits, p));
    shift += rs_width(bits, p);
    kin = kout;
    vin = vout;
  }
  return 0;
}

}  // namespace pbf
