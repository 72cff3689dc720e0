// One-sweep radix sort (round 6, measured and not kept): the kernels that
// scripts/ubench/sort_os_bench.hip times against the library's three-kernel passes
// (plonk-by-fingers_amd/csrc/msm_sort.hpp). Measurement code, not part of libpbf.so.
#pragma once
#include "../../plonk-by-fingers_amd/csrc/msm_sort.hpp"

namespace pbf {

// ---- One-sweep form (round 6). One upsweep (rs_os_hist) counts every pass's digits over the
// whole input; each pass is then ONE kernel (rs_os_scatter): a workgroup takes the next tile
// index from the pass's counter, ranks its entries as rs_scatter does, publishes its per-digit
// counts in a status word per (tile, digit), and sums the counts of all earlier tiles by
// decoupled look-back. Against rs_pass this drops every later pass's histogram kernel (a full
// read of the keys) and every pass's scan; tile t still covers entries [t TILE, (t + 1) TILE)
// and is placed after tiles 0..t-1, so the output is the same stable order.
// Status word (8 B, one `sc1` store, read by `sc1` loads: an untorn {count, tag} granule,
// MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility"): count in the low
// half, tag 2 epoch (this tile's count only) or 2 epoch + 1 (count of tiles 0..t) in the high
// half. Every pass of the process takes a fresh epoch, so the status array is never cleared.
// Progress: a workgroup waits only on smaller tile indices, taken by workgroups already running.
#ifndef PBF_RS_OS_TILE
#define PBF_RS_OS_TILE 1
#endif
constexpr int RS_OS_MAXP = 3;
#ifndef PBF_RS_OS_LB
#define PBF_RS_OS_LB 8
#endif
constexpr int RS_OS_LB = PBF_RS_OS_LB;  // status words polled per look-back step
struct RsOsPasses {
  uint32_t np;
  uint32_t shift[RS_OS_MAXP], mask[RS_OS_MAXP];
};
// the upsweep's counts land in RS_OS_REP replicas (fewer atomics on one address); the scatter
// adds them up
constexpr int RS_OS_REP = 8;
// counters: RS_OS_MAXP per-pass tile counters, then an error flag (a look-back that gave up)
constexpr int RS_OS_ERR = RS_OS_MAXP;
constexpr uint32_t RS_OS_POLL_MAX = 1u << 18;  // bounded wait: the grid always drains

// ghist[p * 256 + d] += the count of digit d of pass p over the input (ghist zeroed before)
template <int ITEMS, bool DIG, typename C>
__global__ void __launch_bounds__(RS_T) rs_os_hist(const uint32_t* keys, uint32_t m, RsOsPasses ps, uint32_t* ghist,
                                                   RsDigitsT<C> dg) {
  __shared__ uint32_t h[RS_WAVES][RS_OS_MAXP][256];
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int w = 0; w < RS_WAVES; ++w)
#pragma unroll
    for (int p = 0; p < RS_OS_MAXP; ++p) h[w][p][threadIdx.x] = 0;
  __syncthreads();
  constexpr uint32_t TILE = RS_T * ITEMS;
  const uint32_t ntiles = (m + TILE - 1) / TILE;
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint32_t e0 = tile * TILE + threadIdx.x;
    uint32_t k[ITEMS];
    if constexpr (DIG) {
      // entry e = w n + i (n >= RS_T: at most one wrap per step of RS_T)
      uint32_t w = e0 / dg.n, i = e0 - w * dg.n;
#pragma unroll
      for (int u = 0; u < ITEMS; ++u) {
        const uint32_t e = e0 + u * RS_T;
        k[u] = e < m ? rs_dig_key((uint32_t)dg.dig[e], w, dg) : 0xFFFFFFFFu;
        i += RS_T;
        const bool wrap = i >= dg.n;
        i -= wrap ? dg.n : 0u;
        w += wrap ? 1u : 0u;
      }
    } else {
#pragma unroll
      for (int u = 0; u < ITEMS; ++u) {
        const uint32_t e = e0 + u * RS_T;
        k[u] = e < m ? keys[e] : 0xFFFFFFFFu;
      }
    }
#pragma unroll
    for (int u = 0; u < ITEMS; ++u)
      if (k[u] != 0xFFFFFFFFu)
        for (uint32_t p = 0; p < ps.np; ++p) atomicAdd(&h[wave][p][(k[u] >> ps.shift[p]) & ps.mask[p]], 1u);
  }
  __syncthreads();
  for (uint32_t p = 0; p < ps.np; ++p) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) c += h[w][p][threadIdx.x];
    if (c) atomicAdd(&ghist[(blockIdx.x % RS_OS_REP) * RS_OS_MAXP * 256 + p * 256 + threadIdx.x], c);
  }
}

__device__ __forceinline__ void rs_os_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t rs_os_load(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// status words of digit t of tiles j-1, j-2, ... (at most RS_OS_LB, none below tile 0)
__device__ __forceinline__ void rs_os_window(uint64_t (&v)[RS_OS_LB], const uint64_t* status, uint32_t j, int t) {
#pragma unroll
  for (int q = 0; q < RS_OS_LB; ++q) v[q] = (uint32_t)q < j ? rs_os_load(status + (uint64_t)(j - 1 - q) * 256 + t) : 0;
}

// One pass of the one-sweep form: (keys, vals) (or dg) -> (okeys, ovals) stably sorted by key
// bits [shift, shift + dbits). total: this pass's 256 digit counts (rs_os_hist: replica r at
// total + r RS_OS_MAXP 256). status: 256
// words per tile; counters[pass]: zero before the pass; epoch: this pass's (>= 1, < 2^31).
template <int ITEMS, bool DIG = false, typename C = uint16_t>
__global__ void __launch_bounds__(RS_T) __attribute__((amdgpu_waves_per_eu(2)))
rs_os_scatter(const uint32_t* keys, const uint32_t* vals, uint32_t* okeys, uint32_t* ovals, uint32_t m,
              uint32_t shift, uint32_t mask, const uint32_t* total, uint64_t* status, uint32_t* counters, uint32_t pass,
              uint32_t epoch, RsDigitsT<C> dg) {
  __shared__ uint32_t s[RS_T];
  __shared__ uint32_t gbase[256], lstart[256];
  __shared__ uint32_t wc[RS_WAVES][256];
  __shared__ uint32_t tile_s;
  constexpr int TILE = RS_T * ITEMS, RS_WQ = TILE / RS_WAVES;
  __shared__ uint32_t lk[TILE], lv[TILE];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  // the tile index comes from the pass's counter; workgroups are normally dispatched in index
  // order, so the entries of tile blockIdx.x are loaded before the counter's answer is known and
  // loaded again only if the answer differs
  uint32_t key[ITEMS], val[DIG ? 1 : ITEMS];
  auto load_tile = [&](uint32_t tl) {
    const uint32_t e0 = tl * TILE + wave * RS_WQ + lane;  // this lane's entries are 64 apart
    if constexpr (DIG) {
#pragma unroll
      for (int r = 0; r < ITEMS; ++r) {
        const uint32_t e = e0 + r * 64;
        key[r] = e < m ? (uint32_t)dg.dig[e] : rs_none<C>();
      }
    } else {
#pragma unroll
      for (int r = 0; r < ITEMS; ++r) {
        const uint32_t e = e0 + r * 64;
        key[r] = e < m ? keys[e] : 0;
        val[r] = e < m ? vals[e] : 0;
      }
    }
  };
#if PBF_RS_OS_TILE == 2  // measurement only (scripts/ubench/sort_os_bench.hip): blockIdx order assumed
  if (t == 0) tile_s = blockIdx.x;
#else
  if (t == 0) tile_s = __hip_atomic_fetch_add(counters + pass, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
#if PBF_RS_OS_TILE >= 1
  load_tile(blockIdx.x);
#endif
#pragma unroll
  for (int w = 0; w < RS_WAVES; ++w) wc[w][t] = 0;
  __syncthreads();
  const uint32_t tile = tile_s, base = tile * TILE;
#if PBF_RS_OS_TILE >= 1
  if (tile != blockIdx.x) load_tile(tile);
#else
  load_tile(tile);
#endif
  const uint32_t e0 = base + wave * RS_WQ + lane;
  uint32_t tot = 0;
#pragma unroll
  for (int r = 0; r < RS_OS_REP; ++r) tot += total[r * RS_OS_MAXP * 256 + t];
  const uint32_t gtot_ex = rs_block_scan(tot, s) - tot;
  // ranks within the wave's quarter, as rs_scatter
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t rank[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const bool valid = e0 + r * 64 < m;
    const uint32_t d =
        DIG ? (key[r] == rs_none<C>() ? dg.zkey : key[r] & (rs_sign<C>() - 1)) & mask : (key[r] >> shift) & mask;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bal = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? bal : ~bal;
    }
    const uint32_t before = __popcll(peers & below);
    rank[r] = wc[wave][d] + before;
    if (valid && before == 0) wc[wave][d] += __popcll(peers);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // this tile's count of digit t; wc[w][t] -> exclusive prefix over the waves
  uint32_t mine = 0;
#pragma unroll
  for (int w = 0; w < RS_WAVES; ++w) {
    const uint32_t c = wc[w][t];
    wc[w][t] = mine;
    mine += c;
  }
  // publish this tile's count of digit t, and issue the look-back's first loads (tiles
  // tile-1 .. tile-LB); their latency overlaps the local placement below
  const uint32_t agg_tag = 2u * epoch, inc_tag = 2u * epoch + 1u;
  uint64_t* st = status + (uint64_t)tile * 256 + t;
  uint32_t excl = 0, j = tile;  // tiles [j, tile) summed into excl
  uint64_t v[RS_OS_LB];
  rs_os_store(st, ((uint64_t)(tile == 0 ? inc_tag : agg_tag) << 32) | mine);
  if (tile > 0) rs_os_window(v, status, j, t);
  const uint32_t lex = rs_block_scan(mine, s) - mine;
  lstart[t] = lex;
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
  // the look-back: walk down from tile-1 adding counts until a tile's inclusive count
  if (tile > 0) {
    for (uint32_t poll = 0;; ++poll) {
      const uint32_t cnt = j < (uint32_t)RS_OS_LB ? j : (uint32_t)RS_OS_LB;
      bool stop = false, done = false;
      uint32_t adv = 0;
#pragma unroll
      for (int q = 0; q < RS_OS_LB; ++q) {
        if (!stop && (uint32_t)q < cnt) {
          const uint32_t tag = (uint32_t)(v[q] >> 32);
          if (tag == inc_tag) {
            excl += (uint32_t)v[q];
            stop = done = true;
          } else if (tag == agg_tag) {
            excl += (uint32_t)v[q];
            adv = q + 1;
          } else {
            stop = true;
          }
        }
      }
      if (done) break;
      j -= adv;
      if (poll >= RS_OS_POLL_MAX) {  // never expected: flag it and let the grid drain
        __hip_atomic_fetch_or(counters + RS_OS_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      if (adv == 0) __builtin_amdgcn_s_sleep(2);
      rs_os_window(v, status, j, t);
    }
    rs_os_store(st, ((uint64_t)inc_tag << 32) | (excl + mine));
  }
  gbase[t] = gtot_ex + excl;
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

// Scratch of the one-sweep sort of m entries: the status words (8 B per digit and tile) and a
// small block (per-pass digit counts, counters, error flag).
inline uint64_t rs_os_status_bytes(uint64_t m, int items = RS_ITEMS) {
  const uint64_t tile = (uint64_t)RS_T * items;
  return ((m + tile - 1) / tile) * 256 * 8;
}
constexpr uint64_t RS_OS_SMALL_BYTES = (RS_OS_REP * RS_OS_MAXP * 256 + 16) * 4;
// the process's next pass epoch (1 .. 2^31 - 1, wrapping)
uint32_t rs_os_next_epoch();

// The one-sweep sort: dg's codes (DIG) or (kin, vin) -> (kout, vout) by key bits [0, sum of
// widths), with np <= 3 passes of the given widths (each <= 8): pass 1 of 2 or 3 writes
// (t1k, t1v), pass 2 of 3 (t2k, t2v), the last pass (kout, vout). The input may alias (t2k, t2v)
// or (kout, vout) (read by the upsweep and pass 1 only). small: RS_OS_SMALL_BYTES of scratch,
// status: rs_os_status_bytes(m) (any content: see the epochs). A memset and np + 1 kernels on s.
template <int ITEMS = RS_ITEMS, bool DIG = false, typename C = uint16_t>
inline hipError_t rs_os_sort(const uint32_t* kin, const uint32_t* vin, uint32_t* t1k, uint32_t* t1v, uint32_t* t2k,
                             uint32_t* t2v, uint32_t* kout, uint32_t* vout, uint32_t m, int np, const int* widths,
                             uint32_t* small, uint64_t* status, hipStream_t s, RsDigitsT<C> dg = {}) {
  if (m == 0 || np < 1 || np > RS_OS_MAXP) return hipErrorInvalidValue;
  constexpr uint32_t TILE = RS_T * ITEMS;
  RsOsPasses ps{};
  ps.np = (uint32_t)np;
  uint32_t sh = 0;
  for (int p = 0; p < np; ++p) {
    ps.shift[p] = sh;
    ps.mask[p] = (1u << widths[p]) - 1;
    sh += (uint32_t)widths[p];
  }
  uint32_t* ghist = small;
  uint32_t* counters = small + RS_OS_REP * RS_OS_MAXP * 256;
  hipError_t e = hipMemsetAsync(small, 0, RS_OS_SMALL_BYTES, s);
  if (e != hipSuccess) return e;
  const uint32_t ntiles = (m + TILE - 1) / TILE;
  const uint32_t hgrid = ntiles < 2048 ? ntiles : 2048;
  hipLaunchKernelGGL((rs_os_hist<ITEMS, DIG, C>), dim3(hgrid), dim3(RS_T), 0, s, kin, m, ps, ghist, dg);
  const uint32_t* ki = kin;
  const uint32_t* vi = vin;
  for (int p = 0; p < np; ++p) {
    uint32_t* ko = p == np - 1 ? kout : (p == 0 ? t1k : t2k);
    uint32_t* vo = p == np - 1 ? vout : (p == 0 ? t1v : t2v);
    const uint32_t ep = rs_os_next_epoch();
    if (p == 0)
      hipLaunchKernelGGL((rs_os_scatter<ITEMS, DIG, C>), dim3(ntiles), dim3(RS_T), 0, s, ki, vi, ko, vo, m,
                         ps.shift[p], ps.mask[p], (const uint32_t*)ghist + p * 256, status, counters, (uint32_t)p, ep,
                         dg);
    else
      hipLaunchKernelGGL((rs_os_scatter<ITEMS, false, uint16_t>), dim3(ntiles), dim3(RS_T), 0, s, ki, vi, ko, vo, m,
                         ps.shift[p], ps.mask[p], (const uint32_t*)ghist + p * 256, status, counters, (uint32_t)p, ep,
                         RsDigits{});
    ki = ko;
    vi = vo;
  }
  return hipGetLastError();
}

}  // namespace pbf
