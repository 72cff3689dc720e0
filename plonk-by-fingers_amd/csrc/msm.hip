// BN254 G1 multi-scalar multiplication (BASELINE config 4) and batch fixed-base
// multiplication — the MI355X replacements of SRS::eval_at_s (src/plonk.rs:51-58, a
// naive left fold of g1s[i] * gf(c_i), each a double-and-add, src/pbh/g1.rs:146-168)
// and SRS::create (src/plonk.rs:35-48, g1s[i] = G * s^i).
//
// MSM = Pippenger, window c = 16 (16 windows over the 254-bit scalars):
//   1. msm_digits: key = (window << 16) | digit per (point, window), digit 0 skipped
//   2. radix sort of (key, point index) pairs (msm_sort.hpp) -> points grouped by bucket
//   3. msm_bucket_bounds: [start, end) of every bucket in the sorted order
//   4. msm_chunk_acc: the sorted list cut into fixed chunks of MSM_CH entries, one thread
//      per chunk accumulating its runs of equal keys in XYZZ (every thread does the same
//      number of additions whatever the bucket sizes); runs that cross a chunk boundary
//      leave partial sums, which a tree join adds up (msm_join_step / msm_join_rest)
//   5. bucket reduction sum_b (b + 1) B_b per window as short parallel trees
//      (msm_fx_cd / msm_fx_subsets / msm_fx_total, see there)
//   6. host: Horner over the 16 window sums (2^16 steps), one inversion to affine.
// The result is a group element, so the canonical affine output is unique.
#include <cstring>
#include <vector>
#include "../../include/pbf.h"
#include "msm.hpp"
#include "msm_l29.hpp"
#include "msm_sort.hpp"

namespace pbf {

constexpr int MSM_C = 16;
constexpr int MSM_NW = 16;
// signed digits in [-2^15, 2^15]: bucket j of a window holds the points whose digit has
// |d| = j + 1 (negated for d < 0), so a window has 2^15 buckets
constexpr int MSM_BB = MSM_C - 1;                            // bucket-index bits
constexpr uint32_t MSM_NB = 1u << MSM_BB;                    // buckets per window
constexpr uint32_t MSM_SENTINEL = (uint32_t)MSM_NW << MSM_BB;  // sorts after every real key
constexpr uint32_t MSM_NEG = 0x80000000u;                    // sign flag in the point index

__device__ __forceinline__ U256 load_u256(const uint64_t* p) {
  U256 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) { r.w[2 * i] = (uint32_t)p[i]; r.w[2 * i + 1] = (uint32_t)(p[i] >> 32); }
  return r;
}
__device__ __forceinline__ void store_u256(uint64_t* p, const U256& v) {
#pragma unroll
  for (int i = 0; i < 4; ++i) p[i] = (uint64_t)v.w[2 * i] | ((uint64_t)v.w[2 * i + 1] << 32);
}

// canonical affine (8 x u64 per point) -> Montgomery Affine; identity flagged in `inf`
__global__ void msm_points_to_mont(const uint64_t* pts, Affine* out, uint8_t* inf, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const U256 x = load_u256(pts + 8 * i), y = load_u256(pts + 8 * i + 4);
    inf[i] = (Fq::is_zero(x) && Fq::is_zero(y)) ? 1 : 0;
    Affine a;
    a.x = Fq::to_mont(x);
    a.y = Fq::to_mont(y);
    out[i] = a;
  }
}

// 16-bit windows recoded to signed digits (d >= 2^15 -> d - 2^16, carry 1 upward); the
// top window of a < 2^254 scalar stays below 2^14 + 1, so 16 windows hold every carry
__global__ void msm_digits(const uint64_t* scalars, const uint8_t* inf, uint32_t* keys, uint32_t* vals, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = scalars + 4 * i;
    const bool skip = inf[i] != 0;
    uint32_t carry = 0;
#pragma unroll
    for (int w = 0; w < MSM_NW; ++w) {
      uint32_t d = (uint32_t)((s[w / 4] >> (16 * (w % 4))) & 0xFFFF) + carry;
      bool neg = false;
      if (d > MSM_NB) {  // d - 2^16 < 0
        d = (1u << MSM_C) - d;
        neg = true;
        carry = 1;
      } else {
        carry = 0;
      }
      keys[(uint64_t)w * n + i] = (d == 0 || skip) ? MSM_SENTINEL : (((uint32_t)w << MSM_BB) | (d - 1));
      vals[(uint64_t)w * n + i] = (uint32_t)i | (neg ? MSM_NEG : 0u);
    }
  }
}

// the same digits as 16-bit codes (msm_sort.hpp RS_DIG_*; the window is the entry's row)
__global__ void msm_digits16(const uint64_t* scalars, const uint8_t* inf, uint16_t* dig, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = scalars + 4 * i;
    const bool skip = inf[i] != 0;
    uint32_t carry = 0;
#pragma unroll
    for (int w = 0; w < MSM_NW; ++w) {
      uint32_t d = (uint32_t)((s[w / 4] >> (16 * (w % 4))) & 0xFFFF) + carry;
      bool neg = false;
      if (d > MSM_NB) {
        d = (1u << MSM_C) - d;
        neg = true;
        carry = 1;
      } else {
        carry = 0;
      }
      dig[(uint64_t)w * n + i] = (d == 0 || skip) ? RS_DIG_NONE : (uint16_t)((d - 1) | (neg ? 0x8000u : 0u));
    }
  }
}

__global__ void msm_bucket_bounds(const uint32_t* keys, uint64_t m, uint32_t* start, uint32_t* end, uint32_t sent) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = keys[j];
    if (k == sent) continue;
    if (j == 0 || keys[j - 1] != k) start[k] = (uint32_t)j;
    if (j == m - 1 || keys[j + 1] != k) end[k] = (uint32_t)(j + 1);
  }
}
// The same bounds, four sorted keys per thread from one 16-B load and no grid-stride loop: the
// loop above kept one load in flight per wave and iteration (~48 dependent iterations per
// thread at 2^28 entries: latency-bound, ~1.3 TB/s).
__global__ void __launch_bounds__(256) msm_bucket_bounds4(const uint32_t* keys, uint64_t m, uint32_t* start,
                                                          uint32_t* end, uint32_t sent) {
  const uint64_t j0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (j0 >= m) return;
  uint32_t k[6];
  if (j0 + 4 <= m) {
    const uint4 v = *(const uint4*)(keys + j0);
    k[1] = v.x; k[2] = v.y; k[3] = v.z; k[4] = v.w;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) k[1 + i] = j0 + i < m ? keys[j0 + i] : sent;
  }
  k[0] = j0 ? keys[j0 - 1] : sent;
  k[5] = j0 + 4 < m ? keys[j0 + 4] : sent;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint64_t j = j0 + i;
    const uint32_t kk = k[1 + i];
    if (j >= m || kk == sent) continue;
    if (j == 0 || k[i] != kk) start[kk] = (uint32_t)j;
    if (j == m - 1 || k[i + 2] != kk) end[kk] = (uint32_t)(j + 1);
  }
}
static void launch_bucket_bounds(const uint32_t* keys, uint64_t m, uint32_t* start, uint32_t* end, uint32_t sent,
                                 hipStream_t s) {
  if (env_default_off("PBF_MSM_BOUNDS1"))  // read per call: an A/B knob (the grid-stride form)
    hipLaunchKernelGGL(msm_bucket_bounds, dim3((uint32_t)(((m + 255) / 256) > 16384 ? 16384 : (m + 255) / 256)),
                       dim3(256), 0, s, keys, m, start, end, sent);
  else
    hipLaunchKernelGGL(msm_bucket_bounds4, dim3((uint32_t)((m + 1023) / 1024)), dim3(256), 0, s, keys, m, start, end,
                       sent);
}

#ifndef PBF_MSM_CH
#define PBF_MSM_CH 43
#endif
#ifndef PBF_MSM_ACC_WPE
#define PBF_MSM_ACC_WPE 3
#endif
constexpr uint32_t MSM_CH = PBF_MSM_CH;  // sorted entries per accumulation thread

struct ChunkPart {
  union {
    Xyzz acc;
    uint32_t raw[36];  // msm_chunk_acc_l29r's unconverted accumulator (msm_l29_finish converts it)
  };
  uint32_t key;  // the sentinel key: no partial
  uint32_t pad[3];
};

// Chunk t = entries [t*CH, (t+1)*CH) of the sorted list (m valid entries). Complete runs
// (the whole bucket inside the chunk) are written to their bucket. head[t]: the first run
// if its bucket started in an earlier chunk; tail[t]: the last run if its bucket starts in
// this chunk and ends in a later one. Buckets with no entry stay zero (ZZ = 0: identity).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PBF_MSM_ACC_WPE))) msm_chunk_acc(const Affine* pts, const uint32_t* keys, const uint32_t* vals,
                                                     const uint32_t* start, const uint32_t* end, uint32_t m,
                                                     Xyzz* buckets, ChunkPart* head, ChunkPart* tail, uint32_t sent,
                                                     const uint32_t* m_dev, uint32_t* hkey, uint32_t* tkey) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c0 = t * MSM_CH;
  if (c0 >= m) return;  // past the chunks of the m-entry list
  head[t].key = sent;
  tail[t].key = sent;
  hkey[t] = sent;
  tkey[t] = sent;
  // m_dev: the valid length, known on the device only (counting sort: no sentinel entries)
  const uint32_t mv = m_dev ? *m_dev : m;
  if (c0 >= mv) return;
  const uint32_t c1 = c0 + MSM_CH < mv ? c0 + MSM_CH : mv;
  uint32_t cur = keys[c0], rs = c0;
  Xyzz acc = G1::identity();
  if (cur == sent) return;  // past the valid prefix (zero digits sort last)
  auto flush = [&](uint32_t re) {
    const uint32_t bs = start[cur], be = end[cur];
    if (bs < rs) {  // continues a bucket of an earlier chunk (possibly spanning this one)
      head[t].acc = acc;
      head[t].key = cur;
      hkey[t] = cur;
    } else if (be > re) {  // starts here, ends in a later chunk
      tail[t].acc = acc;
      tail[t].key = cur;
      tkey[t] = cur;
    } else {
      buckets[cur] = acc;
    }
  };
  // the next entry's point and the entry after it's key and index are loaded while the
  // current addition runs (the point gathers are random: their latency would otherwise stall
  // every step, and a point's address is known only once its index has arrived)
  uint32_t k_nx = cur, v_nx = vals[c0];
  Affine p_nx = pts[v_nx & ~MSM_NEG];
  uint32_t k_n2 = 0, v_n2 = 0;
  if (c0 + 1 < c1) k_n2 = keys[c0 + 1], v_n2 = vals[c0 + 1];
  for (uint32_t j = c0; j < c1; ++j) {
    const uint32_t k = k_nx, v = v_nx;
    Affine p = p_nx;
    if (j + 1 < c1) {
      k_nx = k_n2;
      v_nx = v_n2;
      p_nx = pts[v_nx & ~MSM_NEG];  // a sentinel entry's index is still a valid point
      if (j + 2 < c1) k_n2 = keys[j + 2], v_n2 = vals[j + 2];
    }
    if (k != cur) {
      flush(j);
      if (k == sent) return;
      cur = k;
      rs = j;
      acc = G1::identity();
    }
    if (v & MSM_NEG) p.y = Fq::sub(u256_zero(), p.y);
#ifdef PBF_MSM_MUL2CH
    acc = G1::madd(acc, p);  // A/B build: the two-chain product
#else
    acc = G1::madd_tp(acc, p);
#endif
  }
  flush(c1);
}

// msm_chunk_acc with the accumulator in 29-bit limbs (msm_l29.hpp: no carry folds in the
// products, ~205 instead of 319 VALU each); same chunking, same flush targets, the bucket
// sums converted back to the 32-bit Montgomery form at the flush. Default; PBF_MSM_L29=0
// selects msm_chunk_acc (A/B).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PBF_MSM_ACC_WPE)))
msm_chunk_acc_l29(const Affine* pts, const uint32_t* keys, const uint32_t* vals, const uint32_t* start,
                  const uint32_t* end, uint32_t m, Xyzz* buckets, ChunkPart* head, ChunkPart* tail, uint32_t sent,
                  const uint32_t* m_dev, uint32_t* hkey, uint32_t* tkey) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c0 = t * MSM_CH;
  if (c0 >= m) return;
  head[t].key = sent;
  tail[t].key = sent;
  hkey[t] = sent;
  tkey[t] = sent;
  const uint32_t mv = m_dev ? *m_dev : m;
  if (c0 >= mv) return;
  const uint32_t c1 = c0 + MSM_CH < mv ? c0 + MSM_CH : mv;
  uint32_t cur = keys[c0], rs = c0;
  l29::Acc acc;
  acc.id = true;
  if (cur == sent) return;
  auto flush = [&](uint32_t re) {
    const uint32_t bs = start[cur], be = end[cur];
    const Xyzz v = l29::to_xyzz(acc);
    if (bs < rs) {
      head[t].acc = v;
      head[t].key = cur;
      hkey[t] = cur;
    } else if (be > re) {
      tail[t].acc = v;
      tail[t].key = cur;
      tkey[t] = cur;
    } else {
      buckets[cur] = v;
    }
  };
  uint32_t k_nx = cur, v_nx = vals[c0];
  Affine p_nx = pts[v_nx & ~MSM_NEG];
  uint32_t k_n2 = 0, v_n2 = 0;
  if (c0 + 1 < c1) k_n2 = keys[c0 + 1], v_n2 = vals[c0 + 1];
  for (uint32_t j = c0; j < c1; ++j) {
    const uint32_t k = k_nx, v = v_nx;
    Affine p = p_nx;
    if (j + 1 < c1) {
      k_nx = k_n2;
      v_nx = v_n2;
      p_nx = pts[v_nx & ~MSM_NEG];
      if (j + 2 < c1) k_n2 = keys[j + 2], v_n2 = vals[j + 2];
    }
    if (k != cur) {
      flush(j);
      if (k == sent) return;
      cur = k;
      rs = j;
      acc.id = true;
    }
    if (v & MSM_NEG) p.y = Fq::sub(u256_zero(), p.y);
    if (l29::madd(acc, l29::from_u256(p.x), l29::from_u256(p.y))) {
      // P + P (rare): the doubled point, from the point reloaded
      Affine q = pts[v & ~MSM_NEG];
      if (v & MSM_NEG) q.y = Fq::sub(u256_zero(), q.y);
      acc = l29::from_xyzz(G1::mdbl(q));
    }
  }
  flush(c1);
}
// msm_chunk_acc_l29 with the flush deferred (round 4, default; PBF_MSM_RAWFLUSH=0 selects the
// kernel above): a flush stores the raw 29-bit-limb accumulator (l29::store_raw, 144 B, no
// products) -- into braw[key] for a run complete in this chunk, head[t].raw / tail[t].raw for
// a partial -- and msm_l29_finish converts them afterwards. Lanes of a wave reach their run
// boundaries at different entries; with the conversion (4 products) inside the loop, a wave
// executed it at every entry where any lane flushed: with ~100 entries per bucket (wide
// fixed-base windows, the windowed form) that is most entries. hkey[t] / tkey[t]: the key of
// chunk t's head / tail partial (the sentinel: none), compact for the join and the finish.
#ifndef PBF_MSM_ACC_WPE_R
#define PBF_MSM_ACC_WPE_R 3
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PBF_MSM_ACC_WPE_R)))
msm_chunk_acc_l29r(const Affine* pts, const uint32_t* keys, const uint32_t* vals, const uint32_t* start,
                   const uint32_t* end, uint32_t m, uint32_t* braw, ChunkPart* head, ChunkPart* tail, uint32_t sent,
                   const uint32_t* m_dev, uint32_t* hkey, uint32_t* tkey) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c0 = t * MSM_CH;
  if (c0 >= m) return;
  hkey[t] = sent;
  tkey[t] = sent;
  const uint32_t mv = m_dev ? *m_dev : m;
  if (c0 >= mv) return;
  const uint32_t c1 = c0 + MSM_CH < mv ? c0 + MSM_CH : mv;
  uint32_t cur = keys[c0], rs = c0;
  l29::Acc acc;
  acc.id = true;
  if (cur == sent) return;
  auto flush = [&](uint32_t re) {
    const uint32_t bs = start[cur], be = end[cur];
    uint32_t* dst;
    if (bs < rs) {
      dst = head[t].raw;
      hkey[t] = cur;
    } else if (be > re) {
      dst = tail[t].raw;
      tkey[t] = cur;
    } else {
      dst = braw + 36ull * cur;
    }
    l29::store_raw(acc, dst);
  };
  uint32_t k_nx = cur, v_nx = vals[c0];
  Affine p_nx = pts[v_nx & ~MSM_NEG];
  uint32_t k_n2 = 0, v_n2 = 0;
  if (c0 + 1 < c1) k_n2 = keys[c0 + 1], v_n2 = vals[c0 + 1];
  for (uint32_t j = c0; j < c1; ++j) {
    const uint32_t k = k_nx, v = v_nx;
    Affine p = p_nx;
    if (j + 1 < c1) {
      k_nx = k_n2;
      v_nx = v_n2;
      p_nx = pts[v_nx & ~MSM_NEG];
      if (j + 2 < c1) k_n2 = keys[j + 2], v_n2 = vals[j + 2];
    }
    if (k != cur) {
      flush(j);
      if (k == sent) return;
      cur = k;
      rs = j;
      acc.id = true;
    }
    if (v & MSM_NEG) p.y = Fq::sub(u256_zero(), p.y);
    if (l29::madd(acc, l29::from_u256(p.x), l29::from_u256(p.y))) {
      Affine q = pts[v & ~MSM_NEG];
      if (v & MSM_NEG) q.y = Fq::sub(u256_zero(), q.y);
      acc = l29::from_xyzz(G1::mdbl(q));
    }
  }
  flush(c1);
}
// The conversions msm_chunk_acc_l29r deferred, one per stored sum, every lane busy: buckets
// complete inside one chunk (start and end in the same chunk: the ones fx_bucket reads from
// `buckets`), then every head and tail partial with a key, converted in place.
__global__ void __launch_bounds__(256) msm_l29_finish(const uint32_t* braw, Xyzz* buckets, ChunkPart* head,
                                                      ChunkPart* tail, const uint32_t* hkey, const uint32_t* tkey,
                                                      const uint32_t* start, const uint32_t* end, uint32_t nb,
                                                      uint32_t nchunks, uint32_t sent, uint32_t hmax) {
  // hmax > 0 (the fixed-base wide-window tail): only the partials of buckets spanning more than
  // hmax chunks are converted here; msm_join_heavy and msm_fx_resolve convert the others as they
  // read them (one read of the raw form instead of a converted write and its read)
  auto keep = [&](uint32_t k) { return k != sent && (hmax == 0 || (end[k] - 1) / MSM_CH - start[k] / MSM_CH > hmax); };
  const uint64_t items = (uint64_t)nb + 2ull * nchunks;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < items; i += (uint64_t)gridDim.x * blockDim.x) {
    if (i < nb) {
      const uint32_t bs = start[i], be = end[i];
      if (be > bs && bs / MSM_CH == (be - 1) / MSM_CH) buckets[i] = l29::raw_to_xyzz(braw + 36 * i);
    } else if (i < (uint64_t)nb + nchunks) {
      const uint64_t t = i - nb;
      if (keep(hkey[t])) head[t].acc = l29::raw_to_xyzz(head[t].raw);
    } else {
      const uint64_t t = i - nb - nchunks;
      if (keep(tkey[t])) tail[t].acc = l29::raw_to_xyzz(tail[t].raw);
    }
  }
}
static bool msm_l29() {
  return env_default_on("PBF_MSM_L29");  // read per call: an A/B knob
}
// deferred flush conversion: the default where runs are short (the windowed form, fixed-base
// windows wider than 16 bits: ~30-200 entries per bucket); the c = 16 fixed-base form (~500+
// per bucket) flushes rarely, and the separate conversion pass costs it more than it saves
// (2^24 points: 32.5 against 32.0 ms). PBF_MSM_RAWFLUSH=0/1 forces either (A/B).
static bool msm_rawflush(bool short_runs = true) {
  const char* e = ab_env("PBF_MSM_RAWFLUSH");  // an A/B knob (PBF_AB build only)
  if (e && *e) return atoi(e) != 0;
  return short_runs;
}

// ---------------------------------------------------------------- fixed-base MSM
// KZG commitments are MSMs against the fixed SRS (plonk.rs:51-58), so the SRS points can be
// precomputed once per window: table[w][i] = 2^(FX_C w) P_i (affine, Montgomery). Every
// (point, window) digit then goes to ONE set of buckets (bucket |d| - 1 of entry
// table[w][i], negated for d < 0): one bucket reduction instead of one per window, no
// Horner over windows, no per-call conversion of the points. The window stays at 16-bit
// signed digits (16 windows, 2^15 buckets, the table 16 x n x 64 B = 1 GiB per 2^20
// points). Measured alternatives (2^20-gate proof): 20-bit digits (13 windows: 13 n
// instead of 16 n mixed additions, 2^19 buckets) 50.8 ms against 48.1 -- the accumulation
// did not shrink in proportion and the 2^19-bucket reduction (0.84 ms segments, 0.40 ms
// trees) steals the VALUs; a counting sort by global atomics instead of the radix sort
// 58.3 ms -- count 0.52 + scatter 0.91 ms per MSM: device-scope atomics on MI355X resolve
// beyond the per-XCD L2s (~26 G/s).
constexpr int FX_C = 16, FX_NW = 16;
constexpr uint32_t FX_NB = 1u << (FX_C - 1);  // buckets (|d| - 1, |d| <= 2^(FX_C-1))
static_assert(FX_C * FX_NW >= 255, "windows must cover a 254-bit scalar plus the recoding carry");
// Round 4: the window width of a table is chosen by its size (FxGeom, fx_geom). c-bit signed
// digits need ceil(255 / c) windows (a 254-bit scalar plus the recoding carry) and 2^(c-1)
// buckets, so the accumulation performs ceil(255 / c) n mixed additions: 16 n at c = 16,
// 13 n at c = 20, 12 n at c = 22. The wider windows pay for it with a third sort pass, more
// buckets to reduce (2^(c-1)) and fewer entries per bucket (more flushes), which a large table
// amortises and a small one does not.
struct FxGeom {
  int c = FX_C, nw = FX_NW;  // window bits, windows
  uint32_t nb = FX_NB;       // buckets, 2^(c-1)
  int lb = 8, hb = 7;        // bucket b = 2^lb h + l (l < 2^lb, h < 2^hb), lb + hb = c - 1
};
static FxGeom fx_geom_of(int c) {
  FxGeom g;
  g.c = c;
  g.nw = (255 + c - 1) / c;
  g.nb = 1u << (c - 1);
  g.lb = c / 2;
  g.hb = c - 1 - g.lb;
  return g;
}
// default window width of a table of n points; option msm.fx_c = 16/18/20/22 forces one (read at
// the table build: the tests build the wide tables of large sizes at small ones). Measured (profiles/r04/msm_window_*): a 2^20-point MSM is fastest at c = 16
// (2.27 ms; c = 20: 2.69), 2^22 points at c = 20 (7.60 against 7.71 ms; in the 2^22-gate proof
// 87.6 against 92.0 ms), 2^24 points at c = 22 (27.2 against 29.0 ms; the 2^24-gate proof 327
// against 350 ms). Boundaries at the geometric midpoints.
static int fx_default_c(const pbf_ctx* ctx, uint64_t n) {
  {
    const int v = (int)ctx->options.num("msm.fx_c", 0);
    if (v == 16 || v == 18 || v == 20 || v == 22) return v;
  }
  if (n >= 3ull << 22) return 22;
  if (n >= 3ull << 20) return 20;
  return 16;
}

// table window w from window w-1: FX_C doublings in XYZZ, then affine through a
// block-wide batch inversion of the ZZZ (prefix and suffix products in LDS, one Fermat
// inversion per block); the identity (0, 0) stays (0, 0)
__global__ void __launch_bounds__(256) msm_table_window(const Affine* prev, Affine* next, uint64_t n, int c) {
  __shared__ U256 pre[256], suf[256];
  __shared__ U256 tinv;
  const uint32_t t = threadIdx.x;
  const uint64_t i = (uint64_t)blockIdx.x * 256 + t;
  const U256 one = G1::one_m();
  bool id = true;
  Xyzz acc = G1::identity();
  if (i < n) {
    const Affine a = prev[i];
    id = Fq::is_zero(a.x) && Fq::is_zero(a.y);
    if (!id) {
      acc = G1::mdbl(a);
      for (int k = 1; k < c; ++k) acc = G1::dbl(acc);
    }
  }
  const U256 z = id ? one : acc.ZZZ;
  pre[t] = z;
  suf[t] = z;
  __syncthreads();
  for (uint32_t off = 1; off < 256; off <<= 1) {  // inclusive prefix / suffix products
    U256 p = pre[t], q = suf[t];
    if (t >= off) p = Fq::mul(pre[t - off], p);
    if (t + off < 256) q = Fq::mul(q, suf[t + off]);
    __syncthreads();
    pre[t] = p;
    suf[t] = q;
    __syncthreads();
  }
  if (t == 0) tinv = G1::inv(pre[255]);
  __syncthreads();
  if (i >= n) return;
  Affine r;
  if (id) {
    r.x = u256_zero();
    r.y = u256_zero();
  } else {
    U256 izzz = tinv;  // 1 / ZZZ_t = tinv * prod_{u<t} * prod_{u>t}
    if (t > 0) izzz = Fq::mul(izzz, pre[t - 1]);
    if (t < 255) izzz = Fq::mul(izzz, suf[t + 1]);
    const U256 q = Fq::mul(acc.ZZ, izzz);
    const U256 izz = Fq::mul(q, q);
    r.x = Fq::mul(acc.X, izz);
    r.y = Fq::mul(acc.Y, izzz);
  }
  next[i] = r;
}

// window w's signed digit of a scalar (FX_C bits; d > 2^(FX_C-1) -> d - 2^FX_C, carry 1 upward):
// calls in window order carry through `carry`. Returns |d| (0: no entry), sets neg.
__device__ __forceinline__ uint32_t fx_digit(const uint64_t* s, int w, int c, uint32_t& carry, bool& neg) {
  const int bit = c * w, limb = bit >> 6, off = bit & 63;
  uint64_t v = limb < 4 ? s[limb] >> off : 0;
  if (off + c > 64 && limb + 1 < 4) v |= s[limb + 1] << (64 - off);
  uint32_t d = (uint32_t)(v & ((1u << c) - 1)) + carry;
  neg = false;
  if (d > (1u << (c - 1))) {
    d = (1u << c) - d;
    neg = true;
    carry = 1;
  } else {
    carry = 0;
  }
  return d;
}

// one (key, value) per (point, window): key = |d| - 1 (FX_NB: zero digit or identity
// point, sorts last), value = index of table[w][first + i] | sign
__global__ void __launch_bounds__(256) msm_fx_digits(const uint64_t* scalars, const uint8_t* inf, uint64_t n_table,
                                                     uint64_t first, uint64_t n, uint32_t* keys, uint32_t* vals,
                                                     int c, int nw) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = scalars + 4 * i;
    const bool skip = inf[first + i] != 0;
    uint32_t carry = 0;
    for (int w = 0; w < nw; ++w) {
      bool neg;
      const uint32_t d = fx_digit(s, w, c, carry, neg);
      keys[(uint64_t)w * n + i] = (d == 0 || skip) ? (1u << (c - 1)) : d - 1;
      vals[(uint64_t)w * n + i] = (uint32_t)((uint64_t)w * n_table + first + i) | (neg ? MSM_NEG : 0u);
    }
  }
}

// The same digits as msm_fx_digits as planar codes (msm_sort.hpp RsDigitsT: 16-bit for c <= 16,
// 32-bit above): the first sort pass derives key and value from the code and the entry index
template <typename C, int C_FIX = 0>
__global__ void __launch_bounds__(256) msm_fx_digits_code(const uint64_t* scalars, const uint8_t* inf, uint64_t first,
                                                          uint64_t n, C* dig, int c_rt, int nw_rt) {
  const int c = C_FIX ? C_FIX : c_rt, nw = C_FIX ? (255 + C_FIX - 1) / C_FIX : nw_rt;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = scalars + 4 * i;
    const bool skip = inf[first + i] != 0;
    uint32_t carry = 0;
#pragma unroll
    for (int w = 0; w < (C_FIX ? (255 + C_FIX - 1) / C_FIX : 16); ++w) {
      if (!C_FIX && w >= nw) break;
      bool neg;
      const uint32_t d = fx_digit(s, w, c, carry, neg);
      dig[(uint64_t)w * n + i] = (d == 0 || skip) ? (C)rs_none<C>() : (C)((d - 1) | (neg ? rs_sign<C>() : 0u));
    }
  }
}
static_assert(FX_NB - 1 <= 0x7FFF, "a 16-bit digit code holds |d| - 1 in 15 bits");

// Boundary join (fixed-base form: ~16 n / 2^15 entries per bucket, 512 at 2^20 points, so a
// bucket crossing chunks spans ~12 of them; windowed form: ~2 chunks). Tree over each bucket's
// continuation partials head[o+1 .. e] (o = chunk of the bucket's first entry, e = chunk of
// its last): at step s, the continuation at o + 1 + 2 s j adds head[o + 1 + 2 s j + s] when
// that is <= e. After ceil(log2(span)) steps head[o+1] holds their sum; fx_bucket adds it
// to the owner's tail partial. One work item per (bucket, j) -- not per chunk, so the
// waves of a step hold only adding lanes (a per-chunk grid kept every wave busy at every
// step for a shrinking share of active lanes).
// the largest number of chunks a bucket spans (bounds the tree steps that do any work)
constexpr uint32_t MSM_SPAN_PER = 8;  // buckets per thread of msm_max_span
__global__ void __launch_bounds__(256) msm_max_span(const uint32_t* start, const uint32_t* end, uint32_t nb,
                                                    uint32_t* span) {
  // MSM_SPAN_PER buckets per thread, a wave max, one LDS atomic per wave and one global atomic per
  // workgroup (one bucket per thread and one global atomic per 256 buckets: ~97 us at 2^21 buckets,
  // the atomics on one address serialised)
  __shared__ uint32_t bmax;
  if (threadIdx.x == 0) bmax = 0;
  __syncthreads();
  uint32_t mx = 0;
#pragma unroll
  for (uint32_t i = 0; i < MSM_SPAN_PER; ++i) {
    const uint32_t k = blockIdx.x * (256 * MSM_SPAN_PER) + i * 256 + threadIdx.x;
    if (k < nb) {
      const uint32_t bs = start[k], be = end[k];
      if (be > bs) mx = max(mx, (be - 1) / MSM_CH - bs / MSM_CH);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
  if ((threadIdx.x & 63) == 0 && mx) atomicMax(&bmax, mx);
  __syncthreads();
  if (threadIdx.x == 0 && bmax) atomicMax(span, bmax);
}
static uint32_t max_span_groups(uint32_t nb) { return (nb + 256 * MSM_SPAN_PER - 1) / (256 * MSM_SPAN_PER); }
// cap: buckets spanning more than `cap` chunks are left to msm_join_chunks (the fixed-base form;
// ~0u: none), so the pair slots per bucket follow min(largest span, cap), not the largest span
__global__ void __launch_bounds__(256) msm_join_step(ChunkPart* head, const uint32_t* start, const uint32_t* end,
                                                     uint32_t nb, uint32_t step, const uint32_t* span,
                                                     uint32_t cap) {
  const uint32_t sp0 = *span, sp = sp0 < cap ? sp0 : cap;
  if (step >= sp) return;  // every bucket's continuations already summed
  const uint32_t per = (sp + 2 * step - 1) / (2 * step);  // pair slots per bucket
  const uint64_t items = (uint64_t)nb * per;
  for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < items;
       id += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = (uint32_t)(id / per), j = (uint32_t)(id % per);
    const uint32_t bs = start[k], be = end[k];
    if (be <= bs) continue;
    const uint32_t o = bs / MSM_CH, e = (be - 1) / MSM_CH;
    if (e - o > cap) continue;  // a heavy bucket: msm_join_chunks
    const uint32_t u = o + 1 + 2 * step * j;
    if (u + step <= e) head[u].acc = G1::add2(head[u].acc, head[u + step].acc);
  }
}
// bucket bounds and the span counter of a fixed-base MSM, zeroed in one launch
__global__ void __launch_bounds__(256) msm_fx_clear(uint32_t* start, uint32_t* end, uint32_t* span) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  start[k] = 0;
  end[k] = 0;
  if (k == 0) *span = 0;
}

// Join steps past FX_JOIN_GROUP / 2 are not launched (a bucket of the random-digit case
// spans ~16 chunks); this kernel finishes the rare buckets spanning more than FX_JOIN_GROUP
// continuation chunks (skewed digits): after the steps 1 .. FX_JOIN_GROUP / 2,
// head[o + 1 + G j] holds the sum of group j, so head[o + 1] += sum_{j >= 1} head[o + 1 + G j].
constexpr uint32_t FX_JOIN_GROUP = 32;
__global__ void __launch_bounds__(256) msm_join_rest(ChunkPart* head, const uint32_t* start, const uint32_t* end,
                                                     uint32_t nb, const uint32_t* span) {
  if (*span <= FX_JOIN_GROUP) return;
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nb || end[k] <= start[k]) return;
  const uint32_t o = start[k] / MSM_CH, e = (end[k] - 1) / MSM_CH;
  if (e - o <= FX_JOIN_GROUP) return;
  Xyzz acc = head[o + 1].acc;
  for (uint32_t u = o + 1 + FX_JOIN_GROUP; u <= e; u += FX_JOIN_GROUP) acc = G1::add2(acc, head[u].acc);
  head[o + 1].acc = acc;
}

// The same tree for the heavy buckets (spanning more than `cap` chunks; round 4, the fixed-base
// form), indexed by continuation chunk: work item u < nchunks is chunk u's head partial (hkey[u]:
// its bucket, or the sentinel), so a step costs O(chunks) however few buckets are heavy. Without
// it the per-bucket grid gives every bucket the pair slots of the LARGEST span: a narrow top
// window puts all n of its entries into few buckets (c = 18: 2 bits, 4 buckets; c = 22: 12
// bits), and the steps took up to ~8 ms each. Exits at once when no bucket is heavy.
__global__ void __launch_bounds__(256) msm_join_chunks(ChunkPart* head, const uint32_t* hkey, const uint32_t* start,
                                                       const uint32_t* end, uint32_t nchunks, uint32_t step,
                                                       const uint32_t* span, uint32_t sent, uint32_t cap) {
  const uint32_t sp = *span;
  if (step >= sp || sp <= cap) return;
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < nchunks; u += gridDim.x * blockDim.x) {
    const uint32_t k = hkey[u];
    if (k == sent) continue;
    const uint32_t o = start[k] / MSM_CH, e = (end[k] - 1) / MSM_CH, rel = u - (o + 1);
    if (e - o > cap && rel % (2 * step) == 0 && u + step <= e) head[u].acc = G1::add2(head[u].acc, head[u + step].acc);
  }
}
// msm_join_rest for a group size `group` (the steps launched: 1 .. group / 2)
__global__ void __launch_bounds__(256) msm_join_rest_g(ChunkPart* head, const uint32_t* start, const uint32_t* end,
                                                       uint32_t nb, const uint32_t* span, uint32_t group) {
  if (*span <= group) return;
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nb || end[k] <= start[k]) return;
  const uint32_t o = start[k] / MSM_CH, e = (end[k] - 1) / MSM_CH;
  if (e - o <= group) return;
  Xyzz acc = head[o + 1].acc;
  for (uint32_t u = o + 1 + group; u <= e; u += group) acc = G1::add2(acc, head[u].acc);
  head[o + 1].acc = acc;
}

// Round 5, the wide-window join in two launches instead of ~13 tree steps that each scanned every
// chunk: msm_heavy_list lists the buckets spanning more than `cap` chunks (one atomic per wave),
// msm_join_heavy sums each one's continuations with HJ_LPB lanes (a strided sequence per lane,
// then a shuffle tree inside the lane group) into head[o + 1], as the tree steps did.
// Buckets spanning more than HJ_MAX chunks (skewed scalars: ~6100 at 2^18 equal scalars) are
// left to the tree steps, which the lane groups' sequences would take too long for.
constexpr uint32_t HJ_LPB = 16;    // lanes per heavy bucket (divides 64)
constexpr uint32_t HJ_MAX = 1024;  // at most 64 continuations per lane
__global__ void __launch_bounds__(256) msm_heavy_list(const uint32_t* start, const uint32_t* end, uint32_t nb,
                                                      uint32_t cap, uint32_t hmax, uint32_t* list, uint32_t* count) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  bool h = false;
  if (k < nb) {
    const uint32_t bs = start[k], be = end[k];
    const uint32_t sp = be > bs ? (be - 1) / MSM_CH - bs / MSM_CH : 0;
    h = sp > cap && sp <= hmax;
  }
  const uint64_t mask = __ballot(h);
  if (!mask) return;  // wave-uniform
  const uint32_t lane = threadIdx.x & 63, lead = __ffsll((unsigned long long)mask) - 1;
  uint32_t base = 0;
  if (lane == lead) base = atomicAdd(count, (uint32_t)__popcll(mask));
  base = (uint32_t)__shfl((int)base, (int)lead);
  if (h) list[base + (uint32_t)__popcll(mask & ((1ull << lane) - 1))] = k;
}
__device__ __forceinline__ Xyzz xyzz_shfl_xor(const Xyzz& v, int off) {
  Xyzz r;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r.X.w[i] = (uint32_t)__shfl_xor((int)v.X.w[i], off);
    r.Y.w[i] = (uint32_t)__shfl_xor((int)v.Y.w[i], off);
    r.ZZ.w[i] = (uint32_t)__shfl_xor((int)v.ZZ.w[i], off);
    r.ZZZ.w[i] = (uint32_t)__shfl_xor((int)v.ZZZ.w[i], off);
  }
  return r;
}
// raw: the continuations are still in msm_chunk_acc_l29r's raw form (msm_l29_finish's hmax)
__global__ void __launch_bounds__(256) msm_join_heavy(ChunkPart* head, const uint32_t* list, const uint32_t* count,
                                                      const uint32_t* start, const uint32_t* end, uint32_t raw) {
  const uint32_t cnt = *count, sub = threadIdx.x % HJ_LPB, per_block = 256 / HJ_LPB;
  for (uint32_t b = blockIdx.x * per_block + threadIdx.x / HJ_LPB; b < cnt; b += gridDim.x * per_block) {
    // b is uniform over the lane group: the group's shuffles below see only its own lanes
    const uint32_t k = list[b];
    const uint32_t o = start[k] / MSM_CH, e = (end[k] - 1) / MSM_CH;
    Xyzz acc = G1::identity();
    for (uint32_t u = o + 1 + sub; u <= e; u += HJ_LPB)
      acc = G1::add2(acc, raw ? l29::raw_to_xyzz(head[u].raw) : head[u].acc);
    for (int off = HJ_LPB / 2; off > 0; off >>= 1) acc = G1::add2(acc, xyzz_shfl_xor(acc, off));
    if (sub == 0) head[o + 1].acc = acc;  // every lane of the group has read its parts by now
  }
}

// Bucket b's full sum after the join: a bucket spanning chunks o < e is its chunk-o tail run
// plus the joined continuations head[o + 1]; any other bucket was written whole (or is
// empty: never read).
__device__ __forceinline__ Xyzz fx_bucket(uint32_t k, const Xyzz* buckets, const ChunkPart* head,
                                          const ChunkPart* tail, const uint32_t* start, const uint32_t* end) {
  const uint32_t bs = start[k], be = end[k];
  if (be <= bs) return G1::identity();
  const uint32_t o = bs / MSM_CH, e = (be - 1) / MSM_CH;
  return o < e ? G1::add2(tail[o].acc, head[o + 1].acc) : buckets[k];
}

// Workgroup tree sum of one value per thread (blockDim.x a power of two <= 256) -> *out.
__device__ __forceinline__ void fx_tree(Xyzz v, Xyzz* out) {
  __shared__ Xyzz red[256];
  const uint32_t t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (uint32_t st = blockDim.x / 2; st > 0; st >>= 1) {
    if (t < st) red[t] = G1::add2(red[t], red[t + st]);
    __syncthreads();
  }
  if (t == 0) *out = red[0];
}

// Fixed-base bucket reduction T = sum_{b < 2^15} (b + 1) B_b as short parallel trees instead
// of running sums (the tail is a latency chain: its depth in point additions is its time).
// With b = 256 h + l (h < 128, l < 256), C_h = sum_l B_(256h+l), D_l = sum_h B_(256h+l):
//   T = sum_{k<7} 2^(k+8) Z_k + sum_{k<8} 2^k Y_k + S,
//   Z_k = sum_{h: bit k of h} C_h,  Y_k = sum_{l: bit k of l} D_l,  S = sum_h C_h
// (sum_b b B_b = 256 sum_h h C_h + sum_l l D_l; sum_b B_b = S). Depth: 9 additions (C/D
// trees), 7 (subset trees), <= 14 doublings, 4 (final sum) -- against ~60 for the
// segment running sums and their tree.
constexpr uint32_t FX_NH = FX_NB / 256;  // 128 values of h
static_assert(FX_NH == 128, "2^15 buckets = 128 x 256");
// workgroup (g, w): window w's buckets start at w * 2^15 (keys (w << 15) | b); g < 128: C_g
// (256 buckets), g >= 128: D_(g-128) (128 buckets); cd holds 384 sums per window
__global__ void __launch_bounds__(256) msm_fx_cd(const Xyzz* buckets, const ChunkPart* head, const ChunkPart* tail,
                                                 const uint32_t* start, const uint32_t* end, Xyzz* cd) {
  const uint32_t g = blockIdx.x, t = threadIdx.x, base = blockIdx.y * FX_NB;
  Xyzz v;
  if (g < FX_NH)
    v = fx_bucket(base + 256 * g + t, buckets, head, tail, start, end);
  else
    v = t < FX_NH ? fx_bucket(base + 256 * t + (g - FX_NH), buckets, head, tail, start, end) : G1::identity();
  fx_tree(v, cd + (uint64_t)blockIdx.y * (FX_NH + 256) + g);
}
// The same C_h / D_l sums for many windows at once (the windowed MSM: 16 x 384 trees), where
// throughput matters more than depth: a 256-tree keeps on average a quarter of its lanes
// busy, so each thread first adds SEQ buckets in sequence. Workgroup (g, w), g < 128 / SEQ:
// C_h for h = SEQ g .. SEQ g + SEQ - 1 (256 / SEQ threads per h, SEQ consecutive buckets
// each, then (256 / SEQ)-lane trees); the other 128 / SEQ workgroups: D_l for 2 SEQ values
// of l each (128 / SEQ threads per l, SEQ values of h each, then (128 / SEQ)-lane trees).
// SEQ trades depth (SEQ + log2(lanes) additions) against waves in flight (PBF_MSM_CD_SEQ).
// (Round 3: single-chain products in the sequential part measured no faster, 3.25-3.28 vs
// 3.25 ms per windowed MSM, profiles/r03/msm_addtp_ab.log: two to four waves per SIMD leave
// the interleaved products' latency hiding the better trade here.)
template <int SEQ>
__global__ void __launch_bounds__(256) msm_fx_cd_seq(const Xyzz* buckets, const ChunkPart* head, const ChunkPart* tail,
                                                     const uint32_t* start, const uint32_t* end, Xyzz* cd) {
  __shared__ Xyzz red[256];
  constexpr uint32_t CL = 256 / SEQ, DL = 128 / SEQ, CG = 128 / SEQ;  // lanes per C / D tree
  const uint32_t g = blockIdx.x, t = threadIdx.x, base = blockIdx.y * FX_NB;
  Xyzz* out = cd + (uint64_t)blockIdx.y * (FX_NH + 256);
  Xyzz acc = G1::identity();
  uint32_t lanes;
  if (g < CG) {
    const uint32_t h = SEQ * g + t / CL, l0 = (t % CL) * SEQ;
    for (uint32_t i = 0; i < SEQ; ++i) acc = G1::add2(acc, fx_bucket(base + 256 * h + l0 + i, buckets, head, tail, start, end));
    lanes = CL;
  } else {
    const uint32_t l = 2 * SEQ * (g - CG) + t / DL, h0 = (t % DL) * SEQ;
    for (uint32_t i = 0; i < SEQ; ++i) acc = G1::add2(acc, fx_bucket(base + 256 * (h0 + i) + l, buckets, head, tail, start, end));
    lanes = DL;
  }
  red[t] = acc;
  __syncthreads();
  for (uint32_t st = lanes / 2; st > 0; st >>= 1) {
    if (t % lanes < st) red[t] = G1::add2(red[t], red[t + st]);
    __syncthreads();
  }
  if (t % lanes == 0) out[g < CG ? SEQ * g + t / CL : FX_NH + 2 * SEQ * (g - CG) + t / DL] = red[t];
}
// workgroup (s, w) (128 threads): s < 8: 2^s Y_s; 8 <= s < 15: 2^s Z_(s-8); s = 15: S.
__global__ void __launch_bounds__(128) msm_fx_subsets(const Xyzz* cd, Xyzz* sub) {
  const uint32_t s = blockIdx.x, t = threadIdx.x;
  const Xyzz* C = cd + (uint64_t)blockIdx.y * (FX_NH + 256);
  const Xyzz* D = C + FX_NH;
  Xyzz v;
  if (s < 8) {  // the t-th l with bit s set
    v = D[((t >> s) << (s + 1)) | (1u << s) | (t & ((1u << s) - 1))];
  } else if (s < 15) {
    const uint32_t k = s - 8;
    v = t < 64 ? C[((t >> k) << (k + 1)) | (1u << k) | (t & ((1u << k) - 1))] : G1::identity();
  } else {
    v = C[t];
  }
  __shared__ Xyzz res;
  fx_tree(v, &res);
  if (t == 0) {
    Xyzz r = res;
    const uint32_t e = s < 15 ? s : 0;  // Y_s weight 2^s; Z_k weight 2^(k+8) = 2^s
    for (uint32_t i = 0; i < e; ++i) r = G1::dbl2(r);
    sub[blockIdx.y * 16 + s] = r;
  }
}
// workgroup w (16 threads): window w's sum of its 16 scaled subset sums
__global__ void __launch_bounds__(16) msm_fx_total(const Xyzz* sub, Xyzz* out) {
  fx_tree(sub[blockIdx.x * 16 + threadIdx.x], out + blockIdx.x);
}

// ---- the same reduction tail on quads (G1Quad: each point addition's product steps spread
// over the four lanes of a quad), the default: these kernels are latency chains of a few
// hundred waves, so a chain of quad additions (one product of latency per step) finishes
// about 3x sooner than one of single-lane additions (three or four interleaved products per
// step). PBF_MSM_QUAD=0 restores the single-lane kernels above (A/B).
__device__ __forceinline__ Xyzz fx_bucket_q(uint32_t k, const Xyzz* buckets, const ChunkPart* head,
                                            const ChunkPart* tail, const uint32_t* start, const uint32_t* end) {
  const uint32_t bs = start[k], be = end[k];
  if (be <= bs) return G1::identity();
  const uint32_t o = bs / MSM_CH, e = (be - 1) / MSM_CH;
  return o < e ? G1Quad::add(tail[o].acc, head[o + 1].acc) : buckets[k];
}
// Quad-tree sum of one value per quad (blockDim.x / 4 quads, a power of two); quad 0 returns
// the total (the other quads' return values are partial sums).
__device__ __forceinline__ Xyzz fx_tree_q(Xyzz v, Xyzz* red) {
  const uint32_t t = threadIdx.x, qi = t >> 2, nq = blockDim.x >> 2;
  if ((t & 3) == 0) red[qi] = v;
  __syncthreads();
  for (uint32_t st = nq / 2; st > 0; st >>= 1) {
    if (qi < st) v = G1Quad::add(v, red[qi + st]);
    __syncthreads();
    if (qi < st && (t & 3) == 0) red[qi] = v;
    __syncthreads();
  }
  return v;
}
// msm_fx_cd on quads: workgroup (g, w) of 256 threads (64 quads); g < 128: C_g, each quad
// first adds 4 consecutive buckets; g >= 128: D_(g-128), each quad 2 values of h.
__global__ void __launch_bounds__(256) msm_fx_cd_q(const Xyzz* buckets, const ChunkPart* head, const ChunkPart* tail,
                                                   const uint32_t* start, const uint32_t* end, Xyzz* cd) {
  __shared__ Xyzz red[64];
  const uint32_t g = blockIdx.x, qi = threadIdx.x >> 2, base = blockIdx.y * FX_NB;
  Xyzz v = G1::identity();
  if (g < FX_NH) {
    for (uint32_t i = 0; i < 4; ++i)
      v = G1Quad::add(v, fx_bucket_q(base + 256 * g + 4 * qi + i, buckets, head, tail, start, end));
  } else {
    for (uint32_t i = 0; i < 2; ++i)
      v = G1Quad::add(v, fx_bucket_q(base + 256 * (2 * qi + i) + (g - FX_NH), buckets, head, tail, start, end));
  }
  v = fx_tree_q(v, red);
  if (threadIdx.x == 0) cd[(uint64_t)blockIdx.y * (FX_NH + 256) + g] = v;
}
// msm_fx_subsets on quads: workgroup (s, w) of 512 threads (128 quads), quad i in the role of
// thread i there; quad 0 then applies the 2^s weight.
__global__ void __launch_bounds__(512) msm_fx_subsets_q(const Xyzz* cd, Xyzz* sub) {
  __shared__ Xyzz red[128];
  const uint32_t s = blockIdx.x, t = threadIdx.x >> 2;
  const Xyzz* C = cd + (uint64_t)blockIdx.y * (FX_NH + 256);
  const Xyzz* D = C + FX_NH;
  Xyzz v;
  if (s < 8) {
    v = D[((t >> s) << (s + 1)) | (1u << s) | (t & ((1u << s) - 1))];
  } else if (s < 15) {
    const uint32_t k = s - 8;
    v = t < 64 ? C[((t >> k) << (k + 1)) | (1u << k) | (t & ((1u << k) - 1))] : G1::identity();
  } else {
    v = C[t];
  }
  v = fx_tree_q(v, red);
  if (t == 0) {
    const uint32_t e = s < 15 ? s : 0;
    for (uint32_t i = 0; i < e; ++i) v = G1Quad::dbl(v);
    if (threadIdx.x == 0) sub[blockIdx.y * 16 + s] = v;
  }
}
// msm_fx_total on quads: workgroup w of 64 threads (16 quads)
__global__ void __launch_bounds__(64) msm_fx_total_q(const Xyzz* sub, Xyzz* out) {
  __shared__ Xyzz red[16];
  const Xyzz v = fx_tree_q(sub[blockIdx.x * 16 + (threadIdx.x >> 2)], red);
  if (threadIdx.x == 0) out[blockIdx.x] = v;
}
static bool msm_quad_tail() {
  return env_default_on("PBF_MSM_QUAD");  // read per call: an A/B knob
}
// the wide-window join: light buckets summed in sequence by the C / D sums, heavy ones by
// msm_join_chunks (default), or every bucket by the per-bucket steps (=0: A/B). The c = 16 form
// always takes the per-bucket steps: its spans are even (random scalars: a 14-bit top window),
// and the per-chunk steps would be a dozen idle launches per MSM on the tail stream.
static bool fx_chunk_join() {
  return env_default_on("PBF_MSM_CHUNK_JOIN");  // read per call: an A/B knob
}
constexpr uint32_t FX_JOIN_GROUP_C = 4096;  // per-chunk steps 1 .. 2048, the rest sequential
constexpr uint32_t FX_SEQ_CAP = 4;  // wide windows: spans <= 4 chunks summed in fx_bucket_into

// ---- the fixed-base tail for any window width (FxGeom: 2^(lb + hb) buckets, b = 2^lb h + l):
//   C_h = sum_l B_(2^lb h + l) (2^hb values), D_l = sum_h B_(2^lb h + l) (2^lb values),
//   T = sum_b (b + 1) B_b = sum_{k < hb} 2^(k + lb) Z_k + sum_{k < lb} 2^k Y_k + S,
//   Z_k = sum_{h: bit k of h} C_h, Y_k = sum_{l: bit k of l} D_l, S = sum_h C_h
// (the c = 16 kernels above with 256 -> 2^lb, 128 -> 2^hb). Workgroups of QW quads; every quad
// first adds its share of the values in sequence, then a quad tree. At c = 16 the sequences
// and trees are those of msm_fx_cd_q / msm_fx_subsets_q.
template <int QW>
__global__ void __launch_bounds__(4 * QW) msm_fxg_cd_q(const Xyzz* buckets, const ChunkPart* head,
                                                       const ChunkPart* tail, const uint32_t* start,
                                                       const uint32_t* end, Xyzz* cd, int lb, int hb) {
  __shared__ Xyzz red[QW];
  const uint32_t g = blockIdx.x, qi = threadIdx.x >> 2, L = 1u << lb, NH = 1u << hb;
  Xyzz v = G1::identity();
  if (g < NH) {  // C_g: L consecutive buckets, L / QW per quad
    const uint32_t per = (L + QW - 1) / QW;
    for (uint32_t i = 0; i < per; ++i) {
      const uint32_t l = per * qi + i;  // quad-uniform
      if (l < L) v = G1Quad::add(v, fx_bucket_q(L * g + l, buckets, head, tail, start, end));
    }
  } else {  // D_l: NH buckets L apart
    const uint32_t l = g - NH, per = (NH + QW - 1) / QW;
    for (uint32_t i = 0; i < per; ++i) {
      const uint32_t h = per * qi + i;
      if (h < NH) v = G1Quad::add(v, fx_bucket_q(L * h + l, buckets, head, tail, start, end));
    }
  }
  v = fx_tree_q(v, red);
  if (threadIdx.x == 0) cd[g] = v;
}
// The C_h / D_l sums of msm_fxg_cd_q on single lanes (wide windows: 2^18 .. 2^21 buckets, a
// throughput job; a quad addition costs four lanes for one sum): each lane adds per = count /
// lanes values in sequence, then a `lanes`-lane LDS tree. Workgroup g < gC: C_h for vc = 256 /
// lc values of h (lc = min(256, L / SEQ) lanes each); then D_l for vd values of l.
// Bucket k's parts added into acc: its whole sum (buckets[k]) when it lies in one chunk; its
// chunk-o tail run and its continuations head[o+1 .. e] one by one when it spans at most cap
// chunks (the wide-window tails skip the join for those: ~2 chunks per bucket); else the tail
// run and the joined continuations head[o+1].
__device__ __forceinline__ Xyzz fx_bucket_into(Xyzz acc, uint32_t k, const Xyzz* buckets, const ChunkPart* head,
                                               const ChunkPart* tail, const uint32_t* start, const uint32_t* end,
                                               uint32_t cap) {
  const uint32_t bs = start[k], be = end[k];
  if (be <= bs) return acc;
  const uint32_t o = bs / MSM_CH, e = (be - 1) / MSM_CH;
  if (o == e) return G1::add2(acc, buckets[k]);
  acc = G1::add2(acc, tail[o].acc);
  if (e - o > cap) return G1::add2(acc, head[o + 1].acc);
  for (uint32_t u = o + 1; u <= e; ++u) acc = G1::add2(acc, head[u].acc);
  return acc;
}
// Every bucket spanning chunks resolved to one sum in buckets[k] (one lane per bucket; its tail
// run plus its continuations as fx_bucket_into adds them): the C and D sums then add one value
// per bucket each, where each of them added the bucket's ~3 parts (wide windows, ~100 entries
// per bucket over 43-entry chunks).
__global__ void __launch_bounds__(256) msm_fx_resolve(Xyzz* buckets, const ChunkPart* head, const ChunkPart* tail,
                                                      const uint32_t* start, const uint32_t* end, uint32_t nb,
                                                      uint32_t cap, uint32_t hmax) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nb) return;
  const uint32_t bs = start[k], be = end[k];
  if (be <= bs) return;
  const uint32_t o = bs / MSM_CH, e = (be - 1) / MSM_CH;
  if (o == e) return;  // already whole in buckets[k]
  // hmax > 0: the partials of buckets spanning at most hmax chunks are still raw (msm_l29_finish);
  // a joined head[o + 1] (span > cap) was written converted by its join
  const bool rawp = hmax != 0 && e - o <= hmax;
  Xyzz acc = rawp ? l29::raw_to_xyzz(tail[o].raw) : tail[o].acc;
  if (e - o > cap) {
    acc = G1::add2(acc, head[o + 1].acc);
  } else {
    for (uint32_t u = o + 1; u <= e; ++u) acc = G1::add2(acc, rawp ? l29::raw_to_xyzz(head[u].raw) : head[u].acc);
  }
  buckets[k] = acc;
}
__device__ __forceinline__ Xyzz fx_bucket_resolved(Xyzz acc, uint32_t k, const Xyzz* buckets, const uint32_t* start,
                                                   const uint32_t* end) {
  return end[k] <= start[k] ? acc : G1::add2(acc, buckets[k]);
}
template <int SEQ, bool RES>
__global__ void __launch_bounds__(256) msm_fxg_cd_seq(const Xyzz* buckets, const ChunkPart* head,
                                                      const ChunkPart* tail, const uint32_t* start,
                                                      const uint32_t* end, Xyzz* cd, int lb, int hb, uint32_t cap) {
  __shared__ Xyzz red[256];
  const uint32_t L = 1u << lb, NH = 1u << hb, t = threadIdx.x, g = blockIdx.x;
  const uint32_t lc = L / SEQ < 256 ? L / SEQ : 256, vc = 256 / lc, gC = NH / vc;
  const uint32_t ld = NH / SEQ < 256 ? NH / SEQ : 256, vd = 256 / ld;
  Xyzz acc = G1::identity();
  uint32_t lanes, outi;
  if (g < gC) {
    const uint32_t h = g * vc + t / lc, per = L / lc, l0 = (t % lc) * per;
    for (uint32_t i = 0; i < per; ++i)
      acc = RES ? fx_bucket_resolved(acc, L * h + l0 + i, buckets, start, end)
                : fx_bucket_into(acc, L * h + l0 + i, buckets, head, tail, start, end, cap);
    lanes = lc;
    outi = h;
  } else {
    const uint32_t l = (g - gC) * vd + t / ld, per = NH / ld, h0 = (t % ld) * per;
    for (uint32_t i = 0; i < per; ++i)
      acc = RES ? fx_bucket_resolved(acc, L * (h0 + i) + l, buckets, start, end)
                : fx_bucket_into(acc, L * (h0 + i) + l, buckets, head, tail, start, end, cap);
    lanes = ld;
    outi = NH + l;
  }
  red[t] = acc;
  __syncthreads();
  for (uint32_t st = lanes / 2; st > 0; st >>= 1) {
    if (t % lanes < st) red[t] = G1::add2(red[t], red[t + st]);
    __syncthreads();
  }
  if (t % lanes == 0) cd[outi] = red[t];
}
static uint32_t fxg_cd_seq_groups(const FxGeom& g, uint32_t seq) {
  const uint32_t L = 1u << g.lb, NH = 1u << g.hb;
  const uint32_t lc = L / seq < 256 ? L / seq : 256, ld = NH / seq < 256 ? NH / seq : 256;
  return NH / (256 / lc) + L / (256 / ld);
}
// workgroup s < lb: 2^s Y_s; lb <= s < lb + hb: 2^s Z_(s - lb); s = lb + hb: S
template <int QW>
__global__ void __launch_bounds__(4 * QW) msm_fxg_subsets_q(const Xyzz* cd, Xyzz* sub, int lb, int hb) {
  __shared__ Xyzz red[QW];
  const uint32_t s = blockIdx.x, t = threadIdx.x >> 2, L = 1u << lb, NH = 1u << hb;
  const Xyzz* C = cd;
  const Xyzz* D = cd + NH;
  const uint32_t cnt = s < (uint32_t)lb ? L / 2 : s < (uint32_t)(lb + hb) ? NH / 2 : NH;
  const uint32_t per = (cnt + QW - 1) / QW;
  Xyzz v = G1::identity();
  for (uint32_t i = 0; i < per; ++i) {
    const uint32_t u = t * per + i;  // the u-th index with bit k set
    if (u >= cnt) break;             // quad-uniform
    if (s < (uint32_t)lb) {
      v = G1Quad::add(v, D[((u >> s) << (s + 1)) | (1u << s) | (u & ((1u << s) - 1))]);
    } else if (s < (uint32_t)(lb + hb)) {
      const uint32_t k = s - lb;
      v = G1Quad::add(v, C[((u >> k) << (k + 1)) | (1u << k) | (u & ((1u << k) - 1))]);
    } else {
      v = G1Quad::add(v, C[u]);
    }
  }
  v = fx_tree_q(v, red);
  if (t == 0) {
    const uint32_t e = s < (uint32_t)(lb + hb) ? s : 0;
    for (uint32_t i = 0; i < e; ++i) v = G1Quad::dbl(v);
    if (threadIdx.x == 0) sub[s] = v;
  }
}
// the nsub <= 32 scaled subset sums -> *out (32 quads)
__global__ void __launch_bounds__(128) msm_fxg_total_q(const Xyzz* sub, int nsub, Xyzz* out) {
  __shared__ Xyzz red[32];
  const uint32_t q = threadIdx.x >> 2;
  const Xyzz v = fx_tree_q(q < (uint32_t)nsub ? sub[q] : G1::identity(), red);
  if (threadIdx.x == 0) *out = v;
}

// Exact-content cache validation (snapshot_check below): diff[0] = 1 when a and b differ in
// any of their `words` u64 (benign same-value race; vector stores only).
__global__ void __launch_bounds__(256) k_snap_compare(const uint64_t* a, const uint64_t* b, uint64_t words, int* diff) {
  uint64_t d = 0;
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < words; j += (uint64_t)gridDim.x * 256)
    d |= a[j] ^ b[j];
  if (d) diff[0] = 1;
}

// Fixed-base comb for s * G (SRS::create): table[w][d-1] = d * 2^(8w) * G (affine,
// Montgomery), 32 byte windows x 255 digits (510 KiB, L2-resident); a scalar costs at most
// 32 mixed additions and no doublings (double-and-add: 256 doublings + ~128 additions).
constexpr int G1_TBL_W = 32, G1_TBL_D = 255;
__global__ void __launch_bounds__(256) g1_base_table_kernel(Affine* table) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= G1_TBL_W * G1_TBL_D) return;
  const uint32_t w = id / G1_TBL_D, d = id % G1_TBL_D + 1;
  Affine g;
  {
    U256 one = Fq::one_plain(), two = Fq::one_plain();
    two.w[0] = 2;
    g.x = Fq::to_mont(one);
    g.y = Fq::to_mont(two);
  }
  Xyzz acc = G1::identity();
  for (int b = 7; b >= 0; --b) {
    acc = G1::dbl(acc);
    if ((d >> b) & 1) acc = G1::madd(acc, g);
  }
  for (uint32_t i = 0; i < 8 * w; ++i) acc = G1::dbl(acc);
  U256 x, y;
  G1::to_affine_plain(acc, &x, &y);  // d 2^(8w) < r: never the identity
  table[id].x = Fq::to_mont(x);
  table[id].y = Fq::to_mont(y);
}
__global__ void __launch_bounds__(256) g1_mul_base_comb(const uint64_t* scalars, const Affine* table, uint64_t* out,
                                                        uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = scalars + 4 * i;
    Xyzz acc = G1::identity();
#pragma unroll 4
    for (int w = 0; w < G1_TBL_W; ++w) {
      const uint32_t d = (uint32_t)(s[w >> 3] >> (8 * (w & 7))) & 0xFF;
      if (d) acc = G1::madd(acc, table[w * G1_TBL_D + d - 1]);
    }
    U256 x, y;
    G1::to_affine_plain(acc, &x, &y);
    store_u256(out + 8 * i, x);
    store_u256(out + 8 * i + 4, y);
  }
}

// out_i = s_i * G (affine, canonical); scalars canonical Fr, 4 x u64 each (double-and-add;
// kept as the reference for the comb)
__global__ void __launch_bounds__(256) g1_mul_base_kernel(const uint64_t* scalars, uint64_t* out, uint64_t n) {
  Affine g;
  {
    U256 one = Fq::one_plain(), two = Fq::one_plain();
    two.w[0] = 2;
    g.x = Fq::to_mont(one);
    g.y = Fq::to_mont(two);
  }
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t* s = scalars + 4 * i;
    Xyzz acc = G1::identity();
    for (int b = 255; b >= 0; --b) {
      acc = G1::dbl(acc);
      if ((s[b >> 6] >> (b & 63)) & 1) acc = G1::madd(acc, g);
    }
    U256 x, y;
    G1::to_affine_plain(acc, &x, &y);
    store_u256(out + 8 * i, x);
    store_u256(out + 8 * i + 4, y);
  }
}

// ---------------------------------------------------------------- host orchestration
static uint64_t grid1(uint64_t count) {
  uint64_t b = (count + 255) / 256;
  return b > 16384 ? 16384 : (b ? b : 1);
}

struct MsmWork {
  DevBuf &pts, &inf, &keys, &vals, &keys2, &vals2, &start, &end, &buckets, &shares, &sums, &head, &tail, &parts,
      &span;
};

// scratch owned by the context (freed with it)
static MsmWork msm_work(pbf_ctx* ctx) {
  return MsmWork{ctx->buf("msm.pts"),     ctx->buf("msm.inf"),    ctx->buf("msm.keys"),   ctx->buf("msm.vals"),
                 ctx->buf("msm.keys2"),   ctx->buf("msm.vals2"),  ctx->buf("msm.start"),  ctx->buf("msm.end"),
                 ctx->buf("msm.buckets"), ctx->buf("msm.shares"), ctx->buf("msm.sums"),   ctx->buf("msm.head"),
                 ctx->buf("msm.tail"),    ctx->buf("msm.parts"),  ctx->buf("msm.span")};
}

// (key, value) pairs sorted by key bits [0, bits) into keys2 / vals2 (msm_sort.hpp), with the
// context's scratch
static int msm_sort_pairs(pbf_ctx* ctx, const uint32_t* keys, const uint32_t* vals, uint32_t* keys2, uint32_t* vals2,
                          uint64_t m, int bits, hipStream_t s, const std::string& pre = "msm.") {
  if (m > 0xFFFFFFFFull - RS_TILE_MAX) return fail(PBF_EINVAL, "too many MSM entries");
  DevBuf &tk = ctx->buf(pre + "sort.k"), &tv = ctx->buf(pre + "sort.v"), &hb = ctx->buf(pre + "sort.hist");
  const uint64_t ntiles = (m + RS_TILE - 1) / RS_TILE;
  int rc;
  if ((rc = tk.ensure(m * 4)) || (rc = tv.ensure(m * 4)) || (rc = hb.ensure((256 * ntiles + 256) * 4))) return rc;
  rs_sort(keys, vals, keys2, vals2, (uint32_t*)tk.p, (uint32_t*)tv.p, (uint32_t)m, bits, (uint32_t*)hb.p, s);
  PBF_HIP(hipGetLastError());
  return 0;
}

// The MSM sorts with their first pass from planar 16-bit digit codes (dg.dig, m = 16 n entries): (key, value) pairs sorted by the 16-bit (fixed-base) or 20-bit
// (windowed) key into keys2 / vals2. Pass 1 (bits 0-7) reads the codes, the later passes the
// ping-pong scratch. Default; PBF_MSM_FUSED_SORT=0 selects the (key, value) pair sort.
static bool msm_fused_sort() {
  return env_default_on("PBF_MSM_FUSED_SORT");  // read per call: an A/B knob (=0: pair sort)
}
// digit width of pass p of a `bits`-bit sort: as equal as possible (msm_sort.hpp rs_width);
// PBF_MSM_SORT_W8=1 keeps every pass but the last at 8 bits (A/B)
static int msm_sort_width(int bits, int p) {
  if (env_default_off("PBF_MSM_SORT_W8")) {  // read per call: an A/B knob
    const int rest = bits - 8 * p;
    return rest < 8 ? rest : 8;
  }
  return rs_width(bits, p);
}
// bits: key bits to sort (2 or 3 passes; the last lands in keys2 / vals2, the middle one in
// the caller's mid_k / mid_v buffers, free once the codes are read)
template <typename C>
static int msm_sort_digits(pbf_ctx* ctx, const RsDigitsT<C>& dg, uint32_t* keys2, uint32_t* vals2, uint32_t* mid_k,
                           uint32_t* mid_v, uint64_t m, int bits, hipStream_t s, const std::string& pre = "msm.") {
  if (m > 0xFFFFFFFFull - RS_TILE_MAX) return fail(PBF_EINVAL, "too many MSM entries");
  const int passes = rs_passes(bits), w0 = msm_sort_width(bits, 0);
  if (bits < 9 || bits > 24 || dg.kw % (1u << w0) || !rs_dig_ok(dg.n) || (passes == 3 && (!mid_k || !mid_v)))
    return fail(PBF_EINVAL, "digit sort: 9..24 key bits, whole first-pass digits per window, n >= 256");
  DevBuf &tk = ctx->buf(pre + "sort.k"), &tv = ctx->buf(pre + "sort.v"), &hb = ctx->buf(pre + "sort.hist");
  const uint64_t ntiles = (m + RS_TILE - 1) / RS_TILE;
  int rc;
  if ((rc = tk.ensure(m * 4)) || (rc = tv.ensure(m * 4)) || (rc = hb.ensure((256 * ntiles + 256) * 4))) return rc;
  uint32_t *k1 = (uint32_t*)tk.p, *v1 = (uint32_t*)tv.p, *hist = (uint32_t*)hb.p;
  rs_pass<RS_ITEMS, true, C>(nullptr, nullptr, k1, v1, (uint32_t)m, 0, hist, s, dg, w0);
  const int w1 = msm_sort_width(bits, 1);
  if (passes == 2) {
    rs_pass<RS_ITEMS>(k1, v1, keys2, vals2, (uint32_t)m, w0, hist, s, RsDigits{}, w1);
  } else {
    rs_pass<RS_ITEMS>(k1, v1, mid_k, mid_v, (uint32_t)m, w0, hist, s, RsDigits{}, w1);
    rs_pass<RS_ITEMS>(mid_k, mid_v, keys2, vals2, (uint32_t)m, w0 + w1, hist, s, RsDigits{}, msm_sort_width(bits, 2));
  }
  PBF_HIP(hipGetLastError());
  return 0;
}

// Enqueue the device part; window sums land in w.sums (MSM_NW Xyzz, Montgomery).
static int msm_device(pbf_ctx* ctx, const uint64_t* d_pts, const uint64_t* d_sc, uint64_t n, hipStream_t s,
                      MsmWork& w) {
  // the sort counts n * MSM_NW pairs in an int; scalars must be canonical Fr (< r < 2^254),
  // so the 16-bit signed-digit recoding never carries out of the top window
  if (n > 0x7FFFFFFFull / MSM_NW) return fail(PBF_EINVAL, "too many points (n * 16 must fit an int)");
  const uint64_t m = n * MSM_NW;
  int rc;
  if ((rc = w.pts.ensure(n * sizeof(Affine))) || (rc = w.inf.ensure(n)) || (rc = w.keys.ensure(m * 4)) ||
      (rc = w.vals.ensure(m * 4)) || (rc = w.keys2.ensure(m * 4)) || (rc = w.vals2.ensure(m * 4)) ||
      (rc = w.start.ensure((uint64_t)MSM_NW * MSM_NB * 4)) || (rc = w.end.ensure((uint64_t)MSM_NW * MSM_NB * 4)) ||
      (rc = w.buckets.ensure((uint64_t)MSM_NW * MSM_NB * sizeof(Xyzz))) ||
      (rc = w.shares.ensure((uint64_t)MSM_NW * (FX_NH + 256) * sizeof(Xyzz))) ||
      (rc = w.sums.ensure(MSM_NW * sizeof(Xyzz))) || (rc = w.parts.ensure(MSM_NW * 16 * sizeof(Xyzz))) ||
      (rc = w.span.ensure(4)) ||
      (rc = w.head.ensure((m / MSM_CH + 1) * sizeof(ChunkPart))) ||
      (rc = w.tail.ensure((m / MSM_CH + 1) * sizeof(ChunkPart))))
    return rc;
  hipLaunchKernelGGL(msm_points_to_mont, dim3(grid1(n)), dim3(256), 0, s, d_pts, (Affine*)w.pts.p,
                     (uint8_t*)w.inf.p, n);
  if (msm_fused_sort() && rs_dig_ok(n)) {
    // 16-bit digit codes in w.keys2 (read by pass 1; only pass 3 writes w.keys2 again)
    hipLaunchKernelGGL(msm_digits16, dim3(grid1(n)), dim3(256), 0, s, d_sc, (const uint8_t*)w.inf.p,
                       (uint16_t*)w.keys2.p, n);
    const RsDigits dg{(const uint16_t*)w.keys2.p, (uint32_t)n, 0, 0, 1u << MSM_BB, MSM_SENTINEL, MSM_NEG};
    if ((rc = msm_sort_digits(ctx, dg, (uint32_t*)w.keys2.p, (uint32_t*)w.vals2.p, (uint32_t*)w.keys.p,
                              (uint32_t*)w.vals.p, m, MSM_BB + 5, s)))
      return rc;
  } else {
    hipLaunchKernelGGL(msm_digits, dim3(grid1(n)), dim3(256), 0, s, d_sc, (const uint8_t*)w.inf.p,
                       (uint32_t*)w.keys.p, (uint32_t*)w.vals.p, n);
    if ((rc = msm_sort_pairs(ctx, (const uint32_t*)w.keys.p, (const uint32_t*)w.vals.p, (uint32_t*)w.keys2.p,
                             (uint32_t*)w.vals2.p, m, MSM_BB + 5, s)))
      return rc;
  }
  PBF_HIP(hipMemsetAsync(w.start.p, 0, (uint64_t)MSM_NW * MSM_NB * 4, s));
  PBF_HIP(hipMemsetAsync(w.end.p, 0, (uint64_t)MSM_NW * MSM_NB * 4, s));
  launch_bucket_bounds((const uint32_t*)w.keys2.p, m, (uint32_t*)w.start.p, (uint32_t*)w.end.p, MSM_SENTINEL, s);
  // the valid (non-sentinel) prefix of the sorted list: the sentinel sorts last; its
  // length is known only on the device, so chunks past it return at once. No bucket memset:
  // the reduction reads only the buckets the accumulation wrote (fx_bucket).
  const uint32_t nchunks = (uint32_t)((m + MSM_CH - 1) / MSM_CH);
  // the same tail as the fixed-base form, over 16 windows of 2^15 buckets (bucket id = key)
  constexpr uint32_t NBT = MSM_NW * MSM_NB;
  DevBuf &hk = ctx->buf("msm.hkey"), &tk = ctx->buf("msm.tkey"), &braw = ctx->buf("msm.braw");
  if ((rc = hk.ensure((uint64_t)nchunks * 4 + 4)) || (rc = tk.ensure((uint64_t)nchunks * 4 + 4))) return rc;
  PBF_HIP(hipMemsetAsync(w.span.p, 0, 4, s));
  if (msm_l29() && msm_rawflush()) {
    if ((rc = braw.ensure((uint64_t)NBT * 144))) return rc;
    hipLaunchKernelGGL(msm_chunk_acc_l29r, dim3((nchunks + 255) / 256), dim3(256), 0, s, (const Affine*)w.pts.p,
                       (const uint32_t*)w.keys2.p, (const uint32_t*)w.vals2.p, (const uint32_t*)w.start.p,
                       (const uint32_t*)w.end.p, (uint32_t)m, (uint32_t*)braw.p, (ChunkPart*)w.head.p,
                       (ChunkPart*)w.tail.p, MSM_SENTINEL, (const uint32_t*)nullptr, (uint32_t*)hk.p, (uint32_t*)tk.p);
    hipLaunchKernelGGL(msm_l29_finish, dim3(grid1((uint64_t)NBT + 2ull * nchunks)), dim3(256), 0, s,
                       (const uint32_t*)braw.p, (Xyzz*)w.buckets.p, (ChunkPart*)w.head.p, (ChunkPart*)w.tail.p,
                       (const uint32_t*)hk.p, (const uint32_t*)tk.p, (const uint32_t*)w.start.p,
                       (const uint32_t*)w.end.p, NBT, nchunks, MSM_SENTINEL, 0u);
  } else {
    hipLaunchKernelGGL(msm_l29() ? msm_chunk_acc_l29 : msm_chunk_acc, dim3((nchunks + 255) / 256), dim3(256), 0, s,
                       (const Affine*)w.pts.p, (const uint32_t*)w.keys2.p, (const uint32_t*)w.vals2.p,
                       (const uint32_t*)w.start.p, (const uint32_t*)w.end.p, (uint32_t)m, (Xyzz*)w.buckets.p,
                       (ChunkPart*)w.head.p, (ChunkPart*)w.tail.p, MSM_SENTINEL, (const uint32_t*)nullptr,
                       (uint32_t*)hk.p, (uint32_t*)tk.p);
  }
  hipLaunchKernelGGL(msm_max_span, dim3(max_span_groups(NBT)), dim3(256), 0, s, (const uint32_t*)w.start.p,
                     (const uint32_t*)w.end.p, NBT, (uint32_t*)w.span.p);
  const uint64_t mean_span = m / ((uint64_t)NBT * MSM_CH) + 2;
  for (uint32_t step = 1; step < nchunks && step < FX_JOIN_GROUP; step <<= 1) {
    const uint64_t items = (uint64_t)NBT * ((mean_span + 2 * step - 1) / (2 * step));
    hipLaunchKernelGGL(msm_join_step, dim3((uint32_t)((items + 255) / 256)), dim3(256), 0, s, (ChunkPart*)w.head.p,
                       (const uint32_t*)w.start.p, (const uint32_t*)w.end.p, NBT, step, (const uint32_t*)w.span.p,
                       ~0u);
  }
  hipLaunchKernelGGL(msm_join_rest, dim3(NBT / 256), dim3(256), 0, s, (ChunkPart*)w.head.p,
                     (const uint32_t*)w.start.p, (const uint32_t*)w.end.p, NBT, (const uint32_t*)w.span.p);
  {
    const char* e = ab_env("PBF_MSM_CD_SEQ");  // an A/B knob (PBF_AB build only)
    const int v = e ? atoi(e) : 8;
    const int cd_seq = v == 2 || v == 4 || v == 16 ? v : 8;
    auto* fn = cd_seq == 2 ? msm_fx_cd_seq<2> : cd_seq == 4 ? msm_fx_cd_seq<4> : cd_seq == 16 ? msm_fx_cd_seq<16> : msm_fx_cd_seq<8>;
    hipLaunchKernelGGL(fn, dim3(256 / cd_seq, MSM_NW), dim3(256), 0, s, (const Xyzz*)w.buckets.p,
                       (const ChunkPart*)w.head.p, (const ChunkPart*)w.tail.p, (const uint32_t*)w.start.p,
                       (const uint32_t*)w.end.p, (Xyzz*)w.shares.p);
  }
  if (msm_quad_tail()) {
    hipLaunchKernelGGL(msm_fx_subsets_q, dim3(16, MSM_NW), dim3(512), 0, s, (const Xyzz*)w.shares.p, (Xyzz*)w.parts.p);
    hipLaunchKernelGGL(msm_fx_total_q, dim3(MSM_NW), dim3(64), 0, s, (const Xyzz*)w.parts.p, (Xyzz*)w.sums.p);
  } else {
    hipLaunchKernelGGL(msm_fx_subsets, dim3(16, MSM_NW), dim3(128), 0, s, (const Xyzz*)w.shares.p, (Xyzz*)w.parts.p);
    hipLaunchKernelGGL(msm_fx_total, dim3(MSM_NW), dim3(16), 0, s, (const Xyzz*)w.parts.p, (Xyzz*)w.sums.p);
  }
  PBF_HIP(hipGetLastError());
  return 0;
}

// The 16-window Horner on the device (A/B against msm_finish_host, PBF_MSM_DEVICE_HORNER=1): one
// lane, 15 x (16 doublings + 1 addition) in sequence -- a latency chain that a GPU lane runs at
// ~1 Fq product per ~2200 cycles, the host core far faster.
__global__ void msm_horner_kernel(const Xyzz* sums, Xyzz* out) {
  if (threadIdx.x != 0) return;
  Xyzz acc = sums[MSM_NW - 1];
  for (int w = MSM_NW - 2; w >= 0; --w) {
    for (int i = 0; i < MSM_C; ++i) acc = G1::dbl(acc);
    acc = G1::add(acc, sums[w]);
  }
  *out = acc;
}

static void msm_finish_host(const Xyzz* sums, uint64_t* out) {
  Xyzz acc = sums[MSM_NW - 1];
  for (int w = MSM_NW - 2; w >= 0; --w) {
    for (int i = 0; i < MSM_C; ++i) acc = G1::dbl(acc);
    acc = G1::add(acc, sums[w]);
  }
  U256 x, y;
  G1::to_affine_plain(acc, &x, &y);
  for (int i = 0; i < 4; ++i) {
    out[i] = (uint64_t)x.w[2 * i] | ((uint64_t)x.w[2 * i + 1] << 32);
    out[4 + i] = (uint64_t)y.w[2 * i] | ((uint64_t)y.w[2 * i + 1] << 32);
  }
}

// ---- context caches validated by exact content (the 64-bit XOR fingerprint they
// used before is linear over GF(2), so a chosen circuit or point set could collide with a cached
// one). The context keeps a device copy -- a snapshot -- of every input a cache is derived from;
// a hit requires the input to equal its snapshot word for word.
int snapshot_check(pbf_ctx* ctx, const char* consumer, const SnapItem* items, int k, hipStream_t s, bool* same) {
  DevBuf& fl = ctx->buf("snap.flags");
  int rc = fl.ensure((size_t)k * sizeof(int));
  if (rc) return rc;
  int* flags = (int*)fl.p;
  PBF_HIP(hipMemsetAsync(flags, 0, (size_t)k * sizeof(int), s));
  std::vector<int> fresh(k, 0), diff(k, 0);
  for (int i = 0; i < k; ++i) {
    DevBuf& b = ctx->buf(std::string("snap.") + items[i].name);
    auto it = ctx->snap_words.find(items[i].name);
    if (!b.p || it == ctx->snap_words.end() || it->second != items[i].words) {
      fresh[i] = 1;
      continue;
    }
    if (items[i].words == 0) continue;
    uint64_t blocks = (items[i].words + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_snap_compare, dim3((uint32_t)blocks), dim3(256), 0, s, (const uint64_t*)b.p, items[i].p,
                       items[i].words, flags + i);
  }
  PBF_HIP(hipGetLastError());
  PBF_HIP(hipMemcpyAsync(diff.data(), flags, (size_t)k * sizeof(int), hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  *same = true;
  for (int i = 0; i < k; ++i) {
    const std::string used = std::string(consumer) + "/" + items[i].name;
    if (!fresh[i] && !diff[i]) {
      // the data equals the snapshot; the consumer's cache is current only if it was built from
      // this very snapshot (another consumer may have replaced it since)
      if (ctx->snap_used[used] != ctx->snap_gen[items[i].name]) *same = false;
      ctx->snap_used[used] = ctx->snap_gen[items[i].name];
      continue;
    }
    *same = false;
    DevBuf& b = ctx->buf(std::string("snap.") + items[i].name);
    ctx->snap_words.erase(items[i].name);  // valid again only once the copy is enqueued
    if ((rc = b.ensure(items[i].words * 8 + 8))) return rc;
    if (items[i].words) PBF_HIP(hipMemcpyAsync(b.p, items[i].p, items[i].words * 8, hipMemcpyDeviceToDevice, s));
    ctx->snap_words[items[i].name] = items[i].words;
    ctx->snap_gen[items[i].name] = ctx->snap_next_gen++;
    ctx->snap_used[used] = ctx->snap_gen[items[i].name];
  }
  return 0;
}

// the window table of the n points at d_pts (built on first use; rebuilt when the points
// differ from the ones it was built from, wherever they live); the table's identity flags are
// kept with it (fixed_base.inf)
int msm_fixed_table(pbf_ctx* ctx, const uint64_t* d_pts, uint64_t n, hipStream_t s, const Affine** out) {
  const FxGeom g = fx_geom_of(fx_default_c(ctx, n));
  if (n == 0 || n > 0x7FFFFFFFull / g.nw) return fail(PBF_EINVAL, "fixed-base MSM: bad point count");
  const SnapItem it{"g1pts", d_pts, 8 * n};
  bool same = false;
  int rc = snapshot_check(ctx, "fx", &it, 1, s, &same);
  if (rc) return rc;
  auto& fb = ctx->fixed_base;
  if (same && fb.valid && fb.n == n && fb.c == g.c && fb.table.p) {
    *out = (const Affine*)fb.table.p;
    return 0;
  }
  fb.valid = false;
  if ((rc = fb.table.ensure((uint64_t)g.nw * n * sizeof(Affine))) || (rc = fb.inf.ensure(n))) return rc;
  Affine* tbl = (Affine*)fb.table.p;
  hipLaunchKernelGGL(msm_points_to_mont, dim3(grid1(n)), dim3(256), 0, s, d_pts, tbl, (uint8_t*)fb.inf.p, n);
  for (int w = 1; w < g.nw; ++w)
    hipLaunchKernelGGL(msm_table_window, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                       (const Affine*)(tbl + (uint64_t)(w - 1) * n), tbl + (uint64_t)w * n, n, g.c);
  PBF_HIP(hipGetLastError());
  fb.n = n;
  fb.c = g.c;
  fb.valid = true;
  *out = tbl;
  return 0;
}

// the context's window table if it was built from exactly these points (content checked),
// else null; never builds one
int msm_fixed_lookup(pbf_ctx* ctx, const uint64_t* d_pts, uint64_t n, hipStream_t s, const Affine** out) {
  *out = nullptr;
  auto& fb = ctx->fixed_base;
  if (!fb.valid || fb.n != n || !fb.table.p) return 0;
  auto w = ctx->snap_words.find("g1pts");
  if (w == ctx->snap_words.end() || w->second != 8 * n) return 0;
  if (ctx->snap_used["fx/g1pts"] != ctx->snap_gen["g1pts"]) return 0;  // replaced since the build
  DevBuf& fl = ctx->buf("snap.flags");
  int rc = fl.ensure(sizeof(int));
  if (rc) return rc;
  PBF_HIP(hipMemsetAsync(fl.p, 0, sizeof(int), s));
  uint64_t blocks = (8 * n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_snap_compare, dim3((uint32_t)blocks), dim3(256), 0, s,
                     (const uint64_t*)ctx->buf("snap.g1pts").p, d_pts, 8 * n, (int*)fl.p);
  PBF_HIP(hipGetLastError());
  int diff = 0;
  PBF_HIP(hipMemcpyAsync(&diff, fl.p, sizeof(int), hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  if (!diff) *out = (const Affine*)fb.table.p;
  return 0;
}

int MsmTail::ensure() {
  if (aux) return 0;
  PBF_HIP(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
  PBF_HIP(hipStreamCreateWithFlags(&prep, hipStreamNonBlocking));
  for (int i = 0; i < MSM_TAIL_SLOTS; ++i) {
    PBF_HIP(hipEventCreateWithFlags(&ready[i], hipEventDisableTiming));
    PBF_HIP(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
  }
  for (int i = 0; i < MSM_PREP_SLOTS; ++i) {
    PBF_HIP(hipEventCreateWithFlags(&prep_done[i], hipEventDisableTiming));
    PBF_HIP(hipEventCreateWithFlags(&prep_free[i], hipEventDisableTiming));
  }
  PBF_HIP(hipEventCreateWithFlags(&sc_ready, hipEventDisableTiming));
  return 0;
}
MsmTail::~MsmTail() {
  if (!aux) return;
  (void)hipSetDevice(device);
  if (prep) (void)hipStreamSynchronize(prep);
  (void)hipStreamSynchronize(aux);
  if (prep) (void)hipStreamDestroy(prep);
  (void)hipStreamDestroy(aux);
  for (int i = 0; i < MSM_TAIL_SLOTS; ++i) {
    if (ready[i]) (void)hipEventDestroy(ready[i]);
    if (done[i]) (void)hipEventDestroy(done[i]);
  }
  for (int i = 0; i < MSM_PREP_SLOTS; ++i) {
    if (prep_done[i]) (void)hipEventDestroy(prep_done[i]);
    if (prep_free[i]) (void)hipEventDestroy(prep_free[i]);
  }
  if (sc_ready) (void)hipEventDestroy(sc_ready);
}

// Opt-in (PBF_MSM_PREP=1): measured in the prover (profiles/r04/prep_ab.log) at 2^20 gates 25.3-26.0
// ms against 24.8 ms without it, at 2^24 gates 324.8-325.9 against 328.9 ms -- the sort kernels
// take CU slots from the VALU-bound accumulation they run beside, which slows it by about as
// much as their own time.
hipEvent_t msm_scalars_ready(pbf_ctx* ctx, hipStream_t s) {
  if (!env_default_off("PBF_MSM_PREP")) return nullptr;  // read per call: an A/B knob
  MsmTail& t = ctx->msm_tail;
  if (t.ensure() || hipEventRecord(t.sc_ready, s) != hipSuccess) return nullptr;  // one stream then
  return t.sc_ready;
}

int msm_fixed_wait(pbf_ctx* ctx, hipStream_t s) {
  MsmTail& t = ctx->msm_tail;
  if (t.last >= 0) PBF_HIP(hipStreamWaitEvent(s, t.done[t.last], 0));  // the side stream is in order
  return 0;
}

// sum_i scalars[i] * P_(first + i), i < n, against the context's window table of n_table
// points; the result (XYZZ, Montgomery) is written to *d_result on the device (nothing waits
// for it).
// On `s`: digits, the sort by bucket, bucket bounds and the accumulation
// (throughput-bound, the whole chip). On the context's side stream: the boundary join and
// the bucket reduction (latency-bound chains of a few hundred waves), overlapping whatever
// the caller enqueues next on `s`.
int msm_fixed_device(pbf_ctx* ctx, const Affine* table, uint64_t n_table, uint64_t first, const uint64_t* d_sc,
                     uint64_t n, hipStream_t s, Xyzz* d_result, hipEvent_t sc_ready) {
  if (first + n > n_table) return fail(PBF_EINVAL, "fixed-base MSM: range beyond the table");
  auto& fb = ctx->fixed_base;
  if ((const void*)table != fb.table.p || n_table != fb.n || !fb.inf.p)
    return fail(PBF_EINVAL, "fixed-base MSM: not the context's table");
  const FxGeom g = fx_geom_of(fb.c);
  const uint32_t NB = g.nb;
  const uint64_t m = n * g.nw;  // entries at most (zero digits are skipped)
  MsmTail& tl = ctx->msm_tail;
  int rc;
  if ((rc = tl.ensure())) return rc;
  const int slot = tl.next;
  const std::string pre = "msm.f" + std::to_string(slot) + ".";
  // digits, sort and bucket bounds: on the prep stream q (after the scalars' event; the sort
  // buffers of prep slot ps) or on s
  const bool use_prep = sc_ready != nullptr;
  const int ps = tl.prep_next;
  const hipStream_t q = use_prep ? tl.prep : s;
  const std::string sp = use_prep ? "msm.p" + std::to_string(ps) + "." : std::string("msm.");
  DevBuf &keys = ctx->buf(sp + "keys"), &vals = ctx->buf(sp + "vals"), &keys2 = ctx->buf(sp + "keys2"),
         &vals2 = ctx->buf(sp + "vals2");
  DevBuf &start = ctx->buf(pre + "start"), &end = ctx->buf(pre + "end"), &buckets = ctx->buf(pre + "buckets"),
         &shares = ctx->buf(pre + "shares"), &parts = ctx->buf(pre + "parts"), &head = ctx->buf(pre + "head"),
         &tail = ctx->buf(pre + "tail"), &spb = ctx->buf(pre + "span"), &hk = ctx->buf(pre + "hkey"),
         &tk = ctx->buf(pre + "tkey");
  DevBuf& braw = ctx->buf("msm.braw");  // read only on s (msm_l29_finish), before the tail forks
  if (use_prep) {
    PBF_HIP(hipStreamWaitEvent(q, sc_ready, 0));
    if (tl.prep_used[ps]) {
      PBF_HIP(hipStreamWaitEvent(q, tl.prep_free[ps], 0));  // its last accumulation has read it
      if (keys2.bytes < m * 4 || ctx->buf(sp + "sort.k").bytes < m * 4)
        PBF_HIP(hipEventSynchronize(tl.prep_free[ps]));  // reallocation
    }
  }
  // a slot's buffers may still be read by its previous tail: reuse waits for it, reallocation
  // synchronises
  if (tl.used[slot]) {
    PBF_HIP(hipStreamWaitEvent(s, tl.done[slot], 0));
    if (use_prep) PBF_HIP(hipStreamWaitEvent(q, tl.done[slot], 0));
  }
  const uint64_t hbytes = (m / MSM_CH + 1) * sizeof(ChunkPart);
  const uint64_t nshare = (1ull << g.hb) + (1ull << g.lb);
  if ((head.bytes < hbytes || tail.bytes < hbytes || start.bytes < (uint64_t)NB * 4 || hk.bytes < m / MSM_CH * 4 + 8 ||
       buckets.bytes < (uint64_t)NB * sizeof(Xyzz) || shares.bytes < nshare * sizeof(Xyzz)) &&
      tl.used[slot])
    PBF_HIP(hipEventSynchronize(tl.done[slot]));
  if ((rc = keys.ensure(m * 4)) || (rc = vals.ensure(m * 4)) || (rc = keys2.ensure(m * 4)) ||
      (rc = vals2.ensure(m * 4)) || (rc = start.ensure((uint64_t)NB * 4)) || (rc = end.ensure((uint64_t)NB * 4)) ||
      (rc = buckets.ensure((uint64_t)NB * sizeof(Xyzz))) || (rc = shares.ensure(nshare * sizeof(Xyzz))) ||
      (rc = parts.ensure(32 * sizeof(Xyzz))) || (rc = head.ensure(hbytes)) || (rc = tail.ensure(hbytes)) ||
      (rc = spb.ensure(4)) || (rc = hk.ensure(m / MSM_CH * 4 + 8)) || (rc = tk.ensure(m / MSM_CH * 4 + 8)))
    return rc;
  const uint8_t* inf = (const uint8_t*)fb.inf.p;
  // ---- digits, sort by bucket, bucket bounds (on q)
  if ((uint64_t)g.nw * n_table >= MSM_NEG) return fail(PBF_EINVAL, "fixed-base MSM: table too large");
  if (msm_fused_sort() && rs_dig_ok(n)) {
    // keys holds the digit codes (2 B per entry at c = 16, else 4 B); for a 3-pass sort keys
    // and vals then take the middle pass (the codes are read by then)
    if (g.c == 16) {
      hipLaunchKernelGGL((msm_fx_digits_code<uint16_t, 16>), dim3(grid1(n)), dim3(256), 0, q, d_sc, inf, first, n,
                         (uint16_t*)keys.p, g.c, g.nw);
      const RsDigits dg{(const uint16_t*)keys.p, (uint32_t)n, (uint32_t)n_table, (uint32_t)first, 0, NB, MSM_NEG};
      rc = msm_sort_digits(ctx, dg, (uint32_t*)keys2.p, (uint32_t*)vals2.p, (uint32_t*)keys.p, (uint32_t*)vals.p, m,
                           g.c, q, sp);
    } else {
      auto* dk = g.c == 18 ? msm_fx_digits_code<uint32_t, 18>
                 : g.c == 20 ? msm_fx_digits_code<uint32_t, 20>
                             : msm_fx_digits_code<uint32_t, 22>;
      hipLaunchKernelGGL(dk, dim3(grid1(n)), dim3(256), 0, q, d_sc, inf, first, n, (uint32_t*)keys.p, g.c, g.nw);
      const RsDigitsT<uint32_t> dg{(const uint32_t*)keys.p, (uint32_t)n, (uint32_t)n_table, (uint32_t)first, 0, NB,
                                   MSM_NEG};
      rc = msm_sort_digits(ctx, dg, (uint32_t*)keys2.p, (uint32_t*)vals2.p, (uint32_t*)keys.p, (uint32_t*)vals.p, m,
                           g.c, q, sp);
    }
    if (rc) return rc;
  } else {
    hipLaunchKernelGGL(msm_fx_digits, dim3(grid1(n)), dim3(256), 0, q, d_sc, inf, n_table, first, n,
                       (uint32_t*)keys.p, (uint32_t*)vals.p, g.c, g.nw);
    if ((rc = msm_sort_pairs(ctx, (const uint32_t*)keys.p, (const uint32_t*)vals.p, (uint32_t*)keys2.p,
                             (uint32_t*)vals2.p, m, g.c, q, sp)))
      return rc;
  }
  hipLaunchKernelGGL(msm_fx_clear, dim3(NB / 256), dim3(256), 0, q, (uint32_t*)start.p, (uint32_t*)end.p,
                     (uint32_t*)spb.p);
  launch_bucket_bounds((const uint32_t*)keys2.p, m, (uint32_t*)start.p, (uint32_t*)end.p, NB, q);
  if (use_prep) {
    PBF_HIP(hipGetLastError());
    PBF_HIP(hipEventRecord(tl.prep_done[ps], q));
    PBF_HIP(hipStreamWaitEvent(s, tl.prep_done[ps], 0));
  }
  // ---- accumulation
  // no bucket memset: msm_fx_cd reads only the buckets the accumulation wrote (fx_bucket)
  const uint32_t nchunks = (uint32_t)((m + MSM_CH - 1) / MSM_CH);
  const bool rawf = msm_l29() && msm_rawflush(g.c > 16);
  // the wide-window tail converts the partials of buckets spanning <= HJ_MAX chunks as it reads
  // them (heavy join, resolve); msm_l29_finish only the rest (PBF_MSM_DEFER_CONV=0: all, A/B).
  // The conditions are those of the tail below: wide windows, chunk join, single-lane C / D
  // sums, heavy join and resolve all on.
  const bool defer = rawf && g.c > 16 && fx_chunk_join() && !env_default_off("PBF_MSM_CD_QUAD") &&
                     env_default_on("PBF_MSM_HEAVY_JOIN") && env_default_on("PBF_MSM_CD_RESOLVE") &&
                     env_default_on("PBF_MSM_DEFER_CONV");  // read per call: A/B knobs
  const uint32_t hmax = defer ? HJ_MAX : 0u;
  if (rawf) {
    if ((rc = braw.ensure((uint64_t)NB * 144))) return rc;
    hipLaunchKernelGGL(msm_chunk_acc_l29r, dim3((nchunks + 255) / 256), dim3(256), 0, s, table,
                       (const uint32_t*)keys2.p, (const uint32_t*)vals2.p, (const uint32_t*)start.p,
                       (const uint32_t*)end.p, (uint32_t)m, (uint32_t*)braw.p, (ChunkPart*)head.p, (ChunkPart*)tail.p,
                       NB, (const uint32_t*)nullptr, (uint32_t*)hk.p, (uint32_t*)tk.p);
    hipLaunchKernelGGL(msm_l29_finish, dim3(grid1((uint64_t)NB + 2ull * nchunks)), dim3(256), 0, s,
                       (const uint32_t*)braw.p, (Xyzz*)buckets.p, (ChunkPart*)head.p, (ChunkPart*)tail.p,
                       (const uint32_t*)hk.p, (const uint32_t*)tk.p, (const uint32_t*)start.p, (const uint32_t*)end.p,
                       NB, nchunks, NB, hmax);
  } else {
    hipLaunchKernelGGL(msm_l29() ? msm_chunk_acc_l29 : msm_chunk_acc, dim3((nchunks + 255) / 256), dim3(256), 0, s,
                       table, (const uint32_t*)keys2.p, (const uint32_t*)vals2.p, (const uint32_t*)start.p,
                       (const uint32_t*)end.p, (uint32_t)m, (Xyzz*)buckets.p, (ChunkPart*)head.p, (ChunkPart*)tail.p,
                       NB, (const uint32_t*)nullptr, (uint32_t*)hk.p, (uint32_t*)tk.p);
  }
  hipLaunchKernelGGL(msm_max_span, dim3(max_span_groups(NB)), dim3(256), 0, s, (const uint32_t*)start.p,
                     (const uint32_t*)end.p, NB, (uint32_t*)spb.p);
  PBF_HIP(hipGetLastError());
  if (use_prep) {  // prep slot ps is free once the accumulation has read keys2 / vals2
    PBF_HIP(hipEventRecord(tl.prep_free[ps], s));
    tl.prep_used[ps] = true;
    tl.prep_next = (ps + 1) % MSM_PREP_SLOTS;
  }
  // ---- the tail, on the side stream
  hipStream_t a = tl.aux;
  PBF_HIP(hipEventRecord(tl.ready[slot], s));
  PBF_HIP(hipStreamWaitEvent(a, tl.ready[slot], 0));
  // join steps 1 .. FX_JOIN_GROUP / 2 (steps past the largest span exit at once); wider spans
  // are finished by msm_join_rest. The grid covers the mean span's pair slots (the kernel
  // strides over the rest).
  if (g.c > 16 && fx_chunk_join()) {
    // buckets spanning up to `cap` chunks (twice the mean span, a power of two): the per-bucket
    // steps; heavier ones: the per-chunk steps up to FX_JOIN_GROUP_C / 2 (both exit at once past
    // the largest span), then msm_join_rest_g
    // wide windows (single-lane C / D sums): buckets spanning up to FX_SEQ_CAP chunks are not
    // joined at all, fx_bucket_into adds their continuations in sequence
    const bool wide = !(g.c == 16 || env_default_off("PBF_MSM_CD_QUAD"));
    const uint64_t mean_span = m / ((uint64_t)NB * MSM_CH) + 2;
    uint32_t cap = 2;
    while (cap < 2 * mean_span && cap < FX_JOIN_GROUP_C) cap <<= 1;
    if (wide) cap = FX_SEQ_CAP;
    // wide windows: the heavy buckets listed and joined in two launches (PBF_MSM_HEAVY_JOIN=0:
    // the tree steps below, A/B)
    const bool heavy = wide && env_default_on("PBF_MSM_HEAVY_JOIN");  // read per call: an A/B knob
    if (heavy) {
      DevBuf& hl = ctx->buf(pre + "hlist");
      if (hl.bytes < (uint64_t)NB * 4 + 4 && tl.used[slot]) PBF_HIP(hipEventSynchronize(tl.done[slot]));
      if ((rc = hl.ensure((uint64_t)NB * 4 + 4))) return rc;
      uint32_t* cnt = (uint32_t*)hl.p + NB;
      PBF_HIP(hipMemsetAsync(cnt, 0, 4, a));
      hipLaunchKernelGGL(msm_heavy_list, dim3(NB / 256), dim3(256), 0, a, (const uint32_t*)start.p,
                         (const uint32_t*)end.p, NB, cap, HJ_MAX, (uint32_t*)hl.p, cnt);
      hipLaunchKernelGGL(msm_join_heavy, dim3(1024), dim3(256), 0, a, (ChunkPart*)head.p, (const uint32_t*)hl.p,
                         (const uint32_t*)cnt, (const uint32_t*)start.p, (const uint32_t*)end.p, (uint32_t)defer);
    }
    // (with the heavy join the tree steps take only the buckets spanning more than HJ_MAX chunks
    // -- skewed scalars -- and exit at once when there are none)
    const uint32_t jcap = heavy ? HJ_MAX : cap;
    for (uint32_t step = 1; step < nchunks && step < FX_JOIN_GROUP_C; step <<= 1) {
      if (step < cap && !wide) {
        const uint64_t items = (uint64_t)NB * ((mean_span + 2 * step - 1) / (2 * step));
        hipLaunchKernelGGL(msm_join_step, dim3((uint32_t)((items + 255) / 256)), dim3(256), 0, a, (ChunkPart*)head.p,
                           (const uint32_t*)start.p, (const uint32_t*)end.p, NB, step, (const uint32_t*)spb.p, cap);
      }
      hipLaunchKernelGGL(msm_join_chunks, dim3((uint32_t)grid1(nchunks)), dim3(256), 0, a, (ChunkPart*)head.p,
                         (const uint32_t*)hk.p, (const uint32_t*)start.p, (const uint32_t*)end.p, nchunks, step,
                         (const uint32_t*)spb.p, NB, jcap);
    }
    hipLaunchKernelGGL(msm_join_rest_g, dim3(NB / 256), dim3(256), 0, a, (ChunkPart*)head.p, (const uint32_t*)start.p,
                       (const uint32_t*)end.p, NB, (const uint32_t*)spb.p, FX_JOIN_GROUP_C);
  } else {
    const uint64_t mean_span = m / ((uint64_t)NB * MSM_CH) + 2;
    for (uint32_t step = 1; step < nchunks && step < FX_JOIN_GROUP; step <<= 1) {
      const uint64_t items = (uint64_t)NB * ((mean_span + 2 * step - 1) / (2 * step));
      hipLaunchKernelGGL(msm_join_step, dim3((uint32_t)((items + 255) / 256)), dim3(256), 0, a, (ChunkPart*)head.p,
                         (const uint32_t*)start.p, (const uint32_t*)end.p, NB, step, (const uint32_t*)spb.p, ~0u);
    }
    hipLaunchKernelGGL(msm_join_rest, dim3(NB / 256), dim3(256), 0, a, (ChunkPart*)head.p, (const uint32_t*)start.p,
                       (const uint32_t*)end.p, NB, (const uint32_t*)spb.p);
  }
  if (g.c == 16 && !msm_quad_tail()) {
    hipLaunchKernelGGL(msm_fx_cd, dim3(FX_NH + 256), dim3(256), 0, a, (const Xyzz*)buckets.p, (const ChunkPart*)head.p,
                       (const ChunkPart*)tail.p, (const uint32_t*)start.p, (const uint32_t*)end.p, (Xyzz*)shares.p);
    hipLaunchKernelGGL(msm_fx_subsets, dim3(16), dim3(128), 0, a, (const Xyzz*)shares.p, (Xyzz*)parts.p);
    hipLaunchKernelGGL(msm_fx_total, dim3(1), dim3(16), 0, a, (const Xyzz*)parts.p, d_result);
  } else {
    // C / D sums: quads at c = 16 (latency: 384 short trees), single lanes above (throughput:
    // 2^18 .. 2^21 buckets); then the subset trees on quads
    if (g.c == 16 || env_default_off("PBF_MSM_CD_QUAD")) {  // read per call: an A/B knob
      auto* cd = g.c == 16 ? msm_fxg_cd_q<64> : msm_fxg_cd_q<128>;
      const uint32_t qw = g.c == 16 ? 64 : 128;
      hipLaunchKernelGGL(cd, dim3((uint32_t)nshare), dim3(4 * qw), 0, a, (const Xyzz*)buckets.p,
                         (const ChunkPart*)head.p, (const ChunkPart*)tail.p, (const uint32_t*)start.p,
                         (const uint32_t*)end.p, (Xyzz*)shares.p, g.lb, g.hb);
    } else {
      const uint32_t cap_seq = g.c > 16 && fx_chunk_join() ? FX_SEQ_CAP : 1;
      // resolve the spanning buckets once (default; PBF_MSM_CD_RESOLVE=0: the C and D sums each
      // add the parts, A/B)
      const bool res = env_default_on("PBF_MSM_CD_RESOLVE");  // read per call: an A/B knob
      if (res)
        hipLaunchKernelGGL(msm_fx_resolve, dim3(NB / 256), dim3(256), 0, a, (Xyzz*)buckets.p, (const ChunkPart*)head.p,
                           (const ChunkPart*)tail.p, (const uint32_t*)start.p, (const uint32_t*)end.p, NB, cap_seq,
                           hmax);
      const bool s32 = env_default_off("PBF_MSM_CD_SEQ32");  // read per call: an A/B knob
      auto* cdk = s32 ? (res ? msm_fxg_cd_seq<32, true> : msm_fxg_cd_seq<32, false>)
                      : (res ? msm_fxg_cd_seq<8, true> : msm_fxg_cd_seq<8, false>);
      hipLaunchKernelGGL(cdk, dim3(fxg_cd_seq_groups(g, s32 ? 32 : 8)), dim3(256), 0, a, (const Xyzz*)buckets.p,
                         (const ChunkPart*)head.p, (const ChunkPart*)tail.p, (const uint32_t*)start.p,
                         (const uint32_t*)end.p, (Xyzz*)shares.p, g.lb, g.hb, cap_seq);
    }
    hipLaunchKernelGGL(msm_fxg_subsets_q<128>, dim3(g.lb + g.hb + 1), dim3(512), 0, a, (const Xyzz*)shares.p,
                       (Xyzz*)parts.p, g.lb, g.hb);
    hipLaunchKernelGGL(msm_fxg_total_q, dim3(1), dim3(128), 0, a, (const Xyzz*)parts.p, g.lb + g.hb + 1, d_result);
  }
  PBF_HIP(hipGetLastError());
  PBF_HIP(hipEventRecord(tl.done[slot], a));
  tl.used[slot] = true;
  tl.last = slot;
  tl.next = (slot + 1) % MSM_TAIL_SLOTS;
  return 0;
}

void xyzz_to_affine_u64(const Xyzz& p, uint64_t* out) {
  U256 x, y;
  G1::to_affine_plain(p, &x, &y);
  u256_to_u64(x, out);
  u256_to_u64(y, out + 4);
}

static bool host_fq_canonical(const uint64_t* v) {
  U256 x;
  for (int i = 0; i < 4; ++i) { x.w[2 * i] = (uint32_t)v[i]; x.w[2 * i + 1] = (uint32_t)(v[i] >> 32); }
  return !Fq::geq_p(x);
}
static bool host_fr_canonical(const uint64_t* v) {
  U256 x;
  for (int i = 0; i < 4; ++i) { x.w[2 * i] = (uint32_t)v[i]; x.w[2 * i + 1] = (uint32_t)(v[i] >> 32); }
  return !Fr::geq_p(x);
}

}  // namespace pbf

using namespace pbf;

extern "C" {

// SRS::eval_at_s (plonk.rs:51-58): out = sum_i scalars[i] * points[i] (host buffers)
int pbf_msm_g1_bn254(pbf_ctx* ctx, const uint64_t* points, const uint64_t* scalars, size_t n, uint64_t* out) {
  if (!ctx || !out || (n && (!points || !scalars))) return fail(PBF_EINVAL, "null argument");
  for (size_t i = 0; i < n; ++i)
    if (!host_fq_canonical(points + 8 * i) || !host_fq_canonical(points + 8 * i + 4) ||
        !host_fr_canonical(scalars + 4 * i))
      return fail(PBF_EINVAL, "input not canonical");
  if (n == 0) { for (int i = 0; i < 8; ++i) out[i] = 0; return PBF_OK; }
  PBF_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->host_stream();
  int rc;
  if ((rc = ctx->io0.ensure(n * 64)) || (rc = ctx->io1.ensure(n * 32))) return rc;
  PBF_HIP(hipMemcpyAsync(ctx->io0.p, points, n * 64, hipMemcpyHostToDevice, s));
  PBF_HIP(hipMemcpyAsync(ctx->io1.p, scalars, n * 32, hipMemcpyHostToDevice, s));
  MsmWork w = msm_work(ctx);
  if ((rc = msm_device(ctx, (const uint64_t*)ctx->io0.p, (const uint64_t*)ctx->io1.p, n, s, w))) return rc;
  std::vector<Xyzz> sums(MSM_NW);
  PBF_HIP(hipMemcpyAsync(sums.data(), w.sums.p, MSM_NW * sizeof(Xyzz), hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  msm_finish_host(sums.data(), out);
  return PBF_OK;
}

// device inputs; synchronous on `stream` (the final 16-window Horner runs on the host)
int pbf_msm_g1_bn254_dev(pbf_ctx* ctx, const uint64_t* d_points, const uint64_t* d_scalars, size_t n, uint64_t* out,
                         void* stream) {
  if (!ctx || !out || (n && (!d_points || !d_scalars))) return fail(PBF_EINVAL, "null argument");
  if (n == 0) { for (int i = 0; i < 8; ++i) out[i] = 0; return PBF_OK; }
  hipStream_t s = (hipStream_t)stream;
  MsmWork w = msm_work(ctx);
  int rc = msm_device(ctx, d_points, d_scalars, n, s, w);
  if (rc) return rc;
  if (ab_env("PBF_MSM_DEVICE_HORNER")) {  // A/B (PBF_AB build only)
    DevBuf& res = ctx->buf("msm.horner");
    if ((rc = res.ensure(sizeof(Xyzz)))) return rc;
    hipLaunchKernelGGL(msm_horner_kernel, dim3(1), dim3(64), 0, s, (const Xyzz*)w.sums.p, (Xyzz*)res.p);
    PBF_HIP(hipGetLastError());
    Xyzz r;
    PBF_HIP(hipMemcpyAsync(&r, res.p, sizeof(Xyzz), hipMemcpyDeviceToHost, s));
    PBF_HIP(hipStreamSynchronize(s));
    xyzz_to_affine_u64(r, out);
    return PBF_OK;
  }
  std::vector<Xyzz> sums(MSM_NW);
  PBF_HIP(hipMemcpyAsync(sums.data(), w.sums.p, MSM_NW * sizeof(Xyzz), hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  msm_finish_host(sums.data(), out);
  return PBF_OK;
}

// SRS::eval_at_s against a fixed base set (KZG commitments): the first call for a base set
// builds its window table (cached in the context, revalidated against a device copy of the
// points on every call)
int pbf_msm_g1_bn254_fixed_dev(pbf_ctx* ctx, const uint64_t* d_points, size_t n_points, const uint64_t* d_scalars,
                               size_t n, uint64_t* out, void* stream) {
  return pbf_msm_g1_bn254_fixed_range_dev(ctx, d_points, n_points, 0, d_scalars, n, out, stream);
}

// out = sum_{i<n} scalars[i] * points[first + i] against the fixed base set (one rank's point
// range of a sharded commitment)
int pbf_msm_g1_bn254_fixed_range_dev(pbf_ctx* ctx, const uint64_t* d_points, size_t n_points, size_t first,
                                     const uint64_t* d_scalars, size_t n, uint64_t* out, void* stream) {
  if (!ctx || !out || (n && (!d_points || !d_scalars))) return fail(PBF_EINVAL, "null argument");
  if (first > n_points || n > n_points - first) return fail(PBF_EINVAL, "scalar range beyond the base points");
  if (n == 0) { for (int i = 0; i < 8; ++i) out[i] = 0; return PBF_OK; }
  PBF_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  DevBuf& res = ctx->buf("msm.fixed_result");
  int rc = res.ensure(sizeof(Xyzz) + 8);
  if (rc) return rc;
  int* d_diff = (int*)((char*)res.p + sizeof(Xyzz));
  // Round 5: when the context's table was built from the current snapshot of these points, the
  // content check is enqueued and the MSM runs at once against that table; the result and the
  // check's flag come back together, and only a mismatch (the points changed in place) rebuilds
  // the table and runs again. This takes the check's host round trip (~30 us) off every call.
  const Affine* tbl = nullptr;
  {
    auto& fb = ctx->fixed_base;
    const FxGeom g = fx_geom_of(fx_default_c(ctx, n_points));
    auto w = ctx->snap_words.find("g1pts");
    if (fb.valid && fb.n == n_points && fb.c == g.c && fb.table.p && w != ctx->snap_words.end() &&
        w->second == 8 * n_points && ctx->snap_used["fx/g1pts"] == ctx->snap_gen["g1pts"]) {
      PBF_HIP(hipMemsetAsync(d_diff, 0, sizeof(int), s));
      uint64_t blocks = (8 * n_points + 255) / 256;
      if (blocks > 4096) blocks = 4096;
      hipLaunchKernelGGL(k_snap_compare, dim3((uint32_t)blocks), dim3(256), 0, s,
                         (const uint64_t*)ctx->buf("snap.g1pts").p, d_points, 8 * n_points, d_diff);
      PBF_HIP(hipGetLastError());
      tbl = (const Affine*)fb.table.p;
    }
  }
  for (int attempt = 0; attempt < 2; ++attempt) {
    const bool checked = tbl == nullptr;  // the table was (re)validated synchronously
    if (checked && (rc = msm_fixed_table(ctx, d_points, n_points, s, &tbl))) return rc;
    if ((rc = msm_fixed_device(ctx, tbl, n_points, first, d_scalars, n, s, (Xyzz*)res.p))) return rc;
    if ((rc = msm_fixed_wait(ctx, s))) return rc;
    struct {
      Xyzz r;
      int diff, pad;
    } h;
    PBF_HIP(hipMemcpyAsync(&h, res.p, sizeof(Xyzz) + (checked ? 0 : sizeof(int)), hipMemcpyDeviceToHost, s));
    PBF_HIP(hipStreamSynchronize(s));
    if (!checked && h.diff) {  // the points changed since the table was built: rebuild, run again
      tbl = nullptr;
      continue;
    }
    xyzz_to_affine_u64(h.r, out);
    return PBF_OK;
  }
  return fail(PBF_EDEVICE, "fixed-base MSM: table validation did not settle");
}

// out_i = scalars_i * G, affine canonical (device pointers), the SRS::create kernel
int pbf_g1_bn254_mul_base_dev(pbf_ctx* ctx, const uint64_t* d_scalars, uint64_t* d_out, size_t n, void* stream) {
  if (!ctx || (n && (!d_scalars || !d_out))) return fail(PBF_EINVAL, "null argument");
  if (n == 0) return PBF_OK;
  hipStream_t st = (hipStream_t)stream;
  const char* mb = ctx->options.get("g1.mul_base");
  if (mb && strcmp(mb, "daa") == 0) {  // option: cross-check of the comb (tests)
    hipLaunchKernelGGL(g1_mul_base_kernel, dim3(grid1(n)), dim3(256), 0, st, d_scalars, d_out, (uint64_t)n);
    PBF_HIP(hipGetLastError());
    return PBF_OK;
  }
  DevBuf& tbl = ctx->buf("g1.base_table");
  if (tbl.bytes == 0) {  // built once per context
    int rc = tbl.ensure((size_t)G1_TBL_W * G1_TBL_D * sizeof(Affine));
    if (rc) return rc;
    hipLaunchKernelGGL(g1_base_table_kernel, dim3((G1_TBL_W * G1_TBL_D + 255) / 256), dim3(256), 0, st,
                       (Affine*)tbl.p);
    PBF_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(g1_mul_base_comb, dim3(grid1(n)), dim3(256), 0, st, d_scalars, (const Affine*)tbl.p, d_out,
                     (uint64_t)n);
  PBF_HIP(hipGetLastError());
  return PBF_OK;
}

// SRS::create (plonk.rs:35-48): g1s = [G, G*s, G*s^2, ..., G*s^n] -> out has n+1 points
int pbf_srs_create_bn254(pbf_ctx* ctx, const uint64_t* s, size_t n, uint64_t* out) {
  if (!ctx || !s || !out) return fail(PBF_EINVAL, "null argument");
  if (!host_fr_canonical(s)) return fail(PBF_EINVAL, "s not canonical");
  PBF_HIP(hipSetDevice(ctx->device));
  std::vector<uint64_t> pw((n + 1) * 4);
  U256 sm;
  for (int i = 0; i < 4; ++i) { sm.w[2 * i] = (uint32_t)s[i]; sm.w[2 * i + 1] = (uint32_t)(s[i] >> 32); }
  sm = Fr::to_mont(sm);
  U256 acc = Fr::to_mont(Fr::one_plain());
  for (size_t i = 0; i <= n; ++i) {
    const U256 v = Fr::from_mont(acc);
    for (int k = 0; k < 4; ++k) pw[4 * i + k] = (uint64_t)v.w[2 * k] | ((uint64_t)v.w[2 * k + 1] << 32);
    acc = Fr::mul(acc, sm);
  }
  hipStream_t st = ctx->host_stream();
  int rc;
  if ((rc = ctx->io1.ensure((n + 1) * 32)) || (rc = ctx->io0.ensure((n + 1) * 64))) return rc;
  PBF_HIP(hipMemcpyAsync(ctx->io1.p, pw.data(), (n + 1) * 32, hipMemcpyHostToDevice, st));
  if ((rc = pbf_g1_bn254_mul_base_dev(ctx, (const uint64_t*)ctx->io1.p, (uint64_t*)ctx->io0.p, n + 1, st))) return rc;
  PBF_HIP(hipMemcpyAsync(out, ctx->io0.p, (n + 1) * 64, hipMemcpyDeviceToHost, st));
  PBF_HIP(hipStreamSynchronize(st));
  return PBF_OK;
}

}  // extern "C"
