// BN254 G1 multi-scalar multiplication (BASELINE config 4) and batch fixed-base
// multiplication — the MI355X replacements of SRS::eval_at_s (src/plonk.rs:51-58, a
// naive left fold of g1s[i] * gf(c_i), each a double-and-add, src/pbh/g1.rs:146-168)
// and SRS::create (src/plonk.rs:35-48, g1s[i] = G * s^i).
//
// MSM = Pippenger, window c = 16 (16 windows over the 254-bit scalars):
//   1. msm_digits: key = (window << 16) | digit per (point, window), digit 0 skipped
//   2. hipCUB radix sort of (key, point index) pairs  -> points grouped by bucket
//   3. msm_bucket_bounds: [start, end) of every bucket in the sorted order
//   4. msm_chunk_acc: the sorted list cut into fixed chunks of MSM_CH entries, one thread
//      per chunk accumulating its runs of equal keys in XYZZ (every thread does the same
//      number of additions whatever the bucket sizes); runs that cross a chunk boundary
//      leave partial sums, which msm_chunk_join adds up (one thread per bucket that starts
//      in a chunk and ends in a later one)
//   5. msm_segments + msm_window_reduce: per window, segments of 8 buckets; running sums
//      give sum (j-a+1) B_j and sum B_j per segment, + a * (segment sum); the segment
//      shares are summed by LDS trees over (window, part) workgroups, then per window
//   6. host: Horner over the 16 window sums (2^16 steps), one inversion to affine.
// The result is a group element, so the canonical affine output is unique.
#include <hipcub/hipcub.hpp>
#include <vector>
#include "../../include/pbf.h"
#include "ec_bn254.hpp"
#include "internal.hpp"

namespace pbf {

constexpr int MSM_C = 16;
constexpr int MSM_NW = 16;
// signed digits in [-2^15, 2^15]: bucket j of a window holds the points whose digit has
// |d| = j + 1 (negated for d < 0), so a window has 2^15 buckets
constexpr int MSM_BB = MSM_C - 1;                            // bucket-index bits
constexpr uint32_t MSM_NB = 1u << MSM_BB;                    // buckets per window
constexpr uint32_t MSM_SENTINEL = (uint32_t)MSM_NW << MSM_BB;  // sorts after every real key
constexpr uint32_t MSM_NEG = 0x80000000u;                    // sign flag in the point index
constexpr int MSM_SEG_THREADS = 256;

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

__global__ void msm_bucket_bounds(const uint32_t* keys, uint64_t m, uint32_t* start, uint32_t* end) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = keys[j];
    if (k == MSM_SENTINEL) continue;
    if (j == 0 || keys[j - 1] != k) start[k] = (uint32_t)j;
    if (j == m - 1 || keys[j + 1] != k) end[k] = (uint32_t)(j + 1);
  }
}

#ifndef PBF_MSM_CH
#define PBF_MSM_CH 32
#endif
#ifndef PBF_MSM_ACC_WPE
#define PBF_MSM_ACC_WPE 3
#endif
#ifndef PBF_MSM_SEG_WPE
#define PBF_MSM_SEG_WPE 1
#endif
constexpr uint32_t MSM_CH = PBF_MSM_CH;  // sorted entries per accumulation thread

struct ChunkPart {
  Xyzz acc;
  uint32_t key;  // MSM_SENTINEL: no partial
  uint32_t pad[3];
};

// Chunk t = entries [t*CH, (t+1)*CH) of the sorted list (m valid entries). Complete runs
// (the whole bucket inside the chunk) are written to their bucket. head[t]: the first run
// if its bucket started in an earlier chunk; tail[t]: the last run if its bucket starts in
// this chunk and ends in a later one. Buckets with no entry stay zero (ZZ = 0: identity).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PBF_MSM_ACC_WPE))) msm_chunk_acc(const Affine* pts, const uint32_t* keys, const uint32_t* vals,
                                                     const uint32_t* start, const uint32_t* end, uint32_t m,
                                                     Xyzz* buckets, ChunkPart* head, ChunkPart* tail) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c0 = t * MSM_CH;
  if (c0 >= m) return;
  const uint32_t c1 = c0 + MSM_CH < m ? c0 + MSM_CH : m;
  uint32_t cur = keys[c0], rs = c0;
  Xyzz acc = G1::identity();
  head[t].key = MSM_SENTINEL;
  tail[t].key = MSM_SENTINEL;
  if (cur == MSM_SENTINEL) return;  // past the valid prefix (zero digits sort last)
  auto flush = [&](uint32_t re) {
    const uint32_t bs = start[cur], be = end[cur];
    if (bs < rs) {  // continues a bucket of an earlier chunk (possibly spanning this one)
      head[t].acc = acc;
      head[t].key = cur;
    } else if (be > re) {  // starts here, ends in a later chunk
      tail[t].acc = acc;
      tail[t].key = cur;
    } else {
      buckets[cur] = acc;
    }
  };
  // the next entry's key, index and point are loaded while the current addition runs
  // (the point gathers are random: their latency would otherwise stall every step)
  uint32_t k_nx = cur, v_nx = vals[c0];
  Affine p_nx = pts[v_nx & ~MSM_NEG];
  for (uint32_t j = c0; j < c1; ++j) {
    const uint32_t k = k_nx, v = v_nx;
    Affine p = p_nx;
    if (j + 1 < c1) {
      k_nx = keys[j + 1];
      v_nx = vals[j + 1];
      p_nx = pts[v_nx & ~MSM_NEG];  // a sentinel entry's index is still a valid point
    }
    if (k != cur) {
      flush(j);
      if (k == MSM_SENTINEL) return;
      cur = k;
      rs = j;
      acc = G1::identity();
    }
    if (v & MSM_NEG) p.y = Fq::sub(u256_zero(), p.y);
    acc = G1::madd(acc, p);
  }
  flush(c1);
}

// one thread per chunk owning a boundary-crossing bucket: its tail plus the heads of the
// following chunks the bucket covers
__global__ void __launch_bounds__(256) msm_chunk_join(const ChunkPart* head, const ChunkPart* tail,
                                                      const uint32_t* end, uint32_t nchunks, Xyzz* buckets) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nchunks) return;
  const uint32_t k = tail[t].key;
  if (k == MSM_SENTINEL) return;
  Xyzz acc = tail[t].acc;
  const uint32_t be = end[k];
  for (uint32_t u = t + 1; u < nchunks && u * MSM_CH < be; ++u) acc = G1::add(acc, head[u].acc);
  buckets[k] = acc;
}

__device__ __forceinline__ Xyzz xyzz_neg(const Xyzz& p) {
  Xyzz r = p;
  r.Y = Fq::sub(u256_zero(), p.Y);
  return r;
}

// S_w = sum_j (j + 1) * B_{w,j}, in two launches. (a) one thread per (window, segment of
// MSM_SEG buckets starting at a): running sums give sum (j - a + 1) B_j and sum B_j, and
// the segment's share is wsum + a * running. (b) one workgroup per window sums its segment
// shares (sequential per thread, then an LDS tree).
#ifndef PBF_MSM_SEG
#define PBF_MSM_SEG 8
#endif
constexpr uint32_t MSM_SEG = PBF_MSM_SEG;
constexpr uint32_t MSM_NSEG = MSM_NB / MSM_SEG;

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PBF_MSM_SEG_WPE))) msm_segments(const Xyzz* buckets, Xyzz* shares) {
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= MSM_NW * MSM_NSEG) return;
  const uint32_t w = id / MSM_NSEG, seg = id % MSM_NSEG;
  const uint32_t a = seg * MSM_SEG;
  const Xyzz* B = buckets + (uint64_t)w * MSM_NB;
  Xyzz running = G1::identity(), wsum = G1::identity();
  for (int k = (int)(a + MSM_SEG - 1); k >= (int)a; --k) {
    running = G1::add(running, B[k]);
    wsum = G1::add(wsum, running);
  }
  shares[id] = (a == 0) ? wsum : G1::add(wsum, G1::mul_small(running, a));
}

// tree sum of `count` points (count <= MSM_SEG_THREADS) into out
__device__ __forceinline__ void msm_tree_sum(const Xyzz* in, uint32_t count, Xyzz* out) {
  __shared__ Xyzz red[MSM_SEG_THREADS];
  const uint32_t t = threadIdx.x;
  red[t] = t < count ? in[t] : G1::identity();
  __syncthreads();
  for (uint32_t st = MSM_SEG_THREADS / 2; st > 0; st >>= 1) {
    if (t < st) red[t] = G1::add(red[t], red[t + st]);
    __syncthreads();
  }
  if (t == 0) *out = red[0];
}
constexpr uint32_t MSM_NPART = MSM_NSEG / MSM_SEG_THREADS;  // partial sums per window
static_assert(MSM_NSEG % MSM_SEG_THREADS == 0 && MSM_NPART <= MSM_SEG_THREADS, "reduction shape");

// workgroup (window, part): the tree sum of MSM_SEG_THREADS segment shares
__global__ void __launch_bounds__(MSM_SEG_THREADS) msm_window_reduce(const Xyzz* shares, Xyzz* parts) {
  msm_tree_sum(shares + (uint64_t)blockIdx.x * MSM_SEG_THREADS, MSM_SEG_THREADS, parts + blockIdx.x);
}
// workgroup w: the window sum from its MSM_NPART partial sums
__global__ void __launch_bounds__(MSM_SEG_THREADS) msm_window_final(const Xyzz* parts, Xyzz* sums) {
  msm_tree_sum(parts + (uint64_t)blockIdx.x * MSM_NPART, MSM_NPART, sums + blockIdx.x);
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
  DevBuf &pts, &inf, &keys, &vals, &keys2, &vals2, &start, &end, &buckets, &shares, &sums, &temp, &head, &tail,
      &parts;
};

// scratch owned by the context (freed with it)
static MsmWork msm_work(pbf_ctx* ctx) {
  return MsmWork{ctx->buf("msm.pts"),     ctx->buf("msm.inf"),    ctx->buf("msm.keys"),   ctx->buf("msm.vals"),
                 ctx->buf("msm.keys2"),   ctx->buf("msm.vals2"),  ctx->buf("msm.start"),  ctx->buf("msm.end"),
                 ctx->buf("msm.buckets"), ctx->buf("msm.shares"), ctx->buf("msm.sums"),   ctx->buf("msm.temp"),
                 ctx->buf("msm.head"),    ctx->buf("msm.tail"),   ctx->buf("msm.parts")};
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
      (rc = w.shares.ensure((uint64_t)MSM_NW * MSM_NSEG * sizeof(Xyzz))) ||
      (rc = w.sums.ensure(MSM_NW * sizeof(Xyzz))) || (rc = w.parts.ensure(MSM_NW * MSM_NPART * sizeof(Xyzz))) ||
      (rc = w.head.ensure((m / MSM_CH + 1) * sizeof(ChunkPart))) ||
      (rc = w.tail.ensure((m / MSM_CH + 1) * sizeof(ChunkPart))))
    return rc;
  hipLaunchKernelGGL(msm_points_to_mont, dim3(grid1(n)), dim3(256), 0, s, d_pts, (Affine*)w.pts.p,
                     (uint8_t*)w.inf.p, n);
  hipLaunchKernelGGL(msm_digits, dim3(grid1(n)), dim3(256), 0, s, d_sc, (const uint8_t*)w.inf.p,
                     (uint32_t*)w.keys.p, (uint32_t*)w.vals.p, n);
  size_t temp_bytes = 0;
  PBF_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, (const uint32_t*)w.keys.p, (uint32_t*)w.keys2.p,
                                             (const uint32_t*)w.vals.p, (uint32_t*)w.vals2.p, (int)m, 0,
                                             MSM_BB + 5, s));
  if ((rc = w.temp.ensure(temp_bytes ? temp_bytes : 1))) return rc;
  PBF_HIP(hipcub::DeviceRadixSort::SortPairs(w.temp.p, temp_bytes, (const uint32_t*)w.keys.p, (uint32_t*)w.keys2.p,
                                             (const uint32_t*)w.vals.p, (uint32_t*)w.vals2.p, (int)m, 0,
                                             MSM_BB + 5, s));
  PBF_HIP(hipMemsetAsync(w.start.p, 0, (uint64_t)MSM_NW * MSM_NB * 4, s));
  PBF_HIP(hipMemsetAsync(w.end.p, 0, (uint64_t)MSM_NW * MSM_NB * 4, s));
  hipLaunchKernelGGL(msm_bucket_bounds, dim3(grid1(m)), dim3(256), 0, s, (const uint32_t*)w.keys2.p, m,
                     (uint32_t*)w.start.p, (uint32_t*)w.end.p);
  // the valid (non-sentinel) prefix of the sorted list: the sentinel sorts last; its
  // length is known only on the device, so chunks past it return at once
  PBF_HIP(hipMemsetAsync(w.buckets.p, 0, (uint64_t)MSM_NW * MSM_NB * sizeof(Xyzz), s));
  const uint32_t nchunks = (uint32_t)((m + MSM_CH - 1) / MSM_CH);
  hipLaunchKernelGGL(msm_chunk_acc, dim3((nchunks + 255) / 256), dim3(256), 0, s, (const Affine*)w.pts.p,
                     (const uint32_t*)w.keys2.p, (const uint32_t*)w.vals2.p, (const uint32_t*)w.start.p,
                     (const uint32_t*)w.end.p, (uint32_t)m, (Xyzz*)w.buckets.p, (ChunkPart*)w.head.p,
                     (ChunkPart*)w.tail.p);
  hipLaunchKernelGGL(msm_chunk_join, dim3((nchunks + 255) / 256), dim3(256), 0, s, (const ChunkPart*)w.head.p,
                     (const ChunkPart*)w.tail.p, (const uint32_t*)w.end.p, nchunks, (Xyzz*)w.buckets.p);
  hipLaunchKernelGGL(msm_segments, dim3((MSM_NW * MSM_NSEG + 255) / 256), dim3(256), 0, s, (const Xyzz*)w.buckets.p,
                     (Xyzz*)w.shares.p);
  hipLaunchKernelGGL(msm_window_reduce, dim3(MSM_NW * MSM_NPART), dim3(MSM_SEG_THREADS), 0, s,
                     (const Xyzz*)w.shares.p, (Xyzz*)w.parts.p);
  hipLaunchKernelGGL(msm_window_final, dim3(MSM_NW), dim3(MSM_SEG_THREADS), 0, s, (const Xyzz*)w.parts.p,
                     (Xyzz*)w.sums.p);
  PBF_HIP(hipGetLastError());
  return 0;
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
  std::vector<Xyzz> sums(MSM_NW);
  PBF_HIP(hipMemcpyAsync(sums.data(), w.sums.p, MSM_NW * sizeof(Xyzz), hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  msm_finish_host(sums.data(), out);
  return PBF_OK;
}

// out_i = scalars_i * G, affine canonical (device pointers), the SRS::create kernel
int pbf_g1_bn254_mul_base_dev(pbf_ctx* ctx, const uint64_t* d_scalars, uint64_t* d_out, size_t n, void* stream) {
  if (!ctx || (n && (!d_scalars || !d_out))) return fail(PBF_EINVAL, "null argument");
  if (n == 0) return PBF_OK;
  hipStream_t st = (hipStream_t)stream;
  if (getenv("PBF_G1_DOUBLE_AND_ADD")) {  // A/B and cross-check of the comb
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
