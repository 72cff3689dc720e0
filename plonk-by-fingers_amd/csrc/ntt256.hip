// BN254-Fr NTT and mul_ntt (BASELINE config 3: "Polynomial multiply via NTT,
// 256-bit scalar field, degree 2^22"). Same Stockham decomposition as the u64 path
// (ntt_kernels.hpp): P passes of radix R over HBM, an in-LDS Stockham of radix-2^LQ
// register sub-DFTs per workgroup; elements are 32 B, Montgomery form inside the
// kernels (canonical at the ABI: converted on the first pass's load and the last
// pass's store). Replaces fft.rs:66-78 and fft.rs:109-132 for the 256-bit field.
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>
#include "../../include/pbf.h"
#include "fp256.hpp"
#include "fr29.hpp"
#include "internal.hpp"

// Product form of the pass kernel's butterflies and twiddles: the single-chain Montgomery
// product (Fq/Fr::mul_tp: ~17 % fewer VALU per product, carry wait states left to the other
// waves of a SIMD) by default; -DPBF_NTT256_MUL2CH builds the two-chain form for A/B.
#ifdef PBF_NTT256_MUL2CH
#define PBF_FRMUL(a, b) Fr::mul(a, b)
#else
#define PBF_FRMUL(a, b) Fr::mul_tp(a, b)
#endif
namespace pbf {
using l29::L29;

struct Pass256 {
  const U256* in;
  U256* out;
  const U256* rtab;    // w_R^m (Montgomery), m < R
  const U256* twpass;  // [r][k] pass twiddles (Montgomery) or null
  const U256* tw0;     // two-level table (Montgomery)
  const U256* tw1;
  const U256* mul_by;  // last pass (Ns > 1) only, or null: outputs become mont(mul_by[i], y) (mul_ntt)
  U256 n_inv;          // Montgomery form
  uint64_t n;
  uint32_t log_n, log_ns, tw_bits, blocks_per_poly, batch;
  uint32_t conv_in, conv_out, scale;
};

__host__ __device__ constexpr int st_logq(int logr, int s, int lq) {
  return (logr % lq == 0) ? lq : (s == 0 ? logr % lq : lq);
}
__host__ __device__ constexpr int st_logl(int logr, int s, int lq) {
  int l = 0;
  for (int i = 0; i < s; ++i) l += st_logq(logr, i, lq);
  return l;
}
__host__ __device__ constexpr int st_count(int logr, int lq) { return (logr + lq - 1) / lq; }
__host__ __device__ constexpr int brev_c(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}

// In-register q-point DIF DFT (natural in, bit-reversed out), unrolled by templates.
template <int LOGQ, int H, int A>
__device__ __forceinline__ void dif256_row(U256* v, const U256* wq) {
  if constexpr (A < H) {
    constexpr int Q = 1 << LOGQ;
#pragma unroll
    for (int blk = 0; blk < Q; blk += 2 * H) {
      const U256 x = v[blk + A], y = v[blk + A + H];
      v[blk + A] = Fr::add(x, y);
      const U256 d = Fr::sub(x, y);
      if constexpr (A == 0) v[blk + A + H] = d;
      else v[blk + A + H] = PBF_FRMUL(d, wq[A * (Q / (2 * H))]);
    }
    dif256_row<LOGQ, H, A + 1>(v, wq);
  }
}
template <int LOGQ, int H>
__device__ __forceinline__ void dif256_levels(U256* v, const U256* wq) {
  if constexpr (H >= 1) {
    dif256_row<LOGQ, H, 0>(v, wq);
    dif256_levels<LOGQ, H / 2>(v, wq);
  }
}
template <int LOGQ>
__device__ __forceinline__ void dft_reg256(U256* v, const U256* wq) {
  dif256_levels<LOGQ, (1 << LOGQ) / 2>(v, wq);
}

template <int LOGR, int W, int NT, int LQ, int S>
__device__ __forceinline__ void stage256(U256* v, U256* lds, const U256* wq, const Pass256& a, const U256* in,
                                         U256* out, uint64_t j0, int t) {
  constexpr int R = 1 << LOGR;
  constexpr int PER = (R * W) / NT;
  constexpr int NST = st_count(LOGR, LQ);
  constexpr int LOGQ = st_logq(LOGR, S, LQ);
  constexpr int Q = 1 << LOGQ;
  constexpr int L = 1 << st_logl(LOGR, S, LQ);
  constexpr int NSUB = PER / Q;
  constexpr int QMAX = 1 << LQ;
  constexpr bool LAST = (S == NST - 1);
  if constexpr (S == 0) {
    // raw loads first (simple body: fully unrolled, v stays in registers)
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      const int sub = t + NT * u;
      const int w = sub % W, i = sub / W;
#pragma unroll
      for (int c = 0; c < Q; ++c) v[u * Q + c] = in[(j0 + w) + (uint64_t)(i + c * (R / Q)) * (a.n >> LOGR)];
    }
    if (a.conv_in) {
#pragma unroll
      for (int e = 0; e < PER; ++e) v[e] = Fr::to_mont(v[e]);
    }
    if (a.log_ns > 0) {
      U256 tw[PER];
      if (a.twpass) {
#pragma unroll
        for (int e = 0; e < PER; ++e) {
          const int sub = t + NT * (e / Q);
          const uint64_t k = (j0 + sub % W) & ((1ull << a.log_ns) - 1);
          const uint64_t r = (uint64_t)(sub / W + (e % Q) * (R / Q));
          tw[e] = a.twpass[(r << a.log_ns) + k];
        }
      } else {
#pragma unroll
        for (int e = 0; e < PER; ++e) {
          const int sub = t + NT * (e / Q);
          const uint64_t k = (j0 + sub % W) & ((1ull << a.log_ns) - 1);
          const uint64_t r = (uint64_t)(sub / W + (e % Q) * (R / Q));
          const uint64_t x = ((r * k) << (a.log_n - a.log_ns - LOGR)) & (a.n - 1);
          tw[e] = Fr::mul(a.tw0[x & ((1ull << a.tw_bits) - 1)], a.tw1[x >> a.tw_bits]);
        }
      }
#pragma unroll
      for (int e = 0; e < PER; ++e) v[e] = PBF_FRMUL(v[e], tw[e]);
    }
  } else {
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      const int sub = t + NT * u;
      const int w = sub % W, i = sub / W;
      const int k = i % L;
#pragma unroll
      for (int c = 0; c < Q; ++c) {
        const int r = i + c * (R / Q);
        U256 x = lds[r * W + w];
        if (c != 0 && k != 0) x = PBF_FRMUL(x, a.rtab[(R / (L * Q)) * c * k]);
        v[u * Q + c] = x;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < NSUB; ++u) {
    U256 wl[Q / 2 > 0 ? Q / 2 : 1];
#pragma unroll
    for (int m = 0; m < Q / 2; ++m) wl[m] = wq[m * (QMAX / Q)];
    dft_reg256<LOGQ>(v + u * Q, wl);
  }
  if constexpr (S > 0) __syncthreads();
#pragma unroll
  for (int u = 0; u < NSUB; ++u) {
    const int sub = t + NT * u;
    const int w = sub % W, i = sub / W;
    const int k = i % L;
#pragma unroll
    for (int d = 0; d < Q; ++d) {
      U256 y = v[u * Q + brev_c(d, LOGQ)];
      const int r = (i / L) * L * Q + k + d * L;
      if constexpr (!LAST) {
        lds[r * W + w] = y;
      } else {
        if (a.scale) y = Fr::mul(y, a.n_inv);
        if (a.conv_out) y = Fr::from_mont(y);
        if (a.log_ns == 0) {
          lds[w * (R + 1) + r] = y;
        } else {
          const uint64_t j = j0 + w;
          const uint64_t msk = (1ull << a.log_ns) - 1;
          const uint64_t o = ((j >> a.log_ns) << (a.log_ns + LOGR)) + (j & msk) + ((uint64_t)r << a.log_ns);
          if (a.mul_by) y = PBF_FRMUL(a.mul_by[(out - a.out) + o], y);  // same element: read, then written
          out[o] = y;
        }
      }
    }
  }
  if constexpr (!LAST) {
    __syncthreads();
    stage256<LOGR, W, NT, LQ, S + 1>(v, lds, wq, a, in, out, j0, t);
  }
}

template <int LOGR, int W, int NT, int LQ>
#ifndef PBF_NTT256_WPE
#define PBF_NTT256_WPE 4
#endif
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(PBF_NTT256_WPE))) ntt256_pass_kernel(Pass256 a) {
  constexpr int R = 1 << LOGR;
  constexpr int E = R * W;
  constexpr int PER = E / NT;
  constexpr int QMAX = 1 << LQ;
  static_assert(PER % QMAX == 0 && LOGR >= LQ, "bad shape");
  __shared__ U256 lds[E + W];
  const uint32_t poly = blockIdx.x / a.blocks_per_poly;
  const uint64_t j0 = (uint64_t)(blockIdx.x % a.blocks_per_poly) * W;
  const U256* in = a.in + (uint64_t)poly * a.n;
  U256* out = a.out + (uint64_t)poly * a.n;
  const int t = threadIdx.x;
  U256 wq[QMAX / 2];
#pragma unroll
  for (int m = 0; m < QMAX / 2; ++m) wq[m] = a.rtab[m * (R / QMAX)];
  U256 v[PER];
  stage256<LOGR, W, NT, LQ, 0>(v, lds, wq, a, in, out, j0, t);
  if (a.log_ns == 0) {
    __syncthreads();
    U256* o = out + j0 * R;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int m = t + NT * u;
      o[m] = lds[(m / R) * (R + 1) + (m % R)];
    }
  }
}

// ---- The same passes on nine 29-bit limbs (round 6, fr29.hpp): ntt256l_pass_kernel. Same
// Stockham shape, tile, tables and element order as ntt256_pass_kernel; the elements stay in
// lazily reduced 29-bit limbs from the pass's loads to its stores (36 B in LDS), every table
// holds w 2^261 mod r in limbs (Pass256L), and the stores are canonical again, so both kernels
// write the same integers. Bounds of every step: fr29.hpp, tests/test_fr29_bounds.py.
struct Pass256L {
  const U256* in;
  U256* out;
  const L29* rtab;    // w_R^m 2^261
  const L29* twpass;  // [r][k] pass twiddles 2^261 (n^-1 folded into the inverse's last pass) or null
  const L29* tw0;     // two-level tables 2^261 (tw1: tw1s for the inverse's last pass)
  const L29* tw1;
  const U256* mul_by;  // last pass only, or null: outputs become mul_by[i] y 2^-256 (mul_ntt)
  uint64_t n;
  uint64_t in_len;     // first pass: input elements at index >= in_len read as zero (not loaded)
  uint32_t log_n, log_ns, tw_bits, blocks_per_poly, batch;
};

// radix-4 DIF in registers (natural in, bit-reversed out; dif256_row's order): inputs normalised
// below 2.05 r, outputs below 12.1 r with limbs below 2^32 (fr29.hpp)
__device__ __forceinline__ void dft4_29(L29* v, const L29& w4) {
  const L29 n0 = fr29::add(v[0], v[2]);
  const L29 n2 = fr29::sub(v[0], v[2], fr29::B4R);
  const L29 n1 = fr29::add(v[1], v[3]);
  const L29 n3 = fr29::mul(fr29::sub(v[1], v[3], fr29::B4R), w4);
  v[0] = fr29::add(n0, n1);
  v[1] = fr29::sub(n0, n1, fr29::B8R);
  v[2] = fr29::add(n2, n3);
  v[3] = fr29::sub(n2, n3, fr29::B2R);
}
__device__ __forceinline__ void dft2_29(L29* v) {
  const L29 a = fr29::add(v[0], v[1]);
  v[1] = fr29::sub(v[0], v[1], fr29::B4R);
  v[0] = a;
}

// An element in LDS: limbs 0..7 as one 16-B aligned 32-B word (two 128-bit LDS accesses) and limb 8
// in an array of its own (36 B per element, as two workgroups per CU need)
struct alignas(16) L8 {
  uint32_t l[8];
};
struct Lds29 {
  L8* lo;
  uint32_t* hi;
  __device__ __forceinline__ L29 ld(int i) const {
    const L8 a = lo[i];
    L29 r;
#pragma unroll
    for (int k = 0; k < 8; ++k) r.l[k] = a.l[k];
    r.l[8] = hi[i];
    return r;
  }
  __device__ __forceinline__ void st(int i, const L29& x) const {
    L8 a;
#pragma unroll
    for (int k = 0; k < 8; ++k) a.l[k] = x.l[k];
    lo[i] = a;
    hi[i] = x.l[8];
  }
};

template <int E, int N, typename F>
__device__ __forceinline__ void unroll_each(F&& f) {
  if constexpr (E < N) {
    f(std::integral_constant<int, E>{});
    unroll_each<E + 1, N>(f);
  }
}

template <int LOGR, int W, int NT, int LQ, int S>
__device__ __forceinline__ void stage29(L29* v, const Lds29& lds, const Pass256L& a, const U256* in, U256* out,
                                        uint64_t j0, int t) {
  constexpr int R = 1 << LOGR;
  constexpr int PER = (R * W) / NT;
  constexpr int NST = st_count(LOGR, LQ);
  constexpr int LOGQ = st_logq(LOGR, S, LQ);
  constexpr int Q = 1 << LOGQ;
  constexpr int L = 1 << st_logl(LOGR, S, LQ);
  constexpr int NSUB = PER / Q;
  constexpr bool LAST = (S == NST - 1);
  static_assert(LQ == 2 && (Q == 2 || Q == 4), "radix-4 register sub-DFTs");
  if constexpr (S == 0) {
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      const int sub = t + NT * u;
      const int w = sub % W, i = sub / W;
#pragma unroll
      for (int c = 0; c < Q; ++c) {
        const uint64_t e = (j0 + w) + (uint64_t)(i + c * (R / Q)) * (a.n >> LOGR);
        v[u * Q + c] = e < a.in_len ? l29::from_u256(in[e]) : L29{};
      }
    }
    // the pass twiddle, one element at a time (a table of 4 limb twiddles would not fit beside v)
    // (compile-time element indices: the loop vectoriser had turned a plain loop here into one
    // over v in scratch memory)
    if (a.log_ns > 0 && a.twpass) {
      unroll_each<0, PER>([&](auto ec) {
        constexpr int e = decltype(ec)::value;
        const int sub = t + NT * (e / Q);
        const uint64_t k = (j0 + sub % W) & ((1ull << a.log_ns) - 1);
        const uint64_t r = (uint64_t)(sub / W + (e % Q) * (R / Q));
        v[e] = fr29::mul(v[e], a.twpass[(r << a.log_ns) + k]);
        __builtin_amdgcn_sched_barrier(0);  // one twiddle's loads and product at a time (VGPRs)
      });
    } else if (a.log_ns > 0) {
      unroll_each<0, PER>([&](auto ec) {
        constexpr int e = decltype(ec)::value;
        const int sub = t + NT * (e / Q);
        const uint64_t k = (j0 + sub % W) & ((1ull << a.log_ns) - 1);
        const uint64_t r = (uint64_t)(sub / W + (e % Q) * (R / Q));
        const uint64_t x = ((r * k) << (a.log_n - a.log_ns - LOGR)) & (a.n - 1);
        v[e] = fr29::mul(v[e], fr29::mul(a.tw0[x & ((1ull << a.tw_bits) - 1)], a.tw1[x >> a.tw_bits]));
        __builtin_amdgcn_sched_barrier(0);
      });
    }
  } else {
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      const int sub = t + NT * u;
      const int w = sub % W, i = sub / W;
      const int k = i % L;
#pragma unroll
      for (int c = 0; c < Q; ++c) {
        const int r = i + c * (R / Q);
        // the previous stage stored its outputs unreduced: the inter-stage twiddle's product
        // (w^0 = 2^261 included, where k = 0) or, for c = 0, reduce() bounds them again
        const L29 x = lds.ld(r * W + w);
        v[u * Q + c] = c != 0 ? fr29::mul(x, a.rtab[(R / (L * Q)) * c * k]) : fr29::reduce(x);
        __builtin_amdgcn_sched_barrier(0);  // one element's load and product at a time (VGPRs)
      }
    }
  }
  if constexpr (Q == 4) {
    const L29 w4 = a.rtab[R / 4];  // uniform: read per stage (scalar loads), not held in VGPRs
#pragma unroll
    for (int u = 0; u < NSUB; ++u) dft4_29(v + u * Q, w4);
  } else {
#pragma unroll
    for (int u = 0; u < NSUB; ++u) dft2_29(v + u * Q);
  }
  if constexpr (S > 0) __syncthreads();
#pragma unroll
  for (int u = 0; u < NSUB; ++u) {
    const int sub = t + NT * u;
    const int w = sub % W, i = sub / W;
    const int k = i % L;
#pragma unroll
    for (int d = 0; d < Q; ++d) {
      const int r = (i / L) * L * Q + k + d * L;
      if constexpr (!LAST) {
        lds.st(r * W + w, v[u * Q + brev_c(d, LOGQ)]);
        continue;
      }
      const L29 y = fr29::reduce(v[u * Q + brev_c(d, LOGQ)]);
      if (a.log_ns == 0) {
        reinterpret_cast<U256*>(lds.lo)[w * (R + 1) + r] = fr29::canon(y);
      } else {
        const uint64_t j = j0 + w;
        const uint64_t msk = (1ull << a.log_ns) - 1;
        const uint64_t o = ((j >> a.log_ns) << (a.log_ns + LOGR)) + (j & msk) + ((uint64_t)r << a.log_ns);
        // mul_ntt's product as in ntt256_pass_kernel (mul_by y 2^-256: the extra-R inverse plans
        // serve both kernels); the same element is read, then written
        const U256 c = fr29::canon(y);
        out[o] = a.mul_by ? Fr::mul_tp(a.mul_by[(out - a.out) + o], c) : c;
      }
    }
  }
  if constexpr (!LAST) {
    __syncthreads();
    stage29<LOGR, W, NT, LQ, S + 1>(v, lds, a, in, out, j0, t);
  }
}

template <int LOGR, int W, int NT, int LQ>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT * 2 >= 1024 ? 4 : 3))) ntt256l_pass_kernel(Pass256L a) {
  constexpr int R = 1 << LOGR;
  constexpr int E = R * W;
  constexpr int PER = E / NT;
  static_assert(PER % 4 == 0 && LOGR >= LQ, "bad shape");
  __shared__ L8 lds_lo[E + W];  // also the last stage's U256 transpose tile (E + W elements)
  __shared__ uint32_t lds_hi[E + W];
  const Lds29 lds{lds_lo, lds_hi};
  const uint32_t poly = blockIdx.x / a.blocks_per_poly;
  const uint64_t j0 = (uint64_t)(blockIdx.x % a.blocks_per_poly) * W;
  const U256* in = a.in + (uint64_t)poly * a.n;
  U256* out = a.out + (uint64_t)poly * a.n;
  const int t = threadIdx.x;
  L29 v[PER];
  stage29<LOGR, W, NT, LQ, 0>(v, lds, a, in, out, j0, t);
  if (a.log_ns == 0) {
    __syncthreads();
    U256* o = out + j0 * R;
    const U256* l = reinterpret_cast<const U256*>(lds_lo);
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int m = t + NT * u;
      o[m] = l[(m / R) * (R + 1) + (m % R)];
    }
  }
}

// table conversion: out[i] = in[i] 2^5 (in: w 2^256 mod r, canonical) in 29-bit limbs = w 2^261
__global__ void tw256_to29_kernel(const U256* in, L29* out, uint64_t count, U256 c32m) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = l29::from_u256(Fr::mul(in[i], c32m));
}

// Whole transform for n <= 2048 in one workgroup (bit-reversed load, radix-2 DIT).
__global__ void __launch_bounds__(256) ntt256_small_kernel(const U256* in, U256* out, const U256* tw, uint32_t logn,
                                                           U256 n_inv, uint32_t scale) {
  __shared__ U256 lds[2048];
  const uint32_t n = 1u << logn;
  const U256* src = in + (uint64_t)blockIdx.x * n;
  U256* dst = out + (uint64_t)blockIdx.x * n;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t r = logn ? (__brev(i) >> (32 - logn)) : 0;
    lds[r] = Fr::to_mont(src[i]);
  }
  __syncthreads();
  for (uint32_t len = 2; len <= n; len <<= 1) {
    const uint32_t half = len >> 1;
    for (uint32_t b = threadIdx.x; b < n / 2; b += blockDim.x) {
      const uint32_t grp = b / half, k = b % half;
      const uint32_t i0 = grp * len + k, i1 = i0 + half;
      const U256 x = lds[i0], y = Fr::mul(lds[i1], tw[(uint64_t)k * (n / len)]);
      lds[i0] = Fr::add(x, y);
      lds[i1] = Fr::sub(x, y);
    }
    __syncthreads();
  }
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    U256 y = lds[i];
    if (scale) y = Fr::mul(y, n_inv);
    dst[i] = Fr::from_mont(y);
  }
}

// Plan-time fill of a per-pass twiddle table T[r][k] = w^(r k n / (Ns R)), r < R, k < Ns, from
// the two-level tables: the values the pass kernel's two-level branch computes per element
// (one Fr product each) computed once instead.
__global__ void tw256_fill_kernel(U256* t, const U256* tw0, const U256* tw1, uint32_t log_n, uint32_t log_ns,
                                  uint32_t logr, uint32_t tw_bits) {
  const uint64_t count = 1ull << (log_ns + logr), n = 1ull << log_n;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = i >> log_ns, k = i & ((1ull << log_ns) - 1);
    const uint64_t x = ((r * k) << (log_n - log_ns - logr)) & (n - 1);
    t[i] = Fr::mul(tw0[x & ((1ull << tw_bits) - 1)], tw1[x >> tw_bits]);
  }
}

// c = a b / R for canonical a, b (one Montgomery product); the inverse transform that follows
// (a get_plan256(..., extra_r) plan) puts the R back
__global__ void pointwise_mont256_kernel(const U256* a, const U256* b, U256* c, uint64_t count) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
    c[i] = Fr::mul_tp(a[i], b[i]);
}

__global__ void pointwise_mul256_kernel(const U256* a, const U256* b, U256* c, uint64_t count) {
  // inputs canonical; mont(a)*b = a*b*R*R^-1 = a*b canonical in one product
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
    c[i] = Fr::mul(Fr::to_mont(a[i]), b[i]);
}

// ---------------------------------------------------------------- host side
static U256 h_from64(const uint64_t* x) {
  U256 r;
  for (int i = 0; i < 4; ++i) { r.w[2 * i] = (uint32_t)x[i]; r.w[2 * i + 1] = (uint32_t)(x[i] >> 32); }
  return r;
}
static bool h_canonical(const U256& x) { return !Fr::geq_p(x); }
static U256 h_pow(U256 base_m, uint64_t e) {  // Montgomery in/out
  U256 r = Fr::to_mont(Fr::one_plain());
  while (e) {
    if (e & 1) r = Fr::mul(r, base_m);
    base_m = Fr::mul(base_m, base_m);
    e >>= 1;
  }
  return r;
}
static U256 h_inv(const U256& a_m) {  // a^(r-2), Montgomery
  // exponent r - 2 as 8 limbs, square-and-multiply from the top
  uint32_t e[8];
  for (int i = 0; i < 8; ++i) e[i] = Bn254FrParams::P[i];
  e[0] -= 2;  // P[0] = 0xf0000001 >= 2
  U256 r = Fr::to_mont(Fr::one_plain());
  for (int i = 255; i >= 0; --i) {
    r = Fr::mul(r, r);
    if ((e[i / 32] >> (i % 32)) & 1) r = Fr::mul(r, a_m);
  }
  return r;
}

struct Plan256 {
  uint64_t n = 0;
  uint32_t log_n = 0;
  int inverse = 0;
  std::vector<int> logr;
  uint32_t tw_bits = 0;
  U256 n_inv{};
  bool fold_scale = false;  // inverse: n^-1 folded into the last pass's twiddles (tw1s / its table)
  DevBuf small_tw, tw0, tw1, tw1s;
  std::vector<std::shared_ptr<DevBuf>> rtab, twpass;
  // the 29-bit-limb passes (option ntt256.l29, default on; multi-pass plans with the scale folded):
  // the same tables as w 2^261 in limbs
  bool l29 = false;
  DevBuf tw0_29, tw1_29, tw1s_29;
  std::vector<std::shared_ptr<DevBuf>> rtab29, twpass29;
};

// in (count U256 Montgomery values w 2^256) -> out (count L29 values w 2^261)
static int to29(const DevBuf& in, DevBuf& out, uint64_t count) {
  if (!count) return 0;
  int rc = out.ensure(count * sizeof(L29));
  if (rc) return rc;
  U256 c32 = Fr::one_plain();
  c32.w[0] = 32;
  uint64_t blocks = (count + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(tw256_to29_kernel, dim3((uint32_t)blocks), dim3(256), 0, 0, (const U256*)in.p, (L29*)out.p, count,
                     Fr::to_mont(c32));
  PBF_HIP(hipGetLastError());
  return 0;
}

static int up256(DevBuf& b, const std::vector<U256>& v) {
  int rc = b.ensure(v.size() * sizeof(U256));
  if (rc) return rc;
  PBF_HIP(hipMemcpy(b.p, v.data(), v.size() * sizeof(U256), hipMemcpyHostToDevice));
  return 0;
}

static std::vector<U256> h_powers(const U256& w_m, uint64_t count) {
  std::vector<U256> t(count);
  U256 x = Fr::to_mont(Fr::one_plain());
  for (uint64_t i = 0; i < count; ++i) { t[i] = x; x = Fr::mul(x, w_m); }
  return t;
}

static int make_plan256(const pbf::Options& o, const uint64_t* omega, uint64_t n, int inverse, Plan256* p) {
  if (n == 0 || (n & (n - 1))) return fail(PBF_EINVAL, "n must be a power of two");
  uint32_t log_n = 0;
  while ((1ull << log_n) < n) ++log_n;
  if (log_n > 28) return fail(PBF_EINVAL, "n exceeds the 2-adicity of BN254 Fr (2^28)");
  U256 w = h_from64(omega);
  if (!h_canonical(w)) return fail(PBF_EINVAL, "omega not canonical");
  U256 wm = Fr::to_mont(w);
  const U256 one_m = Fr::to_mont(Fr::one_plain());
  if (n > 1 && (!Fr::eq(h_pow(wm, n), one_m) || Fr::eq(h_pow(wm, n / 2), one_m)))
    return fail(PBF_EINVAL, "omega does not have order n");
  p->n = n; p->log_n = log_n; p->inverse = inverse;
  U256 nm;
  {
    U256 nn = Fr::one_plain();
    nn.w[0] = (uint32_t)n; nn.w[1] = (uint32_t)(n >> 32);
    nm = Fr::to_mont(nn);
  }
  p->n_inv = h_inv(nm);
  if (inverse == 2) p->n_inv = Fr::mul(p->n_inv, Fr::to_mont(Fr::to_mont(Fr::one_plain())));  // n^-1 R
  if (inverse) wm = h_inv(wm);
  if (n <= 2048) return up256(p->small_tw, h_powers(wm, n));
  // passes of radix <= 2^9 (LDS tile 2048 x 32 B); option ntt256.maxr (4..9) lowers the largest
  // radix (more, lighter passes: every radix family of the planner, tests/test_ntt_fr256_gpu.py)
  int maxr = 9;
  if (const char* e = o.get("ntt256.maxr")) maxr = atoi(e) < 4 ? 4 : (atoi(e) > 9 ? 9 : atoi(e));
  const int P = (log_n + maxr - 1) / maxr;
  p->logr.assign(P, log_n / P);
  for (int i = 0; i < (int)(log_n % P); ++i) p->logr[i] += 1;
  p->tw_bits = (log_n + 1) / 2;
  int rc = up256(p->tw0, h_powers(wm, 1ull << p->tw_bits));
  if (rc) return rc;
  // The inverse's n^-1 rides in its last pass's twiddles (every element of a pass with Ns > 1
  // takes one twiddle product, and the pass is linear): tw1s = tw1 n^-1 for the two-level form,
  // the per-pass table scaled likewise; PBF_NTT256_SCALE_PASS=1 keeps the separate product (A/B).
  p->fold_scale = inverse && !ab_env("PBF_NTT256_SCALE_PASS");
  {
    const U256 step = h_pow(wm, 1ull << p->tw_bits);
    std::vector<U256> t1 = h_powers(step, n >> p->tw_bits);
    rc = up256(p->tw1, t1);
    if (rc) return rc;
    if (p->fold_scale) {
      for (auto& x : t1) x = Fr::mul(x, p->n_inv);
      if ((rc = up256(p->tw1s, t1))) return rc;
    }
  }
  // per-pass tables up to 2^tw_log entries (32 B each); larger passes fall back to the two-level
  // tables (one extra Fr product per element). Tables past 2^20 entries are filled on the device.
  int tw_log = 26;  // option ntt256.twlog: the two-level path of larger passes at test sizes
  if (const char* e = o.get("ntt256.twlog")) tw_log = atoi(e) < 0 ? 0 : (atoi(e) > 30 ? 30 : atoi(e));
  uint64_t ns = 1;
  uint32_t log_ns = 0;
  for (size_t pi = 0; pi < p->logr.size(); ++pi) {
    const int lr = p->logr[pi];
    const uint64_t R = 1ull << lr;
    const bool fold = p->fold_scale && pi + 1 == p->logr.size();
    auto rb = std::make_shared<DevBuf>();
    if ((rc = up256(*rb, h_powers(h_pow(wm, n / R), R)))) return rc;
    p->rtab.push_back(rb);
    auto tb = std::make_shared<DevBuf>();
    if (ns > 1 && R * ns > (1ull << 20) && tw_log > 20 && R * ns <= (1ull << tw_log)) {
      if ((rc = tb->ensure(R * ns * sizeof(U256)))) return rc;
      hipLaunchKernelGGL(tw256_fill_kernel, dim3(2048), dim3(256), 0, 0, (U256*)tb->p, (const U256*)p->tw0.p,
                         (const U256*)(fold ? p->tw1s.p : p->tw1.p), log_n, log_ns, (uint32_t)lr, p->tw_bits);
      PBF_HIP(hipGetLastError());
      PBF_HIP(hipStreamSynchronize(0));
    } else if (ns > 1 && R * ns <= (1ull << 20)) {
      const uint64_t step = n / (ns * R);
      std::vector<U256> t(R * ns);
      for (uint64_t r = 0; r < R; ++r) {
        const U256 wr = h_pow(wm, step * r);
        U256 z = one_m;
        for (uint64_t k = 0; k < ns; ++k) { t[r * ns + k] = fold ? Fr::mul(z, p->n_inv) : z; z = Fr::mul(z, wr); }
      }
      if ((rc = up256(*tb, t))) return rc;
    }
    p->twpass.push_back(tb);
    ns *= R;
    log_ns += lr;
  }
  // the 29-bit-limb passes' tables (ntt256l_pass_kernel; PBF_NTT256_SCALE_PASS / CONV, A/B
  // builds only, keep the 32-bit kernel). A converted per-pass table replaces its 32-bit form.
  p->l29 = o.num("ntt256.l29", 1) != 0 && p->fold_scale == (inverse != 0) && !ab_env("PBF_NTT256_CONV");
  if (p->l29) {
    const uint64_t nlo = 1ull << p->tw_bits, nhi = n >> p->tw_bits;
    if ((rc = to29(p->tw0, p->tw0_29, nlo)) || (rc = to29(p->tw1, p->tw1_29, nhi)) ||
        (p->fold_scale && (rc = to29(p->tw1s, p->tw1s_29, nhi))))
      return rc;
    ns = 1;
    for (size_t pi = 0; pi < p->logr.size(); ++pi) {
      const uint64_t R = 1ull << p->logr[pi];
      auto rb = std::make_shared<DevBuf>(), tb = std::make_shared<DevBuf>();
      if ((rc = to29(*p->rtab[pi], *rb, R))) return rc;
      if (p->twpass[pi]->p) {
        if ((rc = to29(*p->twpass[pi], *tb, R * ns))) return rc;
        PBF_HIP(hipStreamSynchronize(0));
        p->twpass[pi]->release();
      }
      p->rtab29.push_back(rb);
      p->twpass29.push_back(tb);
      ns *= R;
    }
    PBF_HIP(hipStreamSynchronize(0));
  }
  return 0;
}

typedef void (*Pass256Fn)(Pass256);
static int cols256(int logr) { return (2048 >> logr) > 64 ? 64 : (2048 >> logr); }
static Pass256Fn pass256_fn(int logr) {
  switch (logr) {  // W = min(64, 2048 / R), radix-4 register sub-DFTs, 4 elements per thread
    case 4: return ntt256_pass_kernel<4, 64, 256, 2>;
    case 5: return ntt256_pass_kernel<5, 64, 512, 2>;
    case 6: return ntt256_pass_kernel<6, 32, 512, 2>;
    case 7: return ntt256_pass_kernel<7, 16, 512, 2>;
    case 8: return ntt256_pass_kernel<8, 8, 512, 2>;
    case 9: return ntt256_pass_kernel<9, 4, 512, 2>;
    default: return nullptr;
  }
}
static int threads256(int logr) { return ((cols256(logr) << logr) / 4); }
// the 29-bit passes: radix 2^4..2^8 with half the columns per workgroup (half the threads, 4
// elements each: three workgroups of 4 waves per CU at up to 168 VGPRs), radix 2^9 with the full
// tile at 4 waves per SIMD (config 3, 8 + 8 + 7: 3.11 -> 3.04 ms; 4 x 2^26, 9 + 9 + 8: 36.5
// against 37.3 ms with every radix halved; profiles/r06/fr29_ab_c.log)
static int cols256l(int logr) { return logr == 9 ? cols256(logr) : cols256(logr) / 2; }
static int threads256l(int logr) { return ((cols256l(logr) << logr) / 4); }
typedef void (*Pass256LFn)(Pass256L);
static Pass256LFn pass256l_fn(int logr) {
  switch (logr) {  // the shapes of pass256_fn
    case 4: return ntt256l_pass_kernel<4, 32, 128, 2>;
    case 5: return ntt256l_pass_kernel<5, 32, 256, 2>;
    case 6: return ntt256l_pass_kernel<6, 16, 256, 2>;
    case 7: return ntt256l_pass_kernel<7, 8, 256, 2>;
    case 8: return ntt256l_pass_kernel<8, 4, 256, 2>;
    case 9: return ntt256l_pass_kernel<9, 4, 512, 2>;
    default: return nullptr;
  }
}

// mul_by (not for n <= 2048): the last pass multiplies its outputs by mul_by's elements (one
// Montgomery product: mont(m, y) = m y / R) -- mul_ntt's pointwise product fused into the second
// operand's forward transform
static int run256(const Plan256& p, const U256* d_in, U256* d_out, size_t batch, DevBuf& s0, DevBuf& s1,
                  hipStream_t st, const U256* mul_by = nullptr, uint64_t in_len = 0) {
  if (batch == 0) return 0;
  if (p.n == 1) {
    if (d_in != d_out) PBF_HIP(hipMemcpyAsync(d_out, d_in, batch * sizeof(U256), hipMemcpyDeviceToDevice, st));
    return 0;
  }
  if (p.logr.empty()) {
    if (mul_by) return fail(PBF_EINVAL, "fused product needs a multi-pass transform");
    hipLaunchKernelGGL(ntt256_small_kernel, dim3(batch), dim3(256), 0, st, d_in, d_out,
                       (const U256*)p.small_tw.p, p.log_n, p.n_inv, (uint32_t)p.inverse);
    PBF_HIP(hipGetLastError());
    return 0;
  }
  const size_t P = p.logr.size();
  const size_t bytes = batch * p.n * sizeof(U256);
  int rc = s0.ensure(bytes);
  if (!rc && P > 2) rc = s1.ensure(bytes);
  if (rc) return rc;
  uint32_t log_ns = 0;
  if (p.l29) {
    for (size_t i = 0; i < P; ++i) {
      const int lr = p.logr[i];
      const int W = cols256l(lr);
      Pass256L a;
      a.in = (i == 0) ? d_in : (const U256*)(((i - 1) & 1) ? s1.p : s0.p);
      a.out = (i == P - 1) ? d_out : (U256*)((i & 1) ? s1.p : s0.p);
      a.rtab = (const L29*)p.rtab29[i]->p;
      a.twpass = (const L29*)p.twpass29[i]->p;
      a.tw0 = (const L29*)p.tw0_29.p;
      a.tw1 = (const L29*)((p.fold_scale && i == P - 1) ? p.tw1s_29.p : p.tw1_29.p);
      a.mul_by = (i == P - 1) ? mul_by : nullptr;
      a.n = p.n;
      a.in_len = (i == 0 && in_len) ? in_len : p.n;
      a.log_n = p.log_n;
      a.log_ns = log_ns;
      a.tw_bits = p.tw_bits;
      a.blocks_per_poly = (uint32_t)((p.n >> lr) / W);
      a.batch = (uint32_t)batch;
      Pass256LFn fn = pass256l_fn(lr);
      if (!fn) return fail(PBF_EINVAL, "no 256-bit kernel for this radix");
      const uint64_t blocks = (uint64_t)a.blocks_per_poly * batch;
      if (blocks > 0x7fffffffull) return fail(PBF_EINVAL, "batch too large");
      hipLaunchKernelGGL(fn, dim3((uint32_t)blocks), dim3(threads256l(lr)), 0, st, a);
      PBF_HIP(hipGetLastError());
      log_ns += lr;
    }
    return 0;
  }
  for (size_t i = 0; i < P; ++i) {
    const int lr = p.logr[i];
    const int W = cols256(lr);
    Pass256 a;
    a.in = (i == 0) ? d_in : (const U256*)(((i - 1) & 1) ? s1.p : s0.p);
    a.out = (i == P - 1) ? d_out : (U256*)((i & 1) ? s1.p : s0.p);
    a.rtab = (const U256*)p.rtab[i]->p;
    a.twpass = (const U256*)p.twpass[i]->p;
    a.tw0 = (const U256*)p.tw0.p;
    a.tw1 = (const U256*)p.tw1.p;
    a.mul_by = (i == P - 1) ? mul_by : nullptr;
    a.n_inv = p.n_inv;
    a.n = p.n;
    a.log_n = p.log_n;
    a.log_ns = log_ns;
    a.tw_bits = p.tw_bits;
    a.blocks_per_poly = (uint32_t)((p.n >> lr) / W);
    a.batch = (uint32_t)batch;
    // no Montgomery conversions: the twiddles (and n^-1) are stored in Montgomery form, so
    // mont(x, w R) = x w keeps canonical data canonical through every product, and the adds
    // are the same in both forms -- the first pass's to_mont and the last pass's from_mont
    // (one product per element each) are not needed (conv_* kept for A/B: PBF_NTT256_CONV=1)
    const bool conv = ab_env("PBF_NTT256_CONV") != nullptr;
    a.conv_in = conv && i == 0;
    a.conv_out = conv && i == P - 1;
    a.scale = (p.inverse && i == P - 1 && !p.fold_scale);
    if (p.fold_scale && i == P - 1) a.tw1 = (const U256*)p.tw1s.p;
    Pass256Fn fn = pass256_fn(lr);
    if (!fn) return fail(PBF_EINVAL, "no 256-bit kernel for this radix");
    const uint64_t blocks = (uint64_t)a.blocks_per_poly * batch;
    if (blocks > 0x7fffffffull) return fail(PBF_EINVAL, "batch too large");
    hipLaunchKernelGGL(fn, dim3((uint32_t)blocks), dim3(threads256(lr)), 0, st, a);
    PBF_HIP(hipGetLastError());
    log_ns += lr;
  }
  return 0;
}

// ---------------------------------------------------------------- multi-GPU
// Stride-sharded Fr transform of N = G * nl points, the 256-bit twin of the u64 shard
// kernels in ntt_kernels.hpp: rank g holds a[g + G*m]; local nl-point NTT (root w^G) stored
// as the send layout [dst][b][kk] (S = nl / G); all-to-all; combine:
//   out[b][q*S + kk] = X[q*nl + r*S + kk] = sum_g w_G^(g q) w^(g k) Y_g[k],  k = r*S + kk.
// The inverse runs it backwards (split_inv applies G^-1 and w^(-g k), the local INTT nl^-1).
// Elements canonical at rest; Montgomery inside the kernels; twiddles Montgomery.
struct Shard256Args {
  const U256* in;
  U256* out;
  const U256* tw0;  // two-level table of the global root (forward w, inverse w^-1), Montgomery
  const U256* tw1;
  uint32_t tw_bits;
  uint64_t nl, s, rank, n_mask, batch;
  U256 wg[8];       // w_G^m (forward) / w_G^-m (inverse), Montgomery
  U256 scale;       // G^-1 (inverse) or 1, Montgomery
};

__device__ __forceinline__ U256 tw256(const Shard256Args& a, uint64_t e) {
  return Fr::mul(a.tw0[e & ((1ull << a.tw_bits) - 1)], a.tw1[e >> a.tw_bits]);
}

// [b][g*S + kk] -> [g][b][kk]
__global__ void shard_split256_kernel(const U256* in, U256* out, uint64_t s, uint64_t nl, uint64_t batch) {
  const uint64_t total = nl * batch;
  for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total; id += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = id / nl, k = id % nl;
    out[((k / s) * batch + b) * s + (k % s)] = in[id];
  }
}
// [g][b][kk] -> [b][g*S + kk]
__global__ void shard_unsplit256_kernel(const U256* in, U256* out, uint64_t s, uint64_t nl, uint64_t batch) {
  const uint64_t total = nl * batch;
  for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total; id += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = id / nl, k = id % nl;
    out[id] = in[((k / s) * batch + b) * s + (k % s)];
  }
}

template <int G>
__global__ void __launch_bounds__(256) shard_combine256_kernel(Shard256Args a) {
  const uint64_t total = a.s * a.batch;
  for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total; id += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = id / a.s, kk = id % a.s;
    const uint64_t k = a.rank * a.s + kk;
    U256 t[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const U256 y = Fr::to_mont(a.in[((uint64_t)g * a.batch + b) * a.s + kk]);
      const uint64_t e = ((uint64_t)g * k) & a.n_mask;
      t[g] = (g == 0 || e == 0) ? y : Fr::mul(y, tw256(a, e));
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
      U256 acc = t[0];
#pragma unroll
      for (int g = 1; g < G; ++g) acc = Fr::add(acc, Fr::mul(t[g], a.wg[(g * q) % G]));
      a.out[b * a.nl + (uint64_t)q * a.s + kk] = Fr::from_mont(acc);
    }
  }
}

template <int G>
__global__ void __launch_bounds__(256) shard_split_inv256_kernel(Shard256Args a) {
  const uint64_t total = a.s * a.batch;
  for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total; id += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = id / a.s, kk = id % a.s;
    const uint64_t k = a.rank * a.s + kk;
    U256 x[G];
#pragma unroll
    for (int q = 0; q < G; ++q) x[q] = Fr::to_mont(a.in[b * a.nl + (uint64_t)q * a.s + kk]);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      U256 acc = x[0];
#pragma unroll
      for (int q = 1; q < G; ++q) acc = Fr::add(acc, Fr::mul(x[q], a.wg[(g * q) % G]));
      const uint64_t e = ((uint64_t)g * k) & a.n_mask;
      if (g != 0 && e != 0) acc = Fr::mul(acc, tw256(a, e));
      acc = Fr::mul(acc, a.scale);
      a.out[((uint64_t)g * a.batch + b) * a.s + kk] = Fr::from_mont(acc);
    }
  }
}

struct TwoLevel256 {
  DevBuf t0, t1;
  uint32_t bits = 0;
};

static uint32_t grid256(uint64_t count) {
  const uint64_t b = (count + 255) / 256;
  return (uint32_t)(b > 8192 ? 8192 : (b ? b : 1));
}

static bool canonical_vec(const uint64_t* v, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (!h_canonical(h_from64(v + 4 * i))) return false;
  return true;
}

}  // namespace pbf

using namespace pbf;

// per-context 256-bit plans live in a side table keyed by the context pointer
#include <map>
#include <mutex>
#include <tuple>
namespace {
struct Key256 {
  const void* ctx;
  uint64_t w[4];
  uint64_t n;
  int inv;
  bool operator<(const Key256& o) const {
    return std::tie(ctx, w[0], w[1], w[2], w[3], n, inv) < std::tie(o.ctx, o.w[0], o.w[1], o.w[2], o.w[3], o.n, o.inv);
  }
};
std::map<Key256, std::unique_ptr<Plan256>>& plans256() {
  static std::map<Key256, std::unique_ptr<Plan256>> m;
  return m;
}
std::mutex& plans256_mu() {
  static std::mutex m;
  return m;
}
// extra_r (inverse only): the plan's scale is n^-1 R, for inputs that came out of one Montgomery
// product too few (pointwise_mont256_kernel): the R rides in the last pass's twiddles for free
int get_plan256(pbf_ctx* ctx, const uint64_t* omega, uint64_t n, int inverse, Plan256** out, bool extra_r = false) {
  const int kind = inverse ? (extra_r ? 2 : 1) : 0;
  Key256 k{ctx, {omega[0], omega[1], omega[2], omega[3]}, n, kind};
  std::lock_guard<std::mutex> g(plans256_mu());
  auto it = plans256().find(k);
  if (it != plans256().end()) { *out = it->second.get(); return 0; }
  std::unique_ptr<Plan256> p(new Plan256());
  PBF_HIP(hipSetDevice(ctx->device));
  int rc = make_plan256(ctx->options, omega, n, kind, p.get());
  if (rc) return rc;
  *out = p.get();
  plans256()[k] = std::move(p);
  return 0;
}
}  // namespace

void pbf_internal_drop_plans256(const void* ctx) {
  std::lock_guard<std::mutex> g(plans256_mu());
  auto& m = plans256();
  for (auto it = m.begin(); it != m.end();) it = (it->first.ctx == ctx) ? m.erase(it) : std::next(it);
}

extern "C" {

// fft.rs:66-78 for the BN254 scalar field (elements 4 x u64 little-endian, canonical)
int pbf_ntt_fr256(pbf_ctx* ctx, const uint64_t* omega, const uint64_t* in, uint64_t* out, size_t n, int inverse) {
  if (!ctx || !omega || (!in && n) || (!out && n)) return fail(PBF_EINVAL, "null argument");
  Plan256* p;
  int rc = get_plan256(ctx, omega, n, inverse, &p);
  if (rc) return rc;
  if (!canonical_vec(in, n)) return fail(PBF_EINVAL, "input not canonical");
  hipStream_t s = ctx->host_stream();
  if ((rc = ctx->io0.ensure(n * 32))) return rc;
  PBF_HIP(hipMemcpyAsync(ctx->io0.p, in, n * 32, hipMemcpyHostToDevice, s));
  if ((rc = run256(*p, (const U256*)ctx->io0.p, (U256*)ctx->io0.p, 1, ctx->scratch0, ctx->scratch1, s))) return rc;
  PBF_HIP(hipMemcpyAsync(out, ctx->io0.p, n * 32, hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  return PBF_OK;
}

int pbf_ntt_fr256_batch_dev(pbf_ctx* ctx, const uint64_t* omega, const uint64_t* d_in, uint64_t* d_out, size_t n,
                            size_t batch, int inverse, void* stream) {
  if (!ctx || !omega || !d_in || !d_out) return fail(PBF_EINVAL, "null argument");
  Plan256* p;
  int rc = get_plan256(ctx, omega, n, inverse, &p);
  if (rc) return rc;
  return run256(*p, (const U256*)d_in, (U256*)d_out, batch, ctx->scratch0, ctx->scratch1, (hipStream_t)stream);
}

}  // extern "C"

// The prover's coset transforms (prover.hip coset_ntt_batch): batch x n elements in d_io, of which
// only the first in_len of each polynomial were written (the rest is zero padding the caller has
// not stored): the 29-bit passes read no element past in_len; the 32-bit ones get the padding
// written first. In place.
int pbf_internal_ntt_fr256_prefix(pbf_ctx* ctx, const uint64_t* omega, uint64_t* d_io, size_t n, size_t batch,
                                  size_t in_len, hipStream_t s) {
  Plan256* p;
  int rc = get_plan256(ctx, omega, n, 0, &p);
  if (rc) return rc;
  if (in_len > n) return fail(PBF_EINVAL, "prefix longer than the transform");
  if (!p->l29 || p->logr.empty()) {
    if (in_len < n)
      PBF_HIP(hipMemset2DAsync(d_io + 4 * in_len, n * 32, 0, (n - in_len) * 32, batch, s));
    in_len = 0;
  }
  return run256(*p, (const U256*)d_io, (U256*)d_io, batch, ctx->scratch0, ctx->scratch1, s, nullptr, in_len);
}

extern "C" {

// fft.rs:109-132 mul_ntt for BN254 Fr; out has la+lb elements (4 x u64 each)
int pbf_mul_ntt_fr256(pbf_ctx* ctx, const uint64_t* omega, const uint64_t* a, size_t la, const uint64_t* b,
                      size_t lb, uint64_t* out) {
  if (!ctx || !omega || !out || (!a && la) || (!b && lb)) return fail(PBF_EINVAL, "null argument");
  const size_t n = la + lb;
  Plan256 *fw, *iv;
  const bool mont = !ab_env("PBF_MUL_NTT_TWO_PRODUCTS");  // A/B: to_mont + product, plain inverse
  int rc = get_plan256(ctx, omega, n, 0, &fw);
  if (!rc) rc = get_plan256(ctx, omega, n, 1, &iv, mont);
  if (rc) return rc;
  if (!canonical_vec(a, la) || !canonical_vec(b, lb)) return fail(PBF_EINVAL, "input not canonical");
  hipStream_t s = ctx->host_stream();
  if ((rc = ctx->io0.ensure(2 * n * 32))) return rc;
  U256* d = (U256*)ctx->io0.p;
  PBF_HIP(hipMemsetAsync(d, 0, 2 * n * 32, s));
  if (la) PBF_HIP(hipMemcpyAsync(d, a, la * 32, hipMemcpyHostToDevice, s));
  if (lb) PBF_HIP(hipMemcpyAsync(d + n, b, lb * 32, hipMemcpyHostToDevice, s));
  if ((rc = run256(*fw, d, d, 2, ctx->scratch0, ctx->scratch1, s))) return rc;
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(mont ? pointwise_mont256_kernel : pointwise_mul256_kernel, dim3(blocks), dim3(256), 0, s, d, d + n,
                     d, (uint64_t)n);
  PBF_HIP(hipGetLastError());
  if ((rc = run256(*iv, d, d, 1, ctx->scratch0, ctx->scratch1, s))) return rc;
  PBF_HIP(hipMemcpyAsync(out, d, n * 32, hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  return PBF_OK;
}

// device-pointer mul_ntt over `batch` pairs: d_a/d_b/d_out hold batch x n elements,
// a and b already zero-padded to n = la + lb (the fft.rs:114-118 padding done by the caller)
int pbf_mul_ntt_fr256_dev(pbf_ctx* ctx, const uint64_t* omega, const uint64_t* d_a, const uint64_t* d_b,
                          uint64_t* d_out, size_t n, size_t batch, void* stream) {
  if (!ctx || !omega || !d_a || !d_b || !d_out) return fail(PBF_EINVAL, "null argument");
  Plan256 *fw, *iv;
  const bool mont = !ab_env("PBF_MUL_NTT_TWO_PRODUCTS");  // A/B: to_mont + product, plain inverse
  int rc = get_plan256(ctx, omega, n, 0, &fw);
  if (!rc) rc = get_plan256(ctx, omega, n, 1, &iv, mont);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  // fused (default past 2048 points): b's forward transform multiplies its last pass's outputs by
  // a's (already in d_out) and stores the product there; PBF_MUL_NTT_NO_FUSE=1: pointwise kernel
  if (mont && n > 2048 && !ab_env("PBF_MUL_NTT_NO_FUSE")) {
    if ((rc = run256(*fw, (const U256*)d_a, (U256*)d_out, batch, ctx->scratch0, ctx->scratch1, s))) return rc;
    if ((rc = run256(*fw, (const U256*)d_b, (U256*)d_out, batch, ctx->scratch0, ctx->scratch1, s, (const U256*)d_out)))
      return rc;
    return run256(*iv, (const U256*)d_out, (U256*)d_out, batch, ctx->scratch0, ctx->scratch1, s);
  }
  if ((rc = ctx->io2.ensure(batch * n * 32))) return rc;
  U256* fb = (U256*)ctx->io2.p;
  if ((rc = run256(*fw, (const U256*)d_a, (U256*)d_out, batch, ctx->scratch0, ctx->scratch1, s))) return rc;
  if ((rc = run256(*fw, (const U256*)d_b, fb, batch, ctx->scratch0, ctx->scratch1, s))) return rc;
  uint64_t blocks = (batch * n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(mont ? pointwise_mont256_kernel : pointwise_mul256_kernel, dim3(blocks), dim3(256), 0, s,
                     (const U256*)d_out, fb, (U256*)d_out, (uint64_t)(batch * n));
  PBF_HIP(hipGetLastError());
  return run256(*iv, (const U256*)d_out, (U256*)d_out, batch, ctx->scratch0, ctx->scratch1, s);
}


}  // extern "C"

namespace {
// per-(context, root, N) two-level tables of the global root for the shard combine
std::map<std::tuple<const void*, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t>, std::unique_ptr<TwoLevel256>>&
tl256() {
  static std::map<std::tuple<const void*, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t>, std::unique_ptr<TwoLevel256>> m;
  return m;
}
int get_tl256(pbf_ctx* ctx, const U256& wm, uint64_t N, TwoLevel256** out) {
  uint64_t w4[4];
  u256_to_u64(wm, w4);
  auto k = std::make_tuple((const void*)ctx, w4[0], w4[1], w4[2], w4[3], N);
  std::lock_guard<std::mutex> g(plans256_mu());
  auto it = tl256().find(k);
  if (it != tl256().end()) { *out = it->second.get(); return 0; }
  std::unique_ptr<TwoLevel256> t(new TwoLevel256());
  PBF_HIP(hipSetDevice(ctx->device));
  uint32_t log_n = 0;
  while ((1ull << log_n) < N) ++log_n;
  t->bits = (log_n + 1) / 2;
  int rc = up256(t->t0, h_powers(wm, 1ull << t->bits));
  if (!rc) rc = up256(t->t1, h_powers(h_pow(wm, 1ull << t->bits), (N >> t->bits) ? (N >> t->bits) : 1));
  if (rc) return rc;
  *out = t.get();
  tl256()[k] = std::move(t);
  return 0;
}
// (omega of order G*nl) checks shared by the two shard entry points; wm = Montgomery omega
int shard256_check(const uint64_t* omega, uint32_t G, size_t nl, U256* wm) {
  if (G != 2 && G != 4 && G != 8) return fail(PBF_EINVAL, "world size must be 2, 4 or 8");
  if (nl < G || (nl & (nl - 1))) return fail(PBF_EINVAL, "per-rank size must be a power of two >= G");
  const U256 w = h_from64(omega);
  if (!h_canonical(w)) return fail(PBF_EINVAL, "omega not canonical");
  *wm = Fr::to_mont(w);
  const uint64_t N = (uint64_t)G * nl;
  const U256 one_m = Fr::to_mont(Fr::one_plain());
  if (!Fr::eq(h_pow(*wm, N), one_m) || Fr::eq(h_pow(*wm, N / 2), one_m))
    return fail(PBF_EINVAL, "omega does not have order G*nl");
  return 0;
}
}  // namespace

void pbf_internal_drop_tl256(const void* ctx) {
  std::lock_guard<std::mutex> g(plans256_mu());
  auto& m = tl256();
  for (auto it = m.begin(); it != m.end();) it = (std::get<0>(it->first) == ctx) ? m.erase(it) : std::next(it);
}

extern "C" {

// Multi-GPU stride-sharded Fr NTT, local step (the u64 pbf_ntt_shard_local_dev for 256-bit
// elements): forward [b][m] stride shard -> send [dst][b][kk]; inverse recv [src][b][kk] ->
// [b][m]. Same ABI layout as the u64 entry point, 4 x u64 per element.
int pbf_ntt_fr256_shard_local_dev(pbf_ctx* ctx, const uint64_t* omega, uint32_t world, const uint64_t* d_in,
                                  uint64_t* d_out, size_t nl, size_t batch, int inverse, void* stream) {
  if (!ctx || !omega || !d_in || !d_out) return fail(PBF_EINVAL, "null argument");
  U256 wm;
  int rc = shard256_check(omega, world, nl, &wm);
  if (rc) return rc;
  PBF_HIP(hipSetDevice(ctx->device));
  uint64_t wl[4];
  u256_to_u64(Fr::from_mont(h_pow(wm, world)), wl);  // local root w^G, order nl
  Plan256* p;
  if ((rc = get_plan256(ctx, wl, nl, inverse, &p))) return rc;
  hipStream_t s = (hipStream_t)stream;
  if ((rc = ctx->scratch2.ensure(batch * nl * 32))) return rc;
  U256* tmp = (U256*)ctx->scratch2.p;
  const uint64_t S = nl / world;
  if (!inverse) {
    if ((rc = run256(*p, (const U256*)d_in, tmp, batch, ctx->scratch0, ctx->scratch1, s))) return rc;
    hipLaunchKernelGGL(shard_split256_kernel, dim3(grid256(nl * batch)), dim3(256), 0, s, (const U256*)tmp,
                       (U256*)d_out, S, (uint64_t)nl, (uint64_t)batch);
    PBF_HIP(hipGetLastError());
    return 0;
  }
  hipLaunchKernelGGL(shard_unsplit256_kernel, dim3(grid256(nl * batch)), dim3(256), 0, s, (const U256*)d_in, tmp, S,
                     (uint64_t)nl, (uint64_t)batch);
  PBF_HIP(hipGetLastError());
  return run256(*p, tmp, (U256*)d_out, batch, ctx->scratch0, ctx->scratch1, s);
}

// Multi-GPU stride-sharded Fr NTT, combine step (forward: recv -> out[b][q*S + kk]);
// inverse: the blocked layout -> send [dst][b][kk] (twiddle w^-(g k), radix-G, G^-1).
int pbf_ntt_fr256_shard_combine_dev(pbf_ctx* ctx, const uint64_t* omega, uint32_t world, uint32_t rank,
                                    const uint64_t* d_in, uint64_t* d_out, size_t nl, size_t batch, int inverse,
                                    void* stream) {
  if (!ctx || !omega || !d_in || !d_out) return fail(PBF_EINVAL, "null argument");
  if (d_in == d_out) return fail(PBF_EINVAL, "combine is out-of-place");
  U256 wm;
  int rc = shard256_check(omega, world, nl, &wm);
  if (rc) return rc;
  if (rank >= world) return fail(PBF_EINVAL, "rank out of range");
  PBF_HIP(hipSetDevice(ctx->device));
  const uint64_t N = (uint64_t)world * nl;
  const U256 root = inverse ? h_inv(wm) : wm;
  TwoLevel256* tl;
  if ((rc = get_tl256(ctx, root, N, &tl))) return rc;
  Shard256Args a;
  a.in = (const U256*)d_in;
  a.out = (U256*)d_out;
  a.tw0 = (const U256*)tl->t0.p;
  a.tw1 = (const U256*)tl->t1.p;
  a.tw_bits = tl->bits;
  a.nl = nl;
  a.s = nl / world;
  a.rank = rank;
  a.n_mask = N - 1;
  a.batch = batch;
  const U256 wG = h_pow(root, nl);  // primitive G-th root (direction-specific)
  U256 x = Fr::to_mont(Fr::one_plain());
  for (uint32_t i = 0; i < 8; ++i) {
    a.wg[i] = x;
    if (i + 1 < world) x = Fr::mul(x, wG);
  }
  {
    U256 gg = Fr::one_plain();
    gg.w[0] = world;
    a.scale = inverse ? h_inv(Fr::to_mont(gg)) : Fr::to_mont(Fr::one_plain());
  }
  void (*fn)(Shard256Args) = nullptr;
  switch (world) {
    case 2: fn = inverse ? shard_split_inv256_kernel<2> : shard_combine256_kernel<2>; break;
    case 4: fn = inverse ? shard_split_inv256_kernel<4> : shard_combine256_kernel<4>; break;
    default: fn = inverse ? shard_split_inv256_kernel<8> : shard_combine256_kernel<8>; break;
  }
  hipLaunchKernelGGL(fn, dim3(grid256(a.s * batch)), dim3(256), 0, (hipStream_t)stream, a);
  PBF_HIP(hipGetLastError());
  return 0;
}

// c[i] = a[i] * b[i] over `count` Fr elements (the pointwise step of mul_ntt, fft.rs:125-129)
int pbf_pointwise_mul_fr256_dev(pbf_ctx* ctx, const uint64_t* d_a, const uint64_t* d_b, uint64_t* d_c, size_t count,
                                void* stream) {
  if (!ctx || (count && (!d_a || !d_b || !d_c))) return fail(PBF_EINVAL, "null argument");
  if (count == 0) return 0;
  PBF_HIP(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(pointwise_mul256_kernel, dim3(grid256(count)), dim3(256), 0, (hipStream_t)stream,
                     (const U256*)d_a, (const U256*)d_b, (U256*)d_c, (uint64_t)count);
  PBF_HIP(hipGetLastError());
  return 0;
}

}  // extern "C"
