// NTT kernels for gfx950 — the MI355X replacement of src/fft.rs CooleyTurkey
// (fft.rs:55-106). Output is the natural-order DFT X_k = sum_j a_j w^(jk), exactly
// what the reference's recursive radix-2 DIT computes, so results are bit-identical.
//
// Structure (DESIGN.md "NTT"): a Stockham autosort over HBM in P passes of radix
// R = 2^LOGR. One pass reads every element once and writes it once:
//   pass input  x[j + r*(n/R)],  j < n/R, r < R        (W consecutive j per workgroup:
//                                                       W-element contiguous runs)
//   pre-twiddle x_r *= w^((n/(Ns*R)) * r * (j mod Ns))  (Ns = product of earlier radices)
//   R-point DFT along r (in LDS + registers, radix-16 register sub-DFTs)
//   pass output y[(j/Ns)*Ns*R + (j mod Ns) + r'*Ns]
// Inside a workgroup the R-point DFT is itself a Stockham over radix-q (q <= 16)
// register sub-DFTs with the LDS as the exchange buffer between stages.
#pragma once
#include "field.hpp"

namespace pbf {

struct PassArgs {
  const uint64_t* in;    // pass input  (batch * n elements)
  uint64_t* out;         // pass output (batch * n elements)
  const uint64_t* tw0;   // w^m for m < 2^tw_bits            (two-level table, low part)
  const uint64_t* tw1;   // w^(m << tw_bits) for m < n>>tw_bits (high part)
  const uint64_t* rtab;  // w_R^m = w^(m*n/R) for m < R
  uint64_t n;            // transform size
  uint64_t n_inv;        // n^-1, applied to outputs when scale != 0
  uint32_t log_n;
  uint32_t log_ns;       // log2 of the product of radices of earlier passes
  uint32_t tw_bits;
  uint32_t blocks_per_poly;
  uint32_t scale;
  uint32_t out_split_log;  // != 0: last pass stores destination-major [n/S][batch][S], S = 2^out_split_log
  uint32_t batch;
  FieldArgs f;
};

// ---- compile-time helpers ----------------------------------------------------
__host__ __device__ constexpr int ntt_nstages(int logr) { return (logr + 3) / 4; }
// remainder radix first, then radix-16 stages
__host__ __device__ constexpr int ntt_stage_logq(int logr, int s) {
  return (logr % 4 == 0) ? 4 : (s == 0 ? logr % 4 : 4);
}
__host__ __device__ constexpr int ntt_stage_logl(int logr, int s) {
  int l = 0;
  for (int i = 0; i < s; ++i) l += ntt_stage_logq(logr, i);
  return l;
}
__host__ __device__ constexpr int bitrev_c(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; ++i) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}

// w^e for e < n from the two-level table (one multiplication).
template <class F>
__device__ __forceinline__ uint64_t tw_pow(const PassArgs& a, uint64_t e) {
  uint64_t lo = a.tw0[e & ((1ull << a.tw_bits) - 1)];
  uint64_t hi = a.tw1[e >> a.tw_bits];
  return F::mul(lo, hi, a.f);
}

// In-register q-point DFT (decimation in frequency, natural in, bit-reversed out).
// wq[m] = w_q^m for m < q/2 (w_q a primitive q-th root of unity).
template <class F, int LOGQ>
__device__ __forceinline__ void dft_reg(uint64_t* v, const uint64_t* wq, const FieldArgs& f) {
  constexpr int Q = 1 << LOGQ;
#pragma unroll
  for (int h = Q / 2; h >= 1; h >>= 1) {
#pragma unroll
    for (int blk = 0; blk < Q; blk += 2 * h) {
#pragma unroll
      for (int a = 0; a < h; ++a) {
        uint64_t x = v[blk + a], y = v[blk + a + h];
        v[blk + a] = F::add(x, y, f);
        uint64_t d = F::sub(x, y, f);
        // w_(2h)^a = w_q^(a * q/(2h))
        v[blk + a + h] = (a == 0) ? d : F::mul(d, wq[a * (Q / (2 * h))], f);
      }
    }
  }
}

// One register/LDS stage S of the in-workgroup R-point Stockham (radix Q = 2^logq).
template <class F, int LOGR, int W, int NT, int S>
__device__ __forceinline__ void ntt_stage(uint64_t* v, uint64_t* lds, const uint64_t* wq, const PassArgs& a,
                                          const uint64_t* in, uint64_t* out, uint64_t j0, int t) {
  constexpr int R = 1 << LOGR;
  constexpr int PER = (R * W) / NT;
  constexpr int NST = ntt_nstages(LOGR);
  constexpr int LOGQ = ntt_stage_logq(LOGR, S);
  constexpr int Q = 1 << LOGQ;
  constexpr int L = 1 << ntt_stage_logl(LOGR, S);
  constexpr int NSUB = PER / Q;
  constexpr bool LAST = (S == NST - 1);
  const uint64_t n = a.n;
  // ---- gather inputs (stage 0 straight from HBM with the pass pre-twiddle)
#pragma unroll
  for (int u = 0; u < NSUB; ++u) {
    const int sub = t + NT * u;
    const int w = sub % W, i = sub / W;
#pragma unroll
    for (int c = 0; c < Q; ++c) {
      const int r = i + c * (R / Q);
      uint64_t x;
      if constexpr (S == 0) {
        x = in[(j0 + w) + (uint64_t)r * (n >> LOGR)];
        if (a.log_ns > 0) {
          const uint64_t k = (j0 + w) & ((1ull << a.log_ns) - 1);
          const uint64_t e = (((uint64_t)r * k) << (a.log_n - a.log_ns - LOGR)) & (n - 1);
          if (e) x = F::mul(x, tw_pow<F>(a, e), a.f);
        }
      } else {
        x = lds[r * W + w];
        const int k = i % L;  // stage twiddle w_(L*Q)^(c*k) = w_R^((R/(L*Q))*c*k)
        if (c != 0 && k != 0) x = F::mul(x, a.rtab[(R / (L * Q)) * c * k], a.f);
      }
      v[u * Q + c] = x;
    }
  }
  // ---- radix-Q DFTs in registers
#pragma unroll
  for (int u = 0; u < NSUB; ++u) {
    if constexpr (LOGQ == 4) {
      dft_reg<F, 4>(v + u * Q, wq, a.f);
    } else if constexpr (LOGQ == 3) {
      const uint64_t w8[4] = {wq[0], wq[2], wq[4], wq[6]};
      dft_reg<F, 3>(v + u * Q, w8, a.f);
    } else if constexpr (LOGQ == 2) {
      const uint64_t w4[2] = {wq[0], wq[4]};
      dft_reg<F, 2>(v + u * Q, w4, a.f);
    } else {
      const uint64_t w2[1] = {wq[0]};
      dft_reg<F, 1>(v + u * Q, w2, a.f);
    }
  }
  if constexpr (S > 0) __syncthreads();  // all reads of the exchange buffer are done
  // ---- scatter outputs
#pragma unroll
  for (int u = 0; u < NSUB; ++u) {
    const int sub = t + NT * u;
    const int w = sub % W, i = sub / W;
    const int k = i % L;
#pragma unroll
    for (int d = 0; d < Q; ++d) {
      uint64_t y = v[u * Q + bitrev_c(d, LOGQ)];
      const int r = (i / L) * L * Q + k + d * L;  // Stockham output slot
      if constexpr (!LAST) {
        lds[r * W + w] = y;
      } else {
        if (a.scale) y = F::mul(y, a.n_inv, a.f);
        if (a.log_ns == 0) {
          lds[w * (R + 1) + r] = y;  // transposed image, stored linearly by the caller
        } else {
          const uint64_t j = j0 + w;
          const uint64_t ns_mask = (1ull << a.log_ns) - 1;
          const uint64_t k = ((j >> a.log_ns) << (a.log_ns + LOGR)) + (j & ns_mask) + ((uint64_t)r << a.log_ns);
          if (a.out_split_log == 0) {
            out[k] = y;
          } else {
            // multi-GPU send layout: block k/S goes to rank k/S, polynomials contiguous per rank
            const uint64_t poly = blockIdx.x / a.blocks_per_poly;
            const uint64_t sl = a.out_split_log;
            a.out[((((k >> sl) * a.batch) + poly) << sl) + (k & ((1ull << sl) - 1))] = y;
          }
        }
      }
    }
  }
  if constexpr (!LAST) {
    __syncthreads();
    ntt_stage<F, LOGR, W, NT, S + 1>(v, lds, wq, a, in, out, j0, t);
  }
}

// One Stockham pass over HBM. NT threads, W columns of R = 2^LOGR points each.
template <class F, int LOGR, int W, int NT>
__global__ void __launch_bounds__(NT) ntt_pass_kernel(PassArgs a) {
  constexpr int R = 1 << LOGR;
  constexpr int E = R * W;
  constexpr int PER = E / NT;
  static_assert(LOGR >= 4, "radix-16 register sub-DFTs need R >= 16");
  static_assert(PER >= 16 && PER % 16 == 0, "each thread must own whole radix-16 sub-DFTs");
  static_assert(E <= 16384, "LDS budget: 128 KiB of elements per workgroup");
  // +W pad keeps the transposed [w][r] image of the first pass bank-conflict free
  __shared__ uint64_t lds[E + W];

  const uint32_t poly = blockIdx.x / a.blocks_per_poly;
  const uint64_t j0 = (uint64_t)(blockIdx.x % a.blocks_per_poly) * W;
  const uint64_t* in = a.in + (uint64_t)poly * a.n;
  uint64_t* out = a.out + (uint64_t)poly * a.n;
  const int t = threadIdx.x;

  uint64_t v[PER];
  uint64_t wq[8];  // w_16^m, m < 8 (the roots for q < 16 are sub-powers)
#pragma unroll
  for (int m = 0; m < 8; ++m) wq[m] = a.rtab[m * (R / 16)];

  ntt_stage<F, LOGR, W, NT, 0>(v, lds, wq, a, in, out, j0, t);

  if (a.log_ns == 0) {
    // first pass: this workgroup's outputs are y[j0*R .. (j0+W)*R), contiguous
    __syncthreads();
    uint64_t* o = out + j0 * R;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int m = t + NT * u;
      o[m] = lds[(m / R) * (R + 1) + (m % R)];
    }
  }
}

// Whole transform of a small n (<= 4096) inside one workgroup per polynomial:
// bit-reversed load into LDS, log2(n) radix-2 DIT stages, natural-order store.
template <class F>
__global__ void __launch_bounds__(256) ntt_small_kernel(const uint64_t* in, uint64_t* out, const uint64_t* tw,
                                                        uint32_t logn, uint64_t n_inv, uint32_t scale,
                                                        FieldArgs f) {
  __shared__ uint64_t lds[4096];
  const uint32_t n = 1u << logn;
  const uint64_t* src = in + (uint64_t)blockIdx.x * n;
  uint64_t* dst = out + (uint64_t)blockIdx.x * n;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t r = logn ? (__brev(i) >> (32 - logn)) : 0;
    lds[r] = src[i];
  }
  __syncthreads();
  for (uint32_t len = 2; len <= n; len <<= 1) {
    const uint32_t half = len >> 1;
    for (uint32_t b = threadIdx.x; b < n / 2; b += blockDim.x) {
      const uint32_t grp = b / half, k = b % half;
      const uint32_t i0 = grp * len + k, i1 = i0 + half;
      const uint64_t w = tw[(uint64_t)k * (n / len)];
      const uint64_t x = lds[i0], y = F::mul(lds[i1], w, f);
      lds[i0] = F::add(x, y, f);
      lds[i1] = F::sub(x, y, f);
    }
    __syncthreads();
  }
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    uint64_t y = lds[i];
    dst[i] = scale ? F::mul(y, n_inv, f) : y;
  }
}

// Multi-GPU combine (DESIGN.md "Multi-GPU"), forward direction. The global
// transform of N = G * nl points is stride-sharded: rank g held a[g + G*m] and
// computed Y_g = NTT_nl(a[g::G]) with root w^G. After the all-to-all, rank r holds
// recv[g][b][kk] = Y_g[r*S + kk] (S = nl/G) and produces, for k = r*S + kk,
//   X[k + q*nl] = sum_g w_G^(g*q) * (w^(g*k) * Y_g[k]),   q < G,
// stored as out[b][q*S + kk]. Inverse: the same butterfly with w^-1 applied in the
// opposite order (twiddle after the G-point DFT), see shard_split_inv_kernel.
struct CombineArgs {
  const uint64_t* recv;
  uint64_t* out;
  const uint64_t* tw0;   // two-level table of the global root (forward: w, inverse: w^-1)
  const uint64_t* tw1;
  uint64_t nl;           // per-rank transform size
  uint64_t s;            // nl / G
  uint64_t rank;
  uint64_t n_mask;       // G*nl - 1
  uint64_t scale;        // multiplier applied to every output (1, or G^-1 for the inverse)
  uint32_t tw_bits;
  uint32_t batch;
  uint64_t wg[8];        // w_G^m (forward) or w_G^-m (inverse), m < G
  FieldArgs f;
};

template <class F>
__device__ __forceinline__ uint64_t tw_pow2(const uint64_t* tw0, const uint64_t* tw1, uint32_t bits, uint64_t e,
                                            const FieldArgs& f) {
  return F::mul(tw0[e & ((1ull << bits) - 1)], tw1[e >> bits], f);
}

template <class F, int G>
__global__ void __launch_bounds__(256) shard_combine_kernel(CombineArgs a) {
  const uint64_t total = a.s * a.batch;
  for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
       id += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = id / a.s, kk = id % a.s;
    const uint64_t k = a.rank * a.s + kk;
    uint64_t t[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      uint64_t y = a.recv[((uint64_t)g * a.batch + b) * a.s + kk];
      const uint64_t e = ((uint64_t)g * k) & a.n_mask;
      t[g] = (g == 0 || e == 0) ? y : F::mul(y, tw_pow2<F>(a.tw0, a.tw1, a.tw_bits, e, a.f), a.f);
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
      uint64_t acc = t[0];
#pragma unroll
      for (int g = 1; g < G; ++g) acc = F::add(acc, F::mul(t[g], a.wg[(g * q) % G], a.f), a.f);
      if (a.scale != 1) acc = F::mul(acc, a.scale, a.f);
      a.out[b * a.nl + (uint64_t)q * a.s + kk] = acc;
    }
  }
}

// Inverse of the combine: rank r holds X (blocked, out[b][q*S + kk] layout) and
// produces send[g][b][kk] = G^-1 * w^(-g*k) * sum_q w_G^(-g*q) X[k + q*nl].
template <class F, int G>
__global__ void __launch_bounds__(256) shard_split_inv_kernel(CombineArgs a) {
  const uint64_t total = a.s * a.batch;
  for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
       id += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = id / a.s, kk = id % a.s;
    const uint64_t k = a.rank * a.s + kk;
    uint64_t x[G];
#pragma unroll
    for (int q = 0; q < G; ++q) x[q] = a.recv[b * a.nl + (uint64_t)q * a.s + kk];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      uint64_t acc = x[0];
#pragma unroll
      for (int q = 1; q < G; ++q) acc = F::add(acc, F::mul(x[q], a.wg[(g * q) % G], a.f), a.f);
      const uint64_t e = ((uint64_t)g * k) & a.n_mask;
      if (g != 0 && e != 0) acc = F::mul(acc, tw_pow2<F>(a.tw0, a.tw1, a.tw_bits, e, a.f), a.f);
      if (a.scale != 1) acc = F::mul(acc, a.scale, a.f);
      a.out[((uint64_t)g * a.batch + b) * a.s + kk] = acc;
    }
  }
}

// Gather the inverse's received blocks recv[g][b][kk] (from rank g, block of this
// rank r) into per-polynomial natural order y[b][g*S + kk] for the local INTT.
__global__ void shard_unsplit_kernel(const uint64_t* recv, uint64_t* out, uint64_t s, uint64_t nl, uint32_t batch,
                                     uint32_t G) {
  const uint64_t total = nl * batch;
  for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
       id += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = id / nl, k = id % nl;
    const uint64_t g = k / s, kk = k % s;
    out[id] = recv[(g * batch + b) * s + kk];
  }
}

// c[i] = a[i] * b[i]  (the pointwise step of mul_ntt, fft.rs:125-129)
template <class F>
__global__ void pointwise_mul_kernel(const uint64_t* a, const uint64_t* b, uint64_t* c, uint64_t count,
                                     FieldArgs f) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
    c[i] = F::mul(a[i], b[i], f);
}

}  // namespace pbf
