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

// Timing-only modes (PassArgs::dbg) are compiled in only with -DPBF_NTT_TIMING_MODES:
// the per-element runtime checks they need split the kernels into many basic blocks.
#ifdef PBF_NTT_TIMING_MODES
#define PBF_DBG(a, bit) (((a).dbg & (bit)) != 0)
#else
#define PBF_DBG(a, bit) false
#endif

struct PassArgs {
  const uint64_t* in;    // pass input  (batch * n elements)
  uint64_t* out;         // pass output (batch * n elements)
  const uint64_t* tw0;   // w^m for m < 2^tw_bits            (two-level table, low part)
  const uint64_t* tw1;   // w^(m << tw_bits) for m < n>>tw_bits (high part)
  const uint64_t* rtab;  // w_R^m = w^(m*n/R) for m < R
  const uint64_t* twfull; // unused (always null; kept for the argument layout)
  const uint64_t* twpass; // this pass's twiddles T[r][k] = w^((n/(Ns*R))*r*k), or null
  uint64_t n;            // transform size
  uint64_t n_inv;        // n^-1, applied to outputs when scale != 0
  uint32_t log_n;
  uint32_t log_ns;       // log2 of the product of radices of earlier passes
  uint32_t tw_bits;
  uint32_t blocks_per_poly;
  uint32_t scale;
  uint32_t dbg;            // timing builds only (PBF_NTT_TIMING_MODES): 1 = no HBM traffic, 2 = no butterflies
  uint32_t cur_poly;       // set per tile inside the kernel
  uint32_t out_split_log;  // != 0: last pass stores destination-major [n/S][batch][S], S = 2^out_split_log
  uint32_t batch;
  uint32_t xcd_kmajor;     // non-persistent grid, gridDim.x % 8 == 0: XCD-aware column-major block order
  FieldArgs f;
};

// ---- compile-time helpers ----------------------------------------------------
// In-workgroup stages: radix 2^LQ (LQ = log2 of the largest register radix), the
// remainder radix first.
__host__ __device__ constexpr int ntt_nstages(int logr, int lq) { return (logr + lq - 1) / lq; }
__host__ __device__ constexpr int ntt_stage_logq(int logr, int s, int lq) {
  return (logr % lq == 0) ? lq : (s == 0 ? logr % lq : lq);
}
__host__ __device__ constexpr int ntt_stage_logl(int logr, int s, int lq) {
  int l = 0;
  for (int i = 0; i < s; ++i) l += ntt_stage_logq(logr, i, lq);
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
// E < 0: twiddles from wq[m] = w_q^m (m < q/2), full multiplications.
// E >= 0: w_q = 2^E (mod p) — Goldilocks standard roots of order <= 64 are powers
// of two — so every twiddle is a shift-reduction; a twiddle -2^(S-96) folds its
// sign into the butterfly's subtraction.
// Twiddle 2^RAW (RAW mod 192; 2^96 = -1) as the cheapest equivalent: x*2^S for S <= 64,
// else -x*2^-(96-S) (a division by 2^K, K < 32, gl_div_pow2), with the sign folded into
// the butterfly's subtraction (NEG) — see DESIGN.md "Goldilocks arithmetic".
template <int RAW_>
struct ShiftKind {
  static constexpr int RAW = ((RAW_ % 192) + 192) % 192;
  static constexpr bool NEG0 = RAW >= 96;
  static constexpr int S0 = NEG0 ? RAW - 96 : RAW;   // x * 2^RAW = (-1)^NEG0 x * 2^S0
  static constexpr bool DIV = S0 > 64;               // 2^S0 = -2^-(96-S0)
  static constexpr bool NEG = DIV ? !NEG0 : NEG0;
  static constexpr int S = DIV ? 96 - S0 : S0;       // shift (DIV: divisor exponent)
};
template <int E, int LOGQ, int H, int A>
struct TwShift : ShiftKind<(E * A * ((1 << LOGQ) / (2 * H))) % 192> {};

// d * 2^S (mul) or d / 2^S (div) for a ShiftKind
template <class F, class T>
__device__ __forceinline__ uint64_t apply_shift(uint64_t d) {
  if constexpr (T::DIV) return gl_div_pow2<T::S>(d);
  else return F::template mul_pow2<T::S>(d);
}

template <class F, int LOGQ, int E, int H, int A>
__device__ __forceinline__ void dif_bfly(uint64_t* v, int blk, const uint64_t* wq, const FieldArgs& f) {
  constexpr int Q = 1 << LOGQ;
  const uint64_t x = v[blk + A], y = v[blk + A + H];
  v[blk + A] = F::add(x, y, f);
  if constexpr (A == 0) {
    v[blk + A + H] = F::sub(x, y, f);
  } else if constexpr (E < 0) {
    v[blk + A + H] = F::mul(F::sub(x, y, f), wq[A * (Q / (2 * H))], f);
  } else {
    using T = TwShift<E, LOGQ, H, A>;
    const uint64_t d = T::NEG ? F::sub(y, x, f) : F::sub(x, y, f);
    v[blk + A + H] = apply_shift<F, T>(d);
  }
}

template <class F, int LOGQ, int E, int H, int A>
__device__ __forceinline__ void dif_row(uint64_t* v, const uint64_t* wq, const FieldArgs& f) {
  if constexpr (A < H) {
    constexpr int Q = 1 << LOGQ;
#pragma unroll
    for (int blk = 0; blk < Q; blk += 2 * H) dif_bfly<F, LOGQ, E, H, A>(v, blk, wq, f);
    dif_row<F, LOGQ, E, H, A + 1>(v, wq, f);
  }
}

template <class F, int LOGQ, int E, int H>
__device__ __forceinline__ void dif_levels(uint64_t* v, const uint64_t* wq, const FieldArgs& f) {
  if constexpr (H >= 1) {
    dif_row<F, LOGQ, E, H, 0>(v, wq, f);
    dif_levels<F, LOGQ, E, H / 2>(v, wq, f);
  }
}

template <class F, int LOGQ, int E>
__device__ __forceinline__ void dft_reg(uint64_t* v, const uint64_t* wq, const FieldArgs& f) {
  dif_levels<F, LOGQ, E, (1 << LOGQ) / 2>(v, wq, f);
}

// Exponent of w_q = 2^E given w_64 = 2^E64 (E64 < 0: table twiddles).
__host__ __device__ constexpr int sub_root_exp(int e64, int logq) {
  return e64 < 0 ? -1 : (e64 * (64 >> logq)) % 192;
}

// Workgroup barrier of the in-tile stages. DB (LDS-DMA double-buffered) kernels use a
// raw s_barrier with lgkmcnt(0) only, so the next tile's LDS-DMA stays in flight
// (hipcc's __syncthreads() would emit vmcnt(0) and drain it: guide "Pipelining
// across barriers").
template <bool DB>
__device__ __forceinline__ void tile_barrier() {
  if constexpr (DB) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  } else {
    __syncthreads();
  }
}

// Raw stage-0 inputs of one tile into registers (the same thread -> element map as stage 0).
template <int LOGR, int W, int NT, int LQ>
__device__ __forceinline__ void tile_load(uint64_t* v, const PassArgs& a, const uint64_t* in, uint64_t j0, int t) {
  constexpr int R = 1 << LOGR;
  constexpr int PER = (R * W) / NT;
  constexpr int Q = 1 << ntt_stage_logq(LOGR, 0, LQ);
#pragma unroll
  for (int u = 0; u < PER / Q; ++u) {
    const int sub = t + NT * u;
    const int w = sub % W, i = sub / W;
#pragma unroll
    for (int c = 0; c < Q; ++c) {
      const int r = i + c * (R / Q);
      v[u * Q + c] = PBF_DBG(a, 1) ? (uint64_t)(t * 0x9E3779B9u + r) * 0x100000001ull
                                 : in[(j0 + w) + (uint64_t)r * (a.n >> LOGR)];
    }
  }
}

// One register/LDS stage S of the in-workgroup R-point Stockham (radix Q = 2^logq).
// Stage 0 takes the raw tile (registers v) and applies the pass twiddle; later stages read
// the exchange buffer and apply the stage twiddle from `rt`. (The LDS-DMA double-buffered and
// register-prefetching persistent forms of rounds 1-2 measured slower; removed in round 6.)
template <class F, int LOGR, int W, int NT, int LQ, int E64, int S>
__device__ __forceinline__ void ntt_stage(uint64_t* v, uint64_t* buf, const uint64_t* rt, const uint64_t* wq,
                                          const PassArgs& a, uint64_t* out, uint64_t j0, int t) {
  constexpr int R = 1 << LOGR;
  constexpr int PER = (R * W) / NT;
  constexpr int NST = ntt_nstages(LOGR, LQ);
  constexpr int LOGQ = ntt_stage_logq(LOGR, S, LQ);
  constexpr int Q = 1 << LOGQ;
  constexpr int L = 1 << ntt_stage_logl(LOGR, S, LQ);
  constexpr int NSUB = PER / Q;
  constexpr bool LAST = (S == NST - 1);
  const uint64_t n = a.n;
  // ---- gather inputs. The pass-twiddle variant is chosen once per tile (uniform
  // branches hoisted out of the unrolled loops) so all PER twiddle loads issue
  // back to back and are waited for once.
  if constexpr (S == 0) {
    if (a.log_ns > 0) {
      const uint64_t kmask = (1ull << a.log_ns) - 1;
      if (a.twpass) {
        // per-pass table [r][k] (k contiguous across lanes: coalesced loads); lanes with
        // r*k == 0 multiply by T = 1 (a per-lane branch would only diverge)
        uint64_t tw[PER];
#pragma unroll
        for (int u = 0; u < NSUB; ++u) {
          const int sub = t + NT * u;
          const int w = sub % W, i = sub / W;
          const uint64_t k = (j0 + w) & kmask;
#pragma unroll
          for (int c = 0; c < Q; ++c) tw[u * Q + c] = a.twpass[((uint64_t)(i + c * (R / Q)) << a.log_ns) + k];
        }
#pragma unroll
        for (int m = 0; m < PER; ++m) v[m] = F::mul(v[m], tw[m], a.f);
      } else {
#pragma unroll
        for (int u = 0; u < NSUB; ++u) {
          const int sub = t + NT * u;
          const int w = sub % W, i = sub / W;
          const uint64_t k = (j0 + w) & kmask;
#pragma unroll
          for (int c = 0; c < Q; ++c) {
            const uint64_t r = i + c * (R / Q);
            const uint64_t e = ((r * k) << (a.log_n - a.log_ns - LOGR)) & (n - 1);
            if (e) v[u * Q + c] = F::mul(v[u * Q + c], tw_pow<F>(a, e), a.f);
          }
        }
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      const int sub = t + NT * u;
      const int w = sub % W, i = sub / W;
      const int k = i % L;  // stage twiddle w_(L*Q)^(c*k) = w_R^((R/(L*Q))*c*k)
#pragma unroll
      for (int c = 0; c < Q; ++c) {
        const uint64_t x = buf[(i + c * (R / Q)) * W + w];
        v[u * Q + c] = (c != 0) ? F::mul(x, rt[(R / (L * Q)) * c * k], a.f) : x;  // k == 0: rt[0] = 1
      }
    }
  }
  // ---- radix-Q DFTs in registers (wq[m] = w_QMAX^m; w_Q = w_QMAX^(QMAX/Q))
  constexpr int QMAX = 1 << LQ;
#pragma unroll
  for (int u = 0; u < NSUB; ++u) {
    uint64_t wloc[Q / 2 > 0 ? Q / 2 : 1];
    if constexpr (E64 < 0) {
#pragma unroll
      for (int m = 0; m < Q / 2; ++m) wloc[m] = wq[m * (QMAX / Q)];
    }
    if (!PBF_DBG(a, 2)) dft_reg<F, LOGQ, sub_root_exp(E64, LOGQ)>(v + u * Q, wloc, a.f);
  }
  if constexpr (S > 0) tile_barrier<false>();  // all reads of the exchange buffer are done
  // ---- scatter outputs (uniform output-mode branches hoisted out of the unrolled loops)
  if constexpr (!LAST) {
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      const int sub = t + NT * u;
      const int w = sub % W, i = sub / W;
#pragma unroll
      for (int d = 0; d < Q; ++d)
        buf[((i / L) * L * Q + (i % L) + d * L) * W + w] = v[u * Q + bitrev_c(d, LOGQ)];  // Stockham slot
    }
  } else {
    if (a.scale) {
#pragma unroll
      for (int m = 0; m < PER; ++m) v[m] = F::mul(v[m], a.n_inv, a.f);
    }
    if (a.log_ns == 0) {
      // transposed image, stored linearly by the caller
#pragma unroll
      for (int u = 0; u < NSUB; ++u) {
        const int sub = t + NT * u;
        const int w = sub % W, i = sub / W;
#pragma unroll
        for (int d = 0; d < Q; ++d)
          buf[w * (R + 1) + (i / L) * L * Q + (i % L) + d * L] = v[u * Q + bitrev_c(d, LOGQ)];
      }
    } else {
      const uint64_t ns_mask = (1ull << a.log_ns) - 1;
      const uint32_t sl = a.out_split_log;
      // output index of element d of sub-DFT u: kbase(u) + (slot << log_ns)
      auto kk_of = [&](int u, int d) -> uint64_t {
        const int sub = t + NT * u;
        const int w = sub % W, i = sub / W;
        const uint64_t j = j0 + w;
        return ((j >> a.log_ns) << (a.log_ns + LOGR)) + (j & ns_mask) +
               ((uint64_t)((i / L) * L * Q + (i % L) + d * L) << a.log_ns);
      };
      if (PBF_DBG(a, 1)) {
#pragma unroll
        for (int u = 0; u < NSUB; ++u)
#pragma unroll
          for (int d = 0; d < Q; ++d) {
            const uint64_t y = v[u * Q + bitrev_c(d, LOGQ)];
            if (y == 0x123456789ull) out[kk_of(u, d)] = y;  // keeps the arithmetic live
          }
      } else if (sl == 0) {
#pragma unroll
        for (int u = 0; u < NSUB; ++u)
#pragma unroll
          for (int d = 0; d < Q; ++d) out[kk_of(u, d)] = v[u * Q + bitrev_c(d, LOGQ)];
      } else {
        // multi-GPU send layout: block kk/S goes to rank kk/S, polynomials contiguous per rank
        const uint64_t smask = (1ull << sl) - 1;
#pragma unroll
        for (int u = 0; u < NSUB; ++u)
#pragma unroll
          for (int d = 0; d < Q; ++d) {
            const uint64_t kk = kk_of(u, d);
            a.out[((((kk >> sl) * a.batch) + a.cur_poly) << sl) + (kk & smask)] = v[u * Q + bitrev_c(d, LOGQ)];
          }
      }
    }
  }
  if constexpr (!LAST) {
    tile_barrier<false>();
    ntt_stage<F, LOGR, W, NT, LQ, E64, S + 1>(v, buf, rt, wq, a, out, j0, t);
  }
}

// Store the first pass's transposed [w][r] image: outputs y[j0*R .. (j0+W)*R) are contiguous.
template <int LOGR, int W, int NT, bool DB>
__device__ __forceinline__ void store_transposed(const uint64_t* buf, uint64_t* out, uint64_t j0, int t,
                                                 const PassArgs& a) {
  constexpr int R = 1 << LOGR;
  constexpr int PER = (R * W) / NT;
  tile_barrier<DB>();
  uint64_t* o = out + j0 * R;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int m = t + NT * u;
    const uint64_t y = buf[(m / R) * (R + 1) + (m % R)];
    if (!PBF_DBG(a, 1) || y == 0x123456789ull) o[m] = y;
  }
}

// One Stockham pass over HBM, one tile per workgroup (tiles too large to double-buffer).
// NT threads, W columns of R = 2^LOGR points, register sub-DFTs of radix up to 2^LQ;
// E64 >= 0 selects shift twiddles for a standard Goldilocks root (w_64 = 2^E64).
// Waves per SIMD the pass kernels are register-budgeted for: as many as the LDS tile
// lets reside (R*W*8 bytes per workgroup of NT threads, 160 KiB per CU), at most 8.
__host__ __device__ constexpr int ntt_waves_per_eu(int e, int nt) {
  int per_cu = 163840 / (8 * e + 2048);
  if (per_cu < 1) per_cu = 1;
  int w = per_cu * (nt / 64) / 4;
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}

template <class F, int LOGR, int W, int NT, int LQ, int E64>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(ntt_waves_per_eu(W << LOGR, NT))))
ntt_pass_kernel(PassArgs a) {
  constexpr int R = 1 << LOGR;
  constexpr int E = R * W;
  constexpr int PER = E / NT;
  constexpr int QMAX = 1 << LQ;
  static_assert(LOGR >= LQ, "register sub-DFTs need R >= 2^LQ");
  static_assert(PER >= QMAX && PER % QMAX == 0, "each thread must own whole register sub-DFTs");
  static_assert(E <= 16384, "LDS budget: 128 KiB of elements per workgroup");
  // +W pad keeps the transposed [w][r] image of the first pass bank-conflict free
  __shared__ uint64_t lds[E + W];

  // Block order: with a pass-twiddle table, blocks of one XCD (blockIdx b, b+8, ... share
  // an L2) take a contiguous range of column blocks, all polynomials of a column block
  // back to back, so each slice of T[r][k] is fetched into that L2 once per pass instead
  // of once per polynomial (PMC: 387 -> ~260 MiB fetched per pass at 2^20 x 32).
  uint32_t poly, kb;
  if (a.xcd_kmajor) {
    const uint32_t v = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    kb = v / a.batch;
    poly = v % a.batch;
  } else {
    poly = blockIdx.x / a.blocks_per_poly;
    kb = blockIdx.x % a.blocks_per_poly;
  }
  const uint64_t j0 = (uint64_t)kb * W;
  const uint64_t* in = a.in + (uint64_t)poly * a.n;
  uint64_t* out = a.out + (uint64_t)poly * a.n;
  const int t = threadIdx.x;
  PassArgs b = a;
  b.cur_poly = poly;

  uint64_t wq[QMAX / 2];  // w_QMAX^m (table-twiddle variant only)
  if constexpr (E64 < 0) {
#pragma unroll
    for (int m = 0; m < QMAX / 2; ++m) wq[m] = a.rtab[m * (R / QMAX)];
  }
  uint64_t v[PER];
  tile_load<LOGR, W, NT, LQ>(v, a, in, j0, t);
  ntt_stage<F, LOGR, W, NT, LQ, E64, 0>(v, lds, a.rtab, wq, b, out, j0, t);
  if (a.log_ns == 0) store_transposed<LOGR, W, NT, false>(lds, out, j0, t, a);
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
static __global__ void shard_unsplit_kernel(const uint64_t* recv, uint64_t* out, uint64_t s, uint64_t nl, uint32_t batch,
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
