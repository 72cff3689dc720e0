// Goldilocks pass kernel for standard roots (gfx950) — the hot path of src/fft.rs
// CooleyTurkey (fft.rs:55-106) at BASELINE configs 2 and 5.
//
// Same Stockham-over-HBM pass structure as ntt_pass_kernel (ntt_kernels.hpp): pass input
// x[j + r*(n/R)], pre-twiddle w^((n/(Ns*R))*r*(j mod Ns)), an R-point DFT along r,
// output y[(j/Ns)*Ns*R + (j mod Ns) + k*Ns]. What differs is how the R-point DFT is
// split, chosen so that every general (table) multiplication that can be a shift is one:
//
//   R = 4 * 16 * C  (C = R/64),   r = 16C*s1 + C*s2 + r2,   k = q1 + 4*q2 + 64*k2
//   stage A  4-point DFT over s1                          -> Z[q1][s2][r2]
//   stage B  Z *= w_64^(s2*q1)  (a power of two: shift)   16-point DFT over s2
//                                                          -> Y[k1 = q1 + 4 q2][r2]
//   stage C  Y *= w_R^(r2*k1)   (table, general multiply)  C-point DFT over r2 -> X[k1 + 64 k2]
//
// For a standard root w (w_64 = 2^39, inverse 2^153) every root of order <= 64 is a
// power of two, so the 4-, 16- and C-point register DFTs and the stage-B twiddle are
// shift-reductions; only stage C's pre-twiddle (and the pass twiddle) multiply by
// table entries: one general multiplication per element per pass, the minimum for
// DFT blocks of <= 64 points (2^20 = 2 passes -> 3 general multiplications per
// element including the one pass twiddle; ntt_pass_kernel's 4|16|16 split needs 5).
//
// Stage B runs one q1 per wave (4 values, 2 waves each), so its twiddle exponents are
// compile-time constants under a wave-uniform switch. LDS layouts (elements of 8 B):
//   Z: ((q1*16 + s2)*C + r2)*W + w           (A writes and B reads 64 contiguous)
//   Y: r2*(65*W) + k1*W + w                  (B writes rows r2 padded by W: 2-pass
//                                             64-bit accesses; C reads contiguous)
// Tile: TILE = R x W elements (W = TILE/R columns: W*8 B contiguous runs in HBM), TILE/16
// threads, 16 elements per thread in every stage.
#pragma once
#include "ntt_kernels.hpp"

// Timing experiment only (make nomath): -DPBF_GL_NOMATH drops every twiddle multiply and
// register DFT of ntt_gl_pass_kernel, leaving its loads, LDS exchanges, barriers and
// stores: the data-movement floor of the kernel. Never the product build.
#ifdef PBF_GL_NOMATH
#define PBF_GL_MATH(x) do { } while (0)
#else
#define PBF_GL_MATH(x) x
#endif
// Timing experiment only (make nomem): every tile loads tile 0 of polynomial 0 (L2-resident)
// and stores only values equal to a sentinel that never occurs: the kernel's compute, LDS
// and barrier time without HBM traffic.
#ifdef PBF_GL_NOMEM
#define PBF_GL_NOMEM_ON 1
#else
#define PBF_GL_NOMEM_ON 0
#endif

namespace pbf {

struct GlPassArgs {
  const uint64_t* in;
  uint64_t* out;
  const uint64_t* twpass;  // per-pass [r][k] table w^((n/(Ns*R))*r*k), or null (two-level)
  const uint64_t* tw0;     // two-level table of w (low part)
  const uint64_t* tw1;     //                     (high part)
  const uint64_t* tc;      // stage-C table [r2][k1] = w_R^(r2*k1) (times n^-1 when scaled)
  const uint64_t* tws_a;   // last pass, split twiddles: A[r][w] = w_p^(r*w)   (or null)
  const uint64_t* tws_b;   //                          B[kb][r] = w_p^(r*kb*W)
  uint64_t n;
  uint32_t log_n;
  uint32_t log_ns;
  uint32_t tw_bits;
  uint32_t blocks_per_poly;
  uint32_t batch;
  uint32_t scaled;         // tc carries n^-1: multiply every element, k1 = 0 / r2 = 0 too
  uint32_t out_split_log;  // != 0: store destination-major [n/S][batch][S] (multi-GPU send layout)
  uint32_t xcd_kmajor;     // XCD-aware column-major block order (pass-twiddle table reuse in L2)
  uint64_t in_pitch, out_pitch;  // elements from one polynomial to the next
  // two-pass plans: the first pass multiplies its outputs by the second pass's twiddle w^(j k)
  // (post_tw = that pass's [r][k] table: r = this pass's column j, k its output digit) and the
  // second pass skips its own (skip_pass_tw)
  const uint64_t* post_tw;
  uint32_t skip_pass_tw;
};

// x * 2^(K mod 192) (mod p), K a compile-time exponent; 2^96 = -1. Exponents in
// (160, 192) are divisions by 2^(192-K) (no sign); a remaining sign costs one subtraction.
template <int K>
__device__ __forceinline__ uint64_t gl_pow2(uint64_t x) {
  constexpr int RAW = ((K % 192) + 192) % 192;
  if constexpr (RAW == 0) {
    return x;
  } else if constexpr (RAW > 160) {
    return gl_div_pow2<192 - RAW>(x);
  } else {
    using T = ShiftKind<RAW>;
    const uint64_t y = apply_shift<Goldilocks, T>(x);
    if constexpr (T::NEG) {
      const FieldArgs f{};
      return Goldilocks::sub(0, y, f);
    } else {
      return y;
    }
  }
}

// Stage-B twiddle: v[s2] *= w_64^(s2*Q1) = 2^(E64*s2*Q1).
template <int E64, int Q1, int S2 = 1>
__device__ __forceinline__ void gl_stage_b_twiddle(uint64_t* v) {
  if constexpr (S2 < 16) {
    v[S2] = gl_pow2<(E64 * S2 * Q1) % 192>(v[S2]);
    gl_stage_b_twiddle<E64, Q1, S2 + 1>(v);
  }
}

// v[bitrev4(e)] *= w_64^(e*Q) = 2^(E64*e*Q): a twiddle on the bit-reversed outputs of a
// 16-point register DFT
template <int E64, int Q, int E = 1>
__device__ __forceinline__ void gl_post_twiddle_br(uint64_t* v) {
  if constexpr (E < 16) {
    v[bitrev_c(E, 4)] = gl_pow2<(E64 * E * Q) % 192>(v[bitrev_c(E, 4)]);
    gl_post_twiddle_br<E64, Q, E + 1>(v);
  }
}
// RG 3 stage C: x[u*4 + r2] *= w_64^(r2 g), g = WV + 4 u (r2 = 1..3, u = 0..3)
template <int E64, int WV, int U = 0>
__device__ __forceinline__ void gl_rg3_c_shift(uint64_t* x) {
  if constexpr (U < 4) {
    constexpr int g = WV + 4 * U;
    x[U * 4 + 1] = gl_pow2<(E64 * g) % 192>(x[U * 4 + 1]);
    x[U * 4 + 2] = gl_pow2<(E64 * 2 * g) % 192>(x[U * 4 + 2]);
    x[U * 4 + 3] = gl_pow2<(E64 * 3 * g) % 192>(x[U * 4 + 3]);
    gl_rg3_c_shift<E64, WV, U + 1>(x);
  }
}

template <int LOGR, int TILE>
struct GlShape {
  static constexpr int R = 1 << LOGR;
  static constexpr int LOGC = LOGR - 6;
  static constexpr int C = 1 << LOGC;
  static constexpr int W = TILE / R;
  static constexpr int NT = TILE / 16;             // 16 elements per thread
  static constexpr int WPQ = NT / 256;              // waves per stage-B q1 value
  // Y rows r2: padded by W (YP = 65 W) so that the four r2 rows of one stage-B write
  // instruction fall on both halves of the banks; for W = 16 the same spread comes from
  // XOR-ing k1's low bit with r2's (YX: no padding, a 4096-element tile is exactly 32 KiB and
  // five workgroups fit a CU; PBF_GL_PAD_Y builds the padded layout for A/B)
#ifdef PBF_GL_PAD_Y
  static constexpr bool YX = false;
#else
  static constexpr bool YX = W == 16 && C > 1;
#endif
  static constexpr int YP = (YX ? 64 : 65) * W;     // Y row pitch (elements)
  static constexpr int LDS = (C * YP > TILE) ? C * YP : TILE;
  static constexpr bool LDS32K = LDS * 8 <= 32768;  // five workgroups per CU by LDS
  static constexpr int NSUB_C = (64 * W) / NT;      // stage-C sub-DFTs per thread
  // Y column swizzle: the first pass's stage C reads all 64 k1 of one column w per wave
  // (so its stores are 512-B runs of out[j*R + k]); w ^ ysw(k1) spreads those reads over
  // the banks, each 8-B bank pair hit twice per 512-B wave access (the minimum). Stage B's
  // writes and later passes' reads stay permutations within a row (conflict-free).
  __host__ __device__ static constexpr int ysw(int k1) {
    return W <= 32 ? (k1 / (32 / W)) & (W - 1) : (k1 & 31);
  }
  // Y element (r2, k1, w)
  __host__ __device__ static constexpr int yidx(int r2, int k1, int w) {
    return r2 * YP + (YX ? (k1 ^ (r2 & 1)) : k1) * W + (w ^ ysw(k1));
  }
};

// Tile id -> (polynomial, column block). With xcd_kmajor the tiles of one XCD (block ids
// congruent mod 8) take a contiguous range
// of column blocks, all polynomials of a block back to back, so each slice of the
// pass-twiddle table is fetched into that XCD's L2 once per pass, not once per polynomial.
__device__ __forceinline__ void gl_tile_coords(const GlPassArgs& a, uint32_t tile, uint32_t tiles, uint32_t* poly,
                                               uint32_t* kb) {
  if (a.xcd_kmajor == 1) {
    const uint32_t v = (tile & 7) * (tiles >> 3) + (tile >> 3);
    *kb = v / a.batch;
    *poly = v % a.batch;
  } else if (a.xcd_kmajor == 2) {
    // XCD-blocked, polynomial-major: workgroups resident together on one XCD take adjacent
    // column blocks, so the 128-B lines their W*8-B runs share are fetched into one L2
    const uint32_t v = (tile & 7) * (tiles >> 3) + (tile >> 3);
    *poly = v / a.blocks_per_poly;
    *kb = v % a.blocks_per_poly;
  } else {
    *poly = tile / a.blocks_per_poly;
    *kb = tile % a.blocks_per_poly;
  }
}

constexpr int GL_STORES = 16;  // global stores per thread per tile (NSUB_C * C)

// One tile: stages A, B, C and the stores.
// RG (regrouped 2^24 plan, ntt_gl_rg2_kernel below): 1 = its first pass, 3 = its last pass.
template <int LOGR, int E64, bool FIRST, int TILE, int RG = 0>
__device__ __forceinline__ void gl_tile(const GlPassArgs& a, uint64_t* lds, uint32_t tile, uint32_t tiles, int t) {
  using Sh = GlShape<LOGR, TILE>;
  constexpr int C = Sh::C, LOGC = Sh::LOGC, W = Sh::W, NT = Sh::NT, YP = Sh::YP;
  (void)YP;
  static_assert(Sh::NSUB_C * C == GL_STORES, "stores per thread");
  static_assert(RG == 0 || (LOGR == 8 && TILE == 4096 && FIRST == (RG == 1)), "RG shape");
  const FieldArgs f{};
  using G = Goldilocks;
  uint32_t poly, kb;
  gl_tile_coords(a, tile, tiles, &poly, &kb);
  if constexpr (PBF_GL_NOMEM_ON) kb &= 1, poly = 0;
  const uint64_t j0 = (uint64_t)kb * W;
  const uint64_t* in = a.in + (uint64_t)poly * a.in_pitch;
  const uint64_t stride = a.n >> LOGR;  // input rows (r) are n/R long

  // ---------------- stage A: load, pass twiddle, 4-point DFTs over s1
  uint64_t v[16];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = t + NT * u;
    const int w = idx % W, r2 = (idx / W) % C, s2 = idx / (C * W);
#pragma unroll
    for (int s1 = 0; s1 < 4; ++s1) {
      const int r = 16 * C * s1 + C * s2 + r2;
      v[u * 4 + s1] = in[(j0 + w) + (uint64_t)r * stride];
    }
  }
  // RG 3: the stage-B general twiddle w^(a0 X) (a0 = r2 + 4 s2, X = 65536 q1 + j), geometric in
  // s2: C[r2][X] D[X]^s2 with C = w^(r2 X), D = w^(4 X) (tws_a, tws_b); C and D are loaded now
  // (in flight during stage A) in the stage-B thread mapping, the powers formed in stage B
  uint64_t t3[RG == 3 ? 2 : 1];
  if constexpr (RG == 3) {
    const int wave = t >> 6, q1 = wave / Sh::WPQ, rw = (wave % Sh::WPQ) * 64 + (t & 63);
    const int r2 = rw / W, w = rw % W;
    const uint64_t X = ((uint64_t)q1 << 16) + j0 + w;
    t3[0] = a.tws_a[((uint64_t)r2 << 18) + X];
    t3[1] = a.tws_b[X];
  }
  if constexpr (!FIRST && RG != 3) if (!a.skip_pass_tw) {
    const uint64_t kmask = (1ull << a.log_ns) - 1;
    // in groups of 8 elements (loads of a group issue back to back; bounded live registers)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint64_t tw[8];
#pragma unroll
      for (int uu = 0; uu < 2; ++uu) {
        const int u = 2 * h + uu;
        const int idx = t + NT * u;
        const int w = idx % W, r2 = (idx / W) % C, s2 = idx / (C * W);
        const uint64_t k = (j0 + w) & kmask;
#pragma unroll
        for (int s1 = 0; s1 < 4; ++s1) {
          const uint64_t r = (uint64_t)(16 * C * s1 + C * s2 + r2);
          if (a.twpass) {
            tw[uu * 4 + s1] = a.twpass[(r << a.log_ns) + k];
          } else if (a.tws_a) {  // last pass: k = kb*W + w
            tw[uu * 4 + s1] = G::mul(a.tws_b[(uint64_t)kb * Sh::R + r], a.tws_a[r * W + w], f);
          } else {
            const uint64_t e = ((r * k) << (a.log_n - a.log_ns - LOGR)) & (a.n - 1);
            tw[uu * 4 + s1] = G::mul(a.tw0[e & ((1ull << a.tw_bits) - 1)], a.tw1[e >> a.tw_bits], f);
          }
        }
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) PBF_GL_MATH(v[8 * h + m] = G::mul(v[8 * h + m], tw[m], f));
#ifdef PBF_GL_NOMATH
#pragma unroll
      for (int m = 0; m < 8; ++m) v[8 * h + m] ^= tw[m];
#endif
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) PBF_GL_MATH((dft_reg<G, 2, sub_root_exp(E64, 2)>(v + u * 4, nullptr, f)));
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = t + NT * u;  // = s2*(C*W) + (r2*W + w)
    const int s2 = idx / (C * W), rw = idx % (C * W);
#pragma unroll
    for (int q1 = 0; q1 < 4; ++q1) lds[(q1 * 16 + s2) * (C * W) + rw] = v[u * 4 + bitrev_c(q1, 2)];
  }
  __syncthreads();

  // ---------------- stage B: one q1 per wave; shift twiddles; 16-point DFT over s2
  {
    const int wave = t >> 6;
    const int q1 = wave / Sh::WPQ;
    const int rw = (wave % Sh::WPQ) * 64 + (t & 63);  // r2*W + w
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) v[s2] = lds[(q1 * 16 + s2) * (C * W) + rw];
#ifndef PBF_GL_NOMATH
    if constexpr (RG == 3) {
      uint64_t p = t3[0];
      const uint64_t d = t3[1];
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        v[s2] = G::mul(v[s2], p, f);
        if (s2 < 15) p = G::mul(p, d, f);
      }
    } else {
      switch (__builtin_amdgcn_readfirstlane(q1)) {
        case 1: gl_stage_b_twiddle<E64, 1>(v); break;
        case 2: gl_stage_b_twiddle<E64, 2>(v); break;
        case 3: gl_stage_b_twiddle<E64, 3>(v); break;
        default: break;
      }
    }
    dft_reg<G, 4, sub_root_exp(E64, 4)>(v, nullptr, f);
#endif
    __syncthreads();
    const int r2 = rw / W, w = rw % W;
#pragma unroll
    for (int q2 = 0; q2 < 16; ++q2) {
      const int k1 = q1 + 4 * q2;
      lds[Sh::yidx(r2, k1, w)] = v[bitrev_c(q2, 4)];
    }
  }
  __syncthreads();

  // ---------------- stage C: table twiddle w_R^(r2*k1); C-point DFT over r2
  // sub-DFT (k1, w) of thread t: FIRST pass all 64 k1 of one column per wave (512-B runs
  // of k in the output rows out[j*R + k]); later passes w fastest (W-element runs of j)
  auto c_map = [&](int u, int* k1, int* w) {
    const int idx = t + NT * u;
    if constexpr (FIRST) {
      *k1 = idx & 63;
      *w = idx >> 6;
    } else {
      *k1 = idx / W;
      *w = idx % W;
    }
  };
  uint64_t x[Sh::NSUB_C * C];
#pragma unroll
  for (int u = 0; u < Sh::NSUB_C; ++u) {
    int k1, w;
    c_map(u, &k1, &w);
#pragma unroll
    for (int r2 = 0; r2 < C; ++r2) x[u * C + r2] = lds[Sh::yidx(r2, k1, w)];
  }
  if constexpr (RG == 3) {
    // w_64^(r2 g), g = k1 >> 2 = wave + 4 u (4-wave tiles, W = 16): wave-uniform shifts
    switch (__builtin_amdgcn_readfirstlane(t >> 6)) {
      case 0: gl_rg3_c_shift<E64, 0>(x); break;
      case 1: gl_rg3_c_shift<E64, 1>(x); break;
      case 2: gl_rg3_c_shift<E64, 2>(x); break;
      default: gl_rg3_c_shift<E64, 3>(x); break;
    }
  } else if constexpr (RG == 1) {
    // tc[a2l][r2][k1] = w_4096^((a2l + 16 r2) k1), a2l = bits 12..15 of the column: every row
    const uint64_t* tc = a.tc + ((j0 >> 12) & 15) * 256;
#pragma unroll
    for (int u = 0; u < Sh::NSUB_C; ++u) {
      int k1, w;
      c_map(u, &k1, &w);
      uint64_t tw[C];
#pragma unroll
      for (int r2 = 0; r2 < C; ++r2) tw[r2] = tc[r2 * 64 + k1];
#pragma unroll
      for (int r2 = 0; r2 < C; ++r2) x[u * C + r2] = G::mul(x[u * C + r2], tw[r2], f);
    }
  } else {
    uint64_t tw[Sh::NSUB_C * C];
    const int r2lo = a.scaled ? 0 : 1;  // scaled table carries n^-1: every element multiplies
#pragma unroll
    for (int u = 0; u < Sh::NSUB_C; ++u) {
      int k1, w;
      c_map(u, &k1, &w);
#pragma unroll
      for (int r2 = 0; r2 < C; ++r2) tw[u * C + r2] = (r2 >= r2lo) ? a.tc[r2 * 64 + k1] : 1;
    }
    if (a.scaled) {
#pragma unroll
      for (int m = 0; m < Sh::NSUB_C * C; ++m) PBF_GL_MATH(x[m] = G::mul(x[m], tw[m], f));
    } else {
      // r2 = 0 rows multiply by 1 and are skipped; k1 = 0 lanes multiply by 1 (a per-lane
      // branch would only diverge)
#pragma unroll
      for (int u = 0; u < Sh::NSUB_C; ++u)
#pragma unroll
        for (int r2 = 1; r2 < C; ++r2) {
          PBF_GL_MATH(x[u * C + r2] = G::mul(x[u * C + r2], tw[u * C + r2], f));
#ifdef PBF_GL_NOMATH
          x[u * C + r2] ^= tw[u * C + r2];
#endif
        }
    }
  }
  if constexpr (C > 1) {
#pragma unroll
    for (int u = 0; u < Sh::NSUB_C; ++u) PBF_GL_MATH((dft_reg<G, LOGC, sub_root_exp(E64, LOGC)>(x + u * C, nullptr, f)));
  }

  // ---------------- store
  if constexpr (FIRST) {
    uint64_t* o = a.out + (uint64_t)poly * a.out_pitch;
#pragma unroll
    for (int u = 0; u < Sh::NSUB_C; ++u) {
      int k1, w;
      c_map(u, &k1, &w);
      const uint64_t base = (j0 + w) << LOGR;
      if (a.post_tw) {
        uint64_t tw[C];
#pragma unroll
        for (int k2 = 0; k2 < C; ++k2) tw[k2] = a.post_tw[base + k1 + 64 * k2];
#pragma unroll
        for (int k2 = 0; k2 < C; ++k2) x[u * C + bitrev_c(k2, LOGC)] = G::mul(x[u * C + bitrev_c(k2, LOGC)], tw[k2], f);
      }
#pragma unroll
      for (int k2 = 0; k2 < C; ++k2)
        if (!PBF_GL_NOMEM_ON || x[u * C + bitrev_c(k2, LOGC)] == 0x123456789ull)
          o[base + k1 + 64 * k2] = x[u * C + bitrev_c(k2, LOGC)];
    }
  } else {
    const uint64_t ns_mask = (1ull << a.log_ns) - 1;
    uint64_t* out = a.out + (uint64_t)poly * a.out_pitch;
    const uint32_t sl = a.out_split_log;
#pragma unroll
    for (int u = 0; u < Sh::NSUB_C; ++u) {
      int k1, w;
      c_map(u, &k1, &w);
      const uint64_t j = j0 + w;
      const uint64_t base = ((j >> a.log_ns) << (a.log_ns + LOGR)) + (j & ns_mask);
      if (sl == 0) {
#pragma unroll
        for (int k2 = 0; k2 < C; ++k2)
          if (!PBF_GL_NOMEM_ON || x[u * C + bitrev_c(k2, LOGC)] == 0x123456789ull)
            out[base + ((uint64_t)(k1 + 64 * k2) << a.log_ns)] = x[u * C + bitrev_c(k2, LOGC)];
      } else {
        const uint64_t smask = (1ull << sl) - 1;
#pragma unroll
        for (int k2 = 0; k2 < C; ++k2) {
          const uint64_t kk = base + ((uint64_t)(k1 + 64 * k2) << a.log_ns);
          a.out[((((kk >> sl) * a.batch) + poly) << sl) + (kk & smask)] = x[u * C + bitrev_c(k2, LOGC)];
        }
      }
    }
  }
}

template <int LOGR, int TILE>
__device__ __forceinline__ void gl_shape_checks() {
  using Sh = GlShape<LOGR, TILE>;
  static_assert(LOGR >= 6 && LOGR <= 10, "radix 2^6 .. 2^10");
  static_assert(Sh::LDS * 8 <= (TILE > 8192 ? 160 : 80) * 1024, "LDS budget");
  static_assert(Sh::W >= 8 && Sh::WPQ >= 1, "tile shape");
}

// One tile per workgroup.
template <int LOGR, int E64, bool FIRST, int TILE, int RG = 0>
// waves per SIMD the VGPR budget allows: 5 where the LDS allows five workgroups and the
// kernel fits 96 VGPRs without spilling (first passes and the regrouped plan's), else 4
__global__ void __launch_bounds__(TILE / 16)
__attribute__((amdgpu_waves_per_eu((FIRST || RG) && GlShape<LOGR, TILE>::LDS32K ? 5 : 4)))
ntt_gl_pass_kernel(GlPassArgs a) {
  gl_shape_checks<LOGR, TILE>();
  __shared__ __attribute__((aligned(16))) uint64_t lds[GlShape<LOGR, TILE>::LDS];
  const uint32_t tiles = a.blocks_per_poly * a.batch;
  gl_tile<LOGR, E64, FIRST, TILE, RG>(a, lds, blockIdx.x, tiles, threadIdx.x);
}

// ---- regrouped 2^24 plan (DESIGN.md §3.1 "Regrouped twiddles") --------------------------
// The three radix-2^8 passes of a 2^24 transform re-cut so that every general (table)
// twiddle sits between DFT blocks of 64 points: with the index bits in four groups of six,
// j = a0 + 64 a1 + 4096 a2 + 2^18 a3 and k = b0 + 64 b1 + 4096 b2 + 2^18 b3, decimation in
// frequency needs only the three twiddle layers w^(4096 a2 b0), w^(64 a1 (b0 + 64 b1)) and
// w^(a0 (b0 + 64 b1 + 4096 b2)); each 64-point group DFT that straddles two passes is split
// 4 x 16 or 16 x 4 with a w_64 (shift) twiddle between its halves. Per element that is 3
// general multiplications for the whole transform instead of 4.25 (0.75 + 1.75 + 1.75):
//   pass 1 (RG 1): DFT-64 over a3 | w_4096^(a2 b0) (a2l = bits 12..15 of the column) | DFT-4
//   pass 2 (this kernel): w_64^(a2l c) | DFT-16 over a2l | T2[a1][K] | DFT-16 over a1h | w_64^(a1l e)
//   pass 3 (RG 3): DFT-4 over a1l | w^(a0 X) = C[r2][X] D[X]^s2 | DFT-16 | w_64^(r2 g) | DFT-4
// Pass 2 needs one LDS exchange (two 16-point stages), not two. Data stays in the Stockham
// layout of the other passes (natural order in and out).
// Pass 2 tile: 256 rows r = 16 a2l + a1h x W = 16 columns j (Ns = 256: j mod 256 = b0 + 64 c,
// the first pass's output digit; bits 14..15 of j = a1l); stage X thread (a1h, w), stage Y
// thread (d, w); LDS [d][a1h ^ (d mod 4)][w] (the XOR spreads the stage-Y reads of four d per
// wave over both halves of the banks: every bank pair is hit exactly twice, the minimum).
template <int E64>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) ntt_gl_rg2_kernel(GlPassArgs a) {
  constexpr int W = 16;
  // 32 KiB; four waves per SIMD: at five the 96-VGPR budget spills 28 B per lane and the pass
  // runs ~2 % slower (profiles/r03/ntt_lds_ab.log)
  __shared__ __attribute__((aligned(16))) uint64_t lds[16 * 16 * W];
  const FieldArgs f{};
  using G = Goldilocks;
  const uint32_t tiles = a.blocks_per_poly * a.batch;
  uint32_t poly, kb;
  gl_tile_coords(a, blockIdx.x, tiles, &poly, &kb);
  const int t = threadIdx.x, w = t % W, a1h = t / W;
  const uint64_t j0 = (uint64_t)kb * W, j = j0 + w;
  const uint32_t c = (uint32_t)(j0 >> 6) & 3, a1l = (uint32_t)(j0 >> 14) & 3;
  const uint64_t* in = a.in + (uint64_t)poly * a.in_pitch;
  const uint64_t stride = a.n >> 8;
  uint64_t v[16], tw[16];
#pragma unroll
  for (int a2l = 0; a2l < 16; ++a2l) v[a2l] = in[j + (uint64_t)(a2l * 16 + a1h) * stride];
  // T2[a1][K] = w^(64 a1 K), a1 = a1l + 4 a1h, K = b0 + 64 b1 = (j mod 256) + 256 d (2 MiB,
  // L2-resident; the geometric form T2[a1][j mod 256] (w^(16384 a1))^d measured 1.5 % slower in
  // round 5, profiles/r05/t2geo_ab.log)
  const uint64_t* t2 = a.twpass + ((uint64_t)(a1l + 4 * a1h) << 12) + (j & 255);
#pragma unroll
  for (int d = 0; d < 16; ++d) tw[d] = t2[256 * d];
  switch (__builtin_amdgcn_readfirstlane(c)) {  // w_64^(a2l c)
    case 1: gl_stage_b_twiddle<E64, 1>(v); break;
    case 2: gl_stage_b_twiddle<E64, 2>(v); break;
    case 3: gl_stage_b_twiddle<E64, 3>(v); break;
    default: break;
  }
  dft_reg<G, 4, sub_root_exp(E64, 4)>(v, nullptr, f);  // output d at v[bitrev4(d)]
#pragma unroll
  for (int d = 0; d < 16; ++d) lds[d * 256 + (a1h ^ (d & 3)) * W + w] = G::mul(v[bitrev_c(d, 4)], tw[d], f);
  __syncthreads();
  const int d2 = t / W;
#pragma unroll
  for (int h = 0; h < 16; ++h) v[h] = lds[d2 * 256 + (h ^ (d2 & 3)) * W + w];
  dft_reg<G, 4, sub_root_exp(E64, 4)>(v, nullptr, f);  // output e at v[bitrev4(e)]
  switch (__builtin_amdgcn_readfirstlane(a1l)) {  // w_64^(a1l e)
    case 1: gl_post_twiddle_br<E64, 1>(v); break;
    case 2: gl_post_twiddle_br<E64, 2>(v); break;
    case 3: gl_post_twiddle_br<E64, 3>(v); break;
    default: break;
  }
  // output digit k = d + 16 e of the Stockham pass (Ns = 256)
  uint64_t* out = a.out + (uint64_t)poly * a.out_pitch;
  const uint64_t base = ((j >> 8) << 16) + (j & 255);
#pragma unroll
  for (int e = 0; e < 16; ++e) out[base + ((uint64_t)(d2 + 16 * e) << 8)] = v[bitrev_c(e, 4)];
}

}  // namespace pbf
