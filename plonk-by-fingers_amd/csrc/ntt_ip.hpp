// Goldilocks NTT, round-3 schedule: in-place digit slots, persistent workgroups with a
// register prefetch of the next tile (gfx950). Same transform as ntt_gl.hpp (src/fft.rs
// CooleyTurkey, fft.rs:55-106: natural order in and out, X_k = sum_j a_j w^(jk)), same
// in-register radix-R DFT (stages A / B / C of ntt_gl.hpp), different data movement:
//
//  * Digit slots. n = 2^L, passes of radix 2^r_0, 2^r_1, ... (top slot first). Pass i owns
//    position bits [lo_i, lo_i + r_i) and writes its output digit k_i back into those bits
//    ("column pass": every tile reads and writes the same addresses), so one scratch buffer
//    S carries every intermediate. The last pass ("row pass", lo = 0) reads rows of R
//    contiguous elements and writes the natural-order output X[K + (n/R) k], K = the
//    earlier output digits (k_0 least significant). In HBM every access is a run of
//    W elements (W * 8 >= 64 B) or a whole row.
//  * Twiddles. Pass i >= 1 multiplies input x of a tile by w^(2^lo_i x K): for a column
//    pass K is fixed per tile (one R-entry row of T_i[h][x], h = the tile's high position
//    bits); the row pass needs w^(x K) for W consecutive K: from a full table T[K][x] when
//    the batch shares it (n <= 2^20: 8 MiB) or as TB[K/W][x] * TA[x][K mod W] (one more
//    product, tables of n/W and R*W entries) -- never the 2^24-entry, 128 MiB table the
//    round-2 plan read in its last pass. The inverse folds n^-1 into the row pass's table.
//  * Persistence and prefetch. A workgroup walks tiles blockIdx.x, +gridDim.x, ...; right
//    after a tile's stage A has moved its data to LDS it issues the next tile's 16 global
//    loads per thread into spare registers, so they are in flight during stages B and C and
//    the stores (the stage-C table lives in LDS, so no later vmcnt wait drains them).
//  * XCD-aware order. Logical tile t of a launch goes to XCD t mod 8 (round-robin dispatch,
//    MI355X_MICROARCH.md) and each XCD takes a contiguous range of (block, polynomial)
//    tiles: adjacent column blocks -- whose W-element runs share 128-B lines -- and every
//    polynomial of one twiddle row run together on one XCD's L2.
// Data-movement floors of these schedules against round 2's (scripts/ubench/ntt_floor.hip,
// profiles/r03/ntt_floor_*.log): 2 x 2^24 three passes 266 us (Stockham 334 us).
#pragma once
#include "ntt_gl.hpp"

namespace pbf {

constexpr int IP_MAXP = 4;

struct IpArgs {
  const uint64_t* in;
  uint64_t* out;
  const uint64_t* tw;   // column pass i >= 1: T[h][x]; row pass: T[K][x] (full) or TB[K/W][x] (split)
  const uint64_t* twa;  // row pass, split form: TA[x][w]; null otherwise
  const uint64_t* tc;   // stage-C table w_R^(r2 k1) (C x 64), copied to LDS once per workgroup
  uint64_t pitch_in, pitch_out;  // polynomial strides (elements)
  uint32_t lo;          // column pass: slot low bit
  uint32_t ncb_log;     // column pass: log2(column blocks) = lo - log2(W)
  uint32_t blocks;      // tiles per polynomial
  uint32_t batch;
  uint32_t tiles;       // blocks * batch
  uint32_t xcd;         // tiles % 8 == 0: XCD-contiguous tile ranges
  uint32_t nd;          // row pass: digits of K (passes before it)
  uint32_t dr[IP_MAXP], dlo[IP_MAXP];  // row pass: radix bits / slot low bit of those passes
  uint32_t out_log;     // row pass: log2(n / R)
  uint32_t prime;       // persistent kernels: entry stores that align the loop's wait counts
};

// Workgroup barrier that leaves global loads in flight: __syncthreads() would also wait for
// vmcnt(0) and drain the next tile's prefetch (and this tile's stores).
__device__ __forceinline__ void ip_bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// tile -> (polynomial, block): block-major, polynomial inner (a block's twiddle row is
// shared by the whole batch), XCD-contiguous ranges
__device__ __forceinline__ void ip_coords(const IpArgs& a, uint32_t tile, uint32_t* poly, uint32_t* blk) {
  if (a.xcd) tile = (tile & 7) * (a.tiles >> 3) + (tile >> 3);
  *blk = tile / a.batch;
  *poly = tile % a.batch;
}

// row pass: input position of column K's row (x = 0): sum_j digit_j(K) << dlo_j
__device__ __forceinline__ uint64_t ip_row_base(const IpArgs& a, uint32_t K) {
  uint64_t pos = 0;
  uint32_t sh = 0;
#pragma unroll
  for (int j = 0; j < IP_MAXP; ++j)
    if (j < (int)a.nd) {
      pos += (uint64_t)((K >> sh) & ((1u << a.dr[j]) - 1)) << a.dlo[j];
      sh += a.dr[j];
    }
  return pos;
}

template <int LOGR, int TILE>
struct IpShape : GlShape<LOGR, TILE> {
  using B = GlShape<LOGR, TILE>;
  static constexpr int DATA = TILE > B::LDS ? TILE : B::LDS;  // elements
  static constexpr int TC = B::C * 64;                         // stage-C table entries
  // row pass raw image: element (x, w) at x*W + (w ^ rsw(x)). Its writes (16 lanes along x,
  // one w) and stage A's reads (lanes along w) both hit distinct bank pairs.
  __host__ __device__ static constexpr int rsw(int x) {
    return B::W >= 16 ? (x & 15) : ((x >> (B::W == 8 ? 1 : (B::W == 4 ? 2 : 3))) & (B::W - 1));
  }
};

// The tile's 16 raw loads per thread. Column pass: stage-A order (element (x, w) with
// x = 16C s1 + C s2 + r2, w fastest across lanes: W-element runs). Row pass: lanes along x
// (each wave-instruction one 512-B piece of a row), stage A reads them back through LDS.
template <int LOGR, int TILE, bool ROW>
__device__ __forceinline__ void ip_load(const IpArgs& a, uint32_t tile, int t, uint64_t* v) {
  using Sh = GlShape<LOGR, TILE>;
  constexpr int C = Sh::C, W = Sh::W, NT = Sh::NT, R = Sh::R;
  uint32_t poly, blk;
  ip_coords(a, tile, &poly, &blk);
  const uint64_t* in = a.in + (uint64_t)poly * a.pitch_in;
  if constexpr (!ROW) {
    const uint32_t cb = blk & ((1u << a.ncb_log) - 1), h = blk >> a.ncb_log;
    const uint64_t base = (uint64_t)cb * W + ((uint64_t)h << (a.lo + LOGR));
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = t + NT * u;
      const int w = idx % W, r2 = (idx / W) % C, s2 = idx / (C * W);
#pragma unroll
      for (int s1 = 0; s1 < 4; ++s1) {
        const int x = 16 * C * s1 + C * s2 + r2;
        v[u * 4 + s1] = in[base + w + ((uint64_t)x << a.lo)];
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int idx = t + NT * u;
      const int x = idx % R, w = idx / R;
      v[u] = in[ip_row_base(a, blk * W + w) + x];
    }
  }
}

template <int LOGR, int E64, int KIND, int TILE, bool SPLIT>
__device__ __forceinline__ void ip_tile(const IpArgs& a, uint64_t* lds, const uint64_t* tcl, uint32_t tile, int t,
                                        uint64_t* v) {
  using Sh = IpShape<LOGR, TILE>;
  constexpr int C = Sh::C, LOGC = Sh::LOGC, W = Sh::W, NT = Sh::NT, YP = Sh::YP, R = Sh::R;
  (void)LOGC;
  (void)YP;
  constexpr bool ROW = KIND == 2;
  const FieldArgs f{};
  using G = Goldilocks;
  uint32_t poly, blk;
  ip_coords(a, tile, &poly, &blk);

  // ---------------- stage A: (row pass: raw image -> stage-A order), pass twiddle, 4-point DFTs
  if constexpr (ROW) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int idx = t + NT * u;
      const int x = idx % R, w = idx / R;
      lds[x * W + (w ^ Sh::rsw(x))] = v[u];
    }
    ip_bar();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = t + NT * u;
      const int w = idx % W, r2 = (idx / W) % C, s2 = idx / (C * W);
#pragma unroll
      for (int s1 = 0; s1 < 4; ++s1) {
        const int x = 16 * C * s1 + C * s2 + r2;
        v[u * 4 + s1] = lds[x * W + (w ^ Sh::rsw(x))];
      }
    }
  }
  if constexpr (KIND >= 1) {
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      uint64_t tw[8];
#pragma unroll
      for (int uu = 0; uu < 2; ++uu) {
        const int u = 2 * h2 + uu;
        const int idx = t + NT * u;
        const int w = idx % W, r2 = (idx / W) % C, s2 = idx / (C * W);
#pragma unroll
        for (int s1 = 0; s1 < 4; ++s1) {
          const uint32_t x = 16 * C * s1 + C * s2 + r2;
          if constexpr (!ROW) {
            tw[uu * 4 + s1] = a.tw[((uint64_t)(blk >> a.ncb_log) << LOGR) + x];
          } else if constexpr (!SPLIT) {
            tw[uu * 4 + s1] = a.tw[((uint64_t)(blk * W + w) << LOGR) + x];
          } else {
            tw[uu * 4 + s1] = G::mul(a.tw[((uint64_t)blk << LOGR) + x], a.twa[x * W + w], f);
          }
        }
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) v[8 * h2 + m] = G::mul(v[8 * h2 + m], tw[m], f);
    }
  }
  if constexpr (ROW) ip_bar();  // raw image consumed before Z overwrites it
#pragma unroll
  for (int u = 0; u < 4; ++u) dft_reg<G, 2, sub_root_exp(E64, 2)>(v + u * 4, nullptr, f);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = t + NT * u;
    const int s2 = idx / (C * W), rw = idx % (C * W);
#pragma unroll
    for (int q1 = 0; q1 < 4; ++q1) lds[(q1 * 16 + s2) * (C * W) + rw] = v[u * 4 + bitrev_c(q1, 2)];
  }
}

// stages B and C and the stores (after ip_tile's stage A; the caller may issue the next
// tile's loads in between)
template <int LOGR, int E64, int KIND, int TILE>
__device__ __forceinline__ void ip_tile_bc(const IpArgs& a, uint64_t* lds, const uint64_t* tcl, uint32_t tile, int t) {
  using Sh = IpShape<LOGR, TILE>;
  constexpr int C = Sh::C, LOGC = Sh::LOGC, W = Sh::W, NT = Sh::NT, YP = Sh::YP;
  (void)YP;
  constexpr bool ROW = KIND == 2;
  const FieldArgs f{};
  using G = Goldilocks;
  uint32_t poly, blk;
  ip_coords(a, tile, &poly, &blk);
  ip_bar();
  // ---------------- stage B: one q1 per wave; shift twiddles; 16-point DFT over s2
  {
    uint64_t v[16];
    const int wave = t >> 6;
    const int q1 = wave / Sh::WPQ;
    const int rw = (wave % Sh::WPQ) * 64 + (t & 63);  // r2*W + w
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) v[s2] = lds[(q1 * 16 + s2) * (C * W) + rw];
    switch (__builtin_amdgcn_readfirstlane(q1)) {
      case 1: gl_stage_b_twiddle<E64, 1>(v); break;
      case 2: gl_stage_b_twiddle<E64, 2>(v); break;
      case 3: gl_stage_b_twiddle<E64, 3>(v); break;
      default: break;
    }
    dft_reg<G, 4, sub_root_exp(E64, 4)>(v, nullptr, f);
    ip_bar();
    const int r2 = rw / W, w = rw % W;
#pragma unroll
    for (int q2 = 0; q2 < 16; ++q2) {
      const int k1 = q1 + 4 * q2;
      lds[Sh::yidx(r2, k1, w)] = v[bitrev_c(q2, 4)];
    }
  }
  ip_bar();
  // ---------------- stage C: w_R^(r2 k1) (LDS table); C-point DFT over r2; stores
  uint64_t x[Sh::NSUB_C * C];
#pragma unroll
  for (int u = 0; u < Sh::NSUB_C; ++u) {
    const int idx = t + NT * u;
    const int k1 = idx / W, w = idx % W;
#pragma unroll
    for (int r2 = 0; r2 < C; ++r2) x[u * C + r2] = lds[Sh::yidx(r2, k1, w)];
#pragma unroll
    for (int r2 = 1; r2 < C; ++r2) x[u * C + r2] = G::mul(x[u * C + r2], tcl[r2 * 64 + k1], f);
  }
  if constexpr (C > 1) {
#pragma unroll
    for (int u = 0; u < Sh::NSUB_C; ++u) dft_reg<G, LOGC, sub_root_exp(E64, LOGC)>(x + u * C, nullptr, f);
  }
  uint64_t* out = a.out + (uint64_t)poly * a.pitch_out;
#pragma unroll
  for (int u = 0; u < Sh::NSUB_C; ++u) {
    const int idx = t + NT * u;
    const int k1 = idx / W, w = idx % W;
    uint64_t base;
    int sh;
    if constexpr (!ROW) {
      const uint32_t cb = blk & ((1u << a.ncb_log) - 1), h = blk >> a.ncb_log;
      base = (uint64_t)cb * W + w + ((uint64_t)h << (a.lo + LOGR));
      sh = (int)a.lo;
    } else {
      base = (uint64_t)blk * W + w;
      sh = (int)a.out_log;
    }
#pragma unroll
    for (int k2 = 0; k2 < C; ++k2) out[base + ((uint64_t)(k1 + 64 * k2) << sh)] = x[u * C + bitrev_c(k2, LOGC)];
  }
}

// The addresses of this thread's 16 stores of `tile` (stage C's mapping), written with v.
template <int LOGR, int KIND, int TILE>
__device__ __forceinline__ void ip_prime_stores(const IpArgs& a, uint32_t tile, int t, const uint64_t* v) {
  using Sh = IpShape<LOGR, TILE>;
  constexpr int C = Sh::C, W = Sh::W, NT = Sh::NT;
  uint32_t poly, blk;
  ip_coords(a, tile, &poly, &blk);
  uint64_t* out = a.out + (uint64_t)poly * a.pitch_out;
#pragma unroll
  for (int u = 0; u < Sh::NSUB_C; ++u) {
    const int idx = t + NT * u;
    const int k1 = idx / W, w = idx % W;
    uint64_t base;
    int sh;
    if constexpr (KIND != 2) {
      const uint32_t cb = blk & ((1u << a.ncb_log) - 1), h = blk >> a.ncb_log;
      base = (uint64_t)cb * W + w + ((uint64_t)h << (a.lo + LOGR));
      sh = (int)a.lo;
    } else {
      base = (uint64_t)blk * W + w;
      sh = (int)a.out_log;
    }
#pragma unroll
    for (int k2 = 0; k2 < C; ++k2) out[base + ((uint64_t)(k1 + 64 * k2) << sh)] = v[u * C + k2];
  }
}

// KIND 0: first column pass (no twiddle); 1: column pass with twiddle; 2: row pass (last).
// waves per SIMD the register allocation must allow: 4 (4 workgroups of 4096-element tiles,
// or 2 of 8192, per CU); radix 2^6 needs 3 (it spills at 128 VGPRs)
#ifndef PBF_IP_WPE
#define PBF_IP_WPE 4
#endif
template <int LOGR, int E64, int KIND, int TILE, bool SPLIT>
__global__ void __launch_bounds__(TILE / 16) __attribute__((amdgpu_waves_per_eu(LOGR == 6 ? 3 : PBF_IP_WPE)))
ntt_ip_kernel(IpArgs a) {
  using Sh = IpShape<LOGR, TILE>;
  static_assert(Sh::DATA * 8 + Sh::TC * 8 <= (TILE > 4096 ? 80 : 40) * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint64_t lds[Sh::DATA];
  __shared__ uint64_t tcl[Sh::TC];
  uint32_t tile = blockIdx.x;
  if (tile >= a.tiles) return;
  for (int i = threadIdx.x; i < Sh::TC; i += Sh::NT) tcl[i] = a.tc[i];
  uint64_t v[16];
  ip_load<LOGR, TILE, KIND == 2>(a, tile, threadIdx.x, v);
  {
    // Make the loop entry look like the back edge to the compiler's wait-count analysis
    // (loads, then 16 stores per thread in flight): it merges the two paths conservatively
    // and would otherwise wait for vmcnt(0) -- this tile's stores -- before every tile.
    // The 16 stores go to this thread's own outputs of the first tile (positions no other
    // workgroup touches), after every thread of the workgroup has its input in registers;
    // the tile's real stores overwrite them later from the same thread, in program order.
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0); expcnt, lgkmcnt fields at their maximum (no wait)
    ip_bar();
    ip_prime_stores<LOGR, KIND, TILE>(a, tile, threadIdx.x, v);
  }
  for (;;) {
    // opaque copy of the thread index: the per-thread address arithmetic of the stages is
    // recomputed in every iteration (hoisted out of the loop, its live values spill)
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
    ip_tile<LOGR, E64, KIND, TILE, SPLIT>(a, lds, tcl, tile, t, v);
    const uint32_t next = tile + gridDim.x;
    if (next < a.tiles) ip_load<LOGR, TILE, KIND == 2>(a, next, t, v);  // in flight during B, C
    ip_tile_bc<LOGR, E64, KIND, TILE>(a, lds, tcl, tile, t);
    if (next >= a.tiles) break;
    tile = next;
    ip_bar();  // every wave has read Y before the next tile writes LDS
  }
}

}  // namespace pbf
