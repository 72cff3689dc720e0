// Two-pass 2^24-point Goldilocks NTT (gfx950): 4096 x 4096, one HBM round trip fewer than the
// three radix-2^8 passes ("Two-pass 2^24 plan"). The hot path of src/fft.rs
// CooleyTurkey (fft.rs:55-106) at the north-star size.
//
// n = 2^24, input index j + 4096 r (j, r < 4096), output index k1 + 4096 k2:
//   pass 1: for every column j, Y[j][k1] = w^(j k1) * DFT_4096 over r of x[j + 4096 r]
//           stored at y[j * 4096 + k1]                       (Stockham, Ns = 1)
//   pass 2: for every column k1, X[k1 + 4096 k2] = DFT_4096 over j of y[k1 + 4096 j]
//           stored at out[k1 + 4096 k2]                      (Stockham, Ns = 4096)
// Both passes run the same kernel: a tile is W = 8 columns (64-B runs) x all 4096 rows, i.e.
// 256 KiB, held in the registers of one 512-thread workgroup (64 elements per thread, 128
// VGPRs of data at two waves per SIMD). Each 4096-point column DFT is 64 x 64:
//   r = 64 a + b, k = c + 64 d
//   stage I   thread (b, w) holds x[64 a + b], a = 0..63: DFT-64 over a in registers (every
//             twiddle inside a 64-point DFT is a power of two: shift-reductions) -> c
//   twiddle   w_4096^(b c)                       (table, one general product per element)
//   exchange  (b, c) transposed through LDS in two rounds of 128 KiB (the tile is twice the
//             LDS): round h carries the pairs with bit 3 of b ^ bit 3 of c == h. Bit 3 of b
//             (writer) and bit 3 of c (reader) are the same thread bit (bit 6: the wave's
//             parity), so every write and read instruction is whole-wave and each thread
//             writes and reads exactly 32 values per round (peak 64 live values).
//   stage II  thread (c, w) holds the 64 b values: DFT-64 over b in registers -> d
//   pass 1 multiplies by the inter-pass twiddle w^(j k) (a 128 MiB [j][k] table, read once per
//   column block for the whole batch: XCD k-major tile order) before storing.
// General products per element over the whole transform: 3 (stage twiddles of both passes and
// the inter-pass twiddle), as in the regrouped three-pass plan, with one HBM pass fewer.
// LDS slot of (c, b, w) within a round: ((c * 32 + (b' ^ (c & 3))) * 8 + w), b' = b without
// bit 3 -- writers store 512-B contiguous runs, readers (8 c's per wave-instruction) hit every
// bank pair of each half-wave exactly once.
#pragma once
#include "ntt_kernels.hpp"

namespace pbf {

struct R4kArgs {
  const uint64_t* in;
  uint64_t* out;
  const uint64_t* tst;   // [b][c] = w_4096^(b c) (times n^-1 in an inverse's second pass)
  const uint64_t* post;  // pass 1: [j][k] = w^(j k), j, k < 4096
  uint32_t batch;
  uint32_t scaled;       // tst carries n^-1: multiply c = 0 too
  uint32_t kmajor;       // XCD k-major tile order (both polynomials of a column block on one XCD)
};

constexpr int R4K_NT = 512;
constexpr uint64_t R4K_N = 1ull << 24;

__device__ __forceinline__ int r4k_slot(int c, int b, int w) {
  const int bq = (b & 7) | ((b >> 4) << 3);
  return ((c * 32 + (bq ^ (c & 3))) << 3) + w;
}

// the (b, c) transpose through LDS: v (stage-I layout, thread (b, w), v[i] = value of c =
// bitrev6(i)) -> u (stage-II layout, thread (c, w), u[b]). v is dead afterwards.
__device__ __forceinline__ void r4k_exchange(uint64_t* lds, uint64_t* v, uint64_t* u, int t) {
  const int w = t & 7, bc = t >> 3;  // stage I: b = bc; stage II: c = bc
  // X = bit 3 of b (as a writer) = bit 3 of c (as a reader) = the wave's parity. Round h carries
  // the pairs with bit 3 of b ^ bit 3 of c == h. Registers i, i ^ 4 hold c, c ^ 8 (c = bitrev6(i));
  // a conditional swap (X, wave-uniform) puts the round-0 value of each pair in the register with
  // bit 2 clear, so the rounds write fixed registers and no branch splits the register liveness.
  const uint32_t X = __builtin_amdgcn_readfirstlane((t >> 6) & 1);
  if (X) {
#pragma unroll
    for (int i = 0; i < 64; ++i)
      if (!(i & 4)) { const uint64_t s = v[i]; v[i] = v[i | 4]; v[i | 4] = s; }
  }
  // slot(c | 8, b, w) = slot(c, b, w) + 2048
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h) __syncthreads();  // round-0 reads done before round-1 writes
    uint64_t* base = lds + ((X ^ h) ? 2048 : 0);
#pragma unroll
    for (int i = 0; i < 64; ++i)
      if (((i >> 2) & 1) == h) base[r4k_slot(bitrev_c(i & ~4, 6), bc, w)] = v[i];
    __syncthreads();
    // reader registers p, p | 8 (bit 3 of b): round h delivers b = p | 8 (X ^ h) into u[p | 8 h]
#pragma unroll
    for (int bb = 0; bb < 64; ++bb)
      if (((bb >> 3) & 1) == h) u[bb] = lds[r4k_slot(bc, bb & ~8, w)];
  }
  if (X) {
#pragma unroll
    for (int bb = 0; bb < 64; ++bb)
      if (!(bb & 8)) { const uint64_t s = u[bb]; u[bb] = u[bb | 8]; u[bb | 8] = s; }
  }
}

// stage I after the loads: DFT-64 over a, then w_4096^(b c) (c = 0 multiplies too: tst[b][0] is
// 1, or n^-1 in an inverse's second pass -- no branch)
template <int E64>
__device__ __forceinline__ void r4k_stage1(const R4kArgs& a, uint64_t* v, int b) {
  const FieldArgs f{};
  using G = Goldilocks;
  dft_reg<G, 6, E64>(v, nullptr, f);  // v[i] = Y[c = bitrev6(i)]
  const uint64_t* tb = a.tst + b * 64;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    uint64_t tw[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) tw[q] = tb[bitrev_c(8 * g + q, 6)];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[8 * g + q] = G::mul(v[8 * g + q], tw[q], f);
    __builtin_amdgcn_sched_barrier(0);  // keep the twiddle loads in groups of 8 (64 data values live)
  }
}

// DIT form of the DFT-64 over a (persistent kernel): e[i] = x[a = 2i], o[i] = x[a = 2i + 1]; two
// DFT-32 (the even half first, so it can run while the odd half is still loading) and the
// radix-2 combine X[c] = E[c] + w_64^c O[c], X[c + 32] = E[c] - w_64^c O[c]. Output v[i] =
// X[bitrev6(i)], as dft_reg's DFT-64 gives it (bitrev6(c) = 2 bitrev5(c) for c < 32, +1 for c + 32).
template <int E64, int I = 0>
__device__ __forceinline__ void r4k_combine(const uint64_t* e, const uint64_t* o, uint64_t* v) {
  if constexpr (I < 32) {
    const FieldArgs f{};
    using G = Goldilocks;
    constexpr int c = bitrev_c(I, 5);
    using T = ShiftKind<(E64 * c) % 192>;
    const uint64_t d = c == 0 ? o[I] : apply_shift<G, T>(o[I]);
    if constexpr (c != 0 && T::NEG) {
      v[2 * I] = G::sub(e[I], d, f);
      v[2 * I + 1] = G::add(e[I], d, f);
    } else {
      v[2 * I] = G::add(e[I], d, f);
      v[2 * I + 1] = G::sub(e[I], d, f);
    }
    r4k_combine<E64, I + 1>(e, o, v);
  }
}

template <int E64>
__device__ __forceinline__ void r4k_twiddle(const R4kArgs& a, uint64_t* v, int b) {
  const FieldArgs f{};
  using G = Goldilocks;
  const uint64_t* tb = a.tst + b * 64;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    uint64_t tw[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) tw[q] = tb[bitrev_c(8 * g + q, 6)];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[8 * g + q] = G::mul(v[8 * g + q], tw[q], f);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// stage II and the stores: DFT-64 over b; u[i] = Z[d = bitrev6(i)], k = c + 64 d
template <int E64, bool FIRST, bool DRAIN = false>
__device__ __forceinline__ void r4k_stage2(const R4kArgs& a, uint64_t* u, int t, uint32_t poly, uint64_t j0) {
  const FieldArgs f{};
  using G = Goldilocks;
  const int w = t & 7, c = t >> 3;
  dft_reg<G, 6, E64>(u, nullptr, f);
  // DRAIN (persistent kernel): the next tile's LDS-DMA, issued before this DFT, has landed
  // before the stores start (waiting after them would wait for the stores too)
  if constexpr (DRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (FIRST) {
    // y[j * 4096 + k] = w^(j k) Z[k], j = j0 + w
    const uint64_t j = j0 + w;
    uint64_t* o = a.out + (uint64_t)poly * R4K_N + (j << 12) + c;
    const uint64_t* pt = a.post + (j << 12) + c;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      uint64_t tw[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) tw[q] = pt[64 * bitrev_c(8 * g + q, 6)];
#pragma unroll
      for (int q = 0; q < 8; ++q) o[64 * bitrev_c(8 * g + q, 6)] = G::mul(u[8 * g + q], tw[q], f);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    // out[j + 4096 k], j = j0 + w
    uint64_t* o = a.out + (uint64_t)poly * R4K_N + j0 + w + ((uint64_t)c << 12);
#pragma unroll
    for (int i = 0; i < 64; ++i) o[(uint64_t)bitrev_c(i, 6) << 18] = u[i];
  }
}

__device__ __forceinline__ void r4k_coords(const R4kArgs& a, uint32_t tile, uint32_t* poly, uint32_t* kb) {
  const uint32_t tiles = 512u * a.batch;
  if (a.kmajor) {
    const uint32_t v = (tile & 7) * (tiles >> 3) + (tile >> 3);
    *kb = v / a.batch;
    *poly = v % a.batch;
  } else {
    *poly = tile >> 9;
    *kb = tile & 511;
  }
}

template <int E64, bool FIRST>
__global__ void __launch_bounds__(R4K_NT) __attribute__((amdgpu_waves_per_eu(2))) ntt_r4k_kernel(R4kArgs a) {
  __shared__ __attribute__((aligned(16))) uint64_t lds[16384];  // 128 KiB: half a tile
  const int t = threadIdx.x, w = t & 7, b = t >> 3;
  uint32_t poly, kb;
  r4k_coords(a, blockIdx.x, &poly, &kb);
  const uint64_t j0 = (uint64_t)kb * 8;
  // ---- x[j + 4096 (64 a + b)], a = 0..63 (a wave-instruction: 8 rows x 8 columns)
  const uint64_t* in = a.in + (uint64_t)poly * R4K_N + j0 + w + ((uint64_t)b << 12);
  uint64_t v[64], u[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) v[i] = in[(uint64_t)i << 18];
  r4k_stage1<E64>(a, v, b);
  r4k_exchange(lds, v, u, t);
  r4k_stage2<E64, FIRST>(a, u, t, poly, j0);
}

// Persistent, software-pipelined form (PBF_NTT_R4K=2): one workgroup per CU walks tiles
// blockIdx.x, + gridDim.x, ...; once a tile's exchange has left the LDS free, the next tile's
// even rows (a = 2i) are LDS-DMA'd into this wave's own 16 KiB image while stage II and the
// stores of the current tile run (each wave fetches exactly the rows its threads will read, so
// its own vmcnt orders them). A tile starts by issuing its odd rows' loads, then runs the even
// half's DFT-32 from the image while they arrive (stage I in DIT form, r4k_combine).
template <int E64, bool FIRST>
__global__ void __launch_bounds__(R4K_NT) __attribute__((amdgpu_waves_per_eu(2))) ntt_r4k_pkernel(R4kArgs a) {
  __shared__ __attribute__((aligned(16))) uint64_t lds[16384];
  const FieldArgs f{};
  using G = Goldilocks;
  const int t = threadIdx.x, w = t & 7, b = t >> 3, wave = t >> 6, lane = t & 63;
  const uint32_t tiles = 512u * a.batch;
  uint32_t tile = blockIdx.x;
  if (tile >= tiles) return;
  uint32_t poly, kb;
  r4k_coords(a, tile, &poly, &kb);
  uint64_t v[64], u[64], e[32], o[32];
  uint64_t* img = lds + wave * 2048;  // this wave's prefetch image [i < 32][b & 7][w], a = 2i
  bool first_tile = true;
  for (;;) {
    const uint64_t j0 = (uint64_t)kb * 8;
    const uint64_t* in = a.in + (uint64_t)poly * R4K_N + j0 + w + ((uint64_t)b << 12);
    if (first_tile) {
#pragma unroll
      for (int i = 0; i < 32; ++i) e[i] = in[(uint64_t)(2 * i) << 18];
    } else {
#pragma unroll
      for (int i = 0; i < 32; ++i) e[i] = img[i * 64 + (b & 7) * 8 + w];
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) o[i] = in[(uint64_t)(2 * i + 1) << 18];
    dft_reg<G, 5, sub_root_exp(E64, 5)>(e, nullptr, f);
    dft_reg<G, 5, sub_root_exp(E64, 5)>(o, nullptr, f);
    r4k_combine<E64>(e, o, v);
    r4k_twiddle<E64>(a, v, b);
    __syncthreads();  // every wave has read its prefetch image before the exchange writes
    r4k_exchange(lds, v, u, t);
    const uint32_t next = tile + gridDim.x;
    uint32_t npoly = 0, nkb = 0;
    if (next < tiles) {
      r4k_coords(a, next, &npoly, &nkb);
      __syncthreads();  // every exchange read is done: the LDS is free
      // even rows a = 2i: 16 LDS-DMA wave-instructions, each 2 i x this wave's 8 b x 64 B
      const uint64_t* nin = a.in + (uint64_t)npoly * R4K_N + nkb * 8;
      const int li = lane >> 5, lb = (lane >> 2) & 7, cp = (lane & 3) * 2;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint64_t row = (uint64_t)(64 * 2 * (2 * k + li) + 8 * wave + lb);
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(nin + cp + (row << 12)),
            (__attribute__((address_space(3))) void*)(img + 128 * k), 16, 0, 0);
      }
    }
    r4k_stage2<E64, FIRST, true>(a, u, t, poly, j0);
    if (next >= tiles) break;
    tile = next;
    poly = npoly;
    kb = nkb;
    first_tile = false;
  }
}

}  // namespace pbf
