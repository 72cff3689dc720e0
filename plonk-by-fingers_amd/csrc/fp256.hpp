// 256-bit prime fields for the BN254 path (BASELINE configs 3-5): Fr (the scalar field,
// NTT / polynomial multiply) and Fq (the base field of G1, MSM).
//
// At the ABI an element is 4 x uint64_t little-endian, canonical. Inside
// kernels elements are in Montgomery form (R = 2^256) as 8 x 32-bit limbs, so the
// 32x32+64 `v_mad_u64_u32` is the multiply-accumulate primitive of the CIOS product.
// Both moduli are < 2^254, so a CIOS result is < 2p and one conditional subtraction
// keeps every value canonical (bit-exact parity needs no lazy state).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "field.hpp"

namespace pbf {

struct U256 {
  uint32_t w[8];
};

struct Bn254FrParams {  // r = 0x30644e72...f0000001
  static constexpr uint32_t P[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t NP = 0xefffffffu;  // -p^-1 mod 2^32
  static constexpr uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                     0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
};

struct Bn254FqParams {  // q = 0x30644e72...d87cfd47
  static constexpr uint32_t P[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t NP = 0xe4866389u;
  static constexpr uint32_t R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                     0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
};

template <class Prm>
struct Fp256 {
  typedef U256 T;

  __host__ __device__ __forceinline__ static bool geq_p(const U256& a) {
#pragma unroll
    for (int i = 7; i >= 0; --i) {
      if (a.w[i] != Prm::P[i]) return a.w[i] > Prm::P[i];
    }
    return true;
  }
  // a - p (assumes a >= p)
  __host__ __device__ __forceinline__ static U256 sub_p(const U256& a) {
    U256 r;
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint64_t d = (uint64_t)a.w[i] - Prm::P[i] - borrow;
      r.w[i] = (uint32_t)d;
      borrow = (d >> 63) & 1;
    }
    return r;
  }
#if defined(__HIP_DEVICE_COMPILE__) && !defined(PBF_NO_ASM_ADD)
  // Device add / sub / reduce_once as explicit 32-bit carry chains: one chain carries through
  // an SGPR pair (VOP3), the other through VCC, p's limbs in VGPRs (an instruction with a
  // carry-in may read no other SGPR or literal on gfx950: one constant-bus read). Written in C++ the compiler rebuilds every limb's
  // carry from 64-bit adds and moves (~70 instructions, ~340 cycles for one add on a lone
  // wave); these are 24 VALU. A VALU carry write read by a VALU needs 2 wait states on gfx950:
  // the two chains are interleaved so each carry has one independent instruction and one
  // s_nop behind it (the compiler does not see inside the asm, so the pads are explicit).
  __device__ __forceinline__ static U256 add(const U256& a, const U256& b, const FieldArgs& = FieldArgs{}) {
    // s = a + b (< 2p < 2^256: no carry out), t = s - p; s where that borrowed (VCC), else t
    U256 s = a, t;
    uint64_t m;
    asm(
        "v_add_co_u32_e64 %0, %16, %0, %17\n\t"
        "s_nop 1\n\t"
        "v_addc_co_u32_e64 %1, %16, %1, %18, %16\n\t"
        "v_subrev_co_u32_e32 %8, vcc, %25, %0\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32_e64 %2, %16, %2, %19, %16\n\t"
        "v_subbrev_co_u32_e32 %9, vcc, %26, %1, vcc\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32_e64 %3, %16, %3, %20, %16\n\t"
        "v_subbrev_co_u32_e32 %10, vcc, %27, %2, vcc\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32_e64 %4, %16, %4, %21, %16\n\t"
        "v_subbrev_co_u32_e32 %11, vcc, %28, %3, vcc\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32_e64 %5, %16, %5, %22, %16\n\t"
        "v_subbrev_co_u32_e32 %12, vcc, %29, %4, vcc\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32_e64 %6, %16, %6, %23, %16\n\t"
        "v_subbrev_co_u32_e32 %13, vcc, %30, %5, vcc\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32_e64 %7, %16, %7, %24, %16\n\t"
        "v_subbrev_co_u32_e32 %14, vcc, %31, %6, vcc\n\t"
        "s_nop 1\n\t"
        "v_subbrev_co_u32_e32 %15, vcc, %32, %7, vcc\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e32 %0, %8, %0, vcc\n\t"
        "v_cndmask_b32_e32 %1, %9, %1, vcc\n\t"
        "v_cndmask_b32_e32 %2, %10, %2, vcc\n\t"
        "v_cndmask_b32_e32 %3, %11, %3, vcc\n\t"
        "v_cndmask_b32_e32 %4, %12, %4, vcc\n\t"
        "v_cndmask_b32_e32 %5, %13, %5, vcc\n\t"
        "v_cndmask_b32_e32 %6, %14, %6, vcc\n\t"
        "v_cndmask_b32_e32 %7, %15, %7, vcc"
        : "+v"(s.w[0]), "+v"(s.w[1]), "+v"(s.w[2]), "+v"(s.w[3]), "+v"(s.w[4]), "+v"(s.w[5]), "+v"(s.w[6]),
          "+v"(s.w[7]), "=&v"(t.w[0]), "=&v"(t.w[1]), "=&v"(t.w[2]), "=&v"(t.w[3]), "=&v"(t.w[4]),
          "=&v"(t.w[5]), "=&v"(t.w[6]), "=&v"(t.w[7]), "=&s"(m)
        : "v"(b.w[0]), "v"(b.w[1]), "v"(b.w[2]), "v"(b.w[3]), "v"(b.w[4]), "v"(b.w[5]), "v"(b.w[6]),
          "v"(b.w[7]), "v"(Prm::P[0]), "v"(Prm::P[1]), "v"(Prm::P[2]), "v"(Prm::P[3]), "v"(Prm::P[4]),
          "v"(Prm::P[5]), "v"(Prm::P[6]), "v"(Prm::P[7])
        : "vcc");
    return s;
  }
  __device__ __forceinline__ static U256 sub(const U256& a, const U256& b, const FieldArgs& = FieldArgs{}) {
    // s = a - b (mod 2^256), t = s + p; t where the subtraction borrowed (m), else s
    U256 s = a, t;
    uint64_t m;
    asm(
        "v_sub_co_u32_e64 %0, %16, %0, %17\n\t"
        "s_nop 1\n\t"
        "v_subb_co_u32_e64 %1, %16, %1, %18, %16\n\t"
        "v_add_co_u32_e32 %8, vcc, %25, %0\n\t"
        "s_nop 0\n\t"
        "v_subb_co_u32_e64 %2, %16, %2, %19, %16\n\t"
        "v_addc_co_u32_e32 %9, vcc, %26, %1, vcc\n\t"
        "s_nop 0\n\t"
        "v_subb_co_u32_e64 %3, %16, %3, %20, %16\n\t"
        "v_addc_co_u32_e32 %10, vcc, %27, %2, vcc\n\t"
        "s_nop 0\n\t"
        "v_subb_co_u32_e64 %4, %16, %4, %21, %16\n\t"
        "v_addc_co_u32_e32 %11, vcc, %28, %3, vcc\n\t"
        "s_nop 0\n\t"
        "v_subb_co_u32_e64 %5, %16, %5, %22, %16\n\t"
        "v_addc_co_u32_e32 %12, vcc, %29, %4, vcc\n\t"
        "s_nop 0\n\t"
        "v_subb_co_u32_e64 %6, %16, %6, %23, %16\n\t"
        "v_addc_co_u32_e32 %13, vcc, %30, %5, vcc\n\t"
        "s_nop 0\n\t"
        "v_subb_co_u32_e64 %7, %16, %7, %24, %16\n\t"
        "v_addc_co_u32_e32 %14, vcc, %31, %6, vcc\n\t"
        "s_nop 1\n\t"
        "v_addc_co_u32_e32 %15, vcc, %32, %7, vcc\n\t"
        "v_cndmask_b32_e64 %0, %0, %8, %16\n\t"
        "v_cndmask_b32_e64 %1, %1, %9, %16\n\t"
        "v_cndmask_b32_e64 %2, %2, %10, %16\n\t"
        "v_cndmask_b32_e64 %3, %3, %11, %16\n\t"
        "v_cndmask_b32_e64 %4, %4, %12, %16\n\t"
        "v_cndmask_b32_e64 %5, %5, %13, %16\n\t"
        "v_cndmask_b32_e64 %6, %6, %14, %16\n\t"
        "v_cndmask_b32_e64 %7, %7, %15, %16"
        : "+v"(s.w[0]), "+v"(s.w[1]), "+v"(s.w[2]), "+v"(s.w[3]), "+v"(s.w[4]), "+v"(s.w[5]), "+v"(s.w[6]),
          "+v"(s.w[7]), "=&v"(t.w[0]), "=&v"(t.w[1]), "=&v"(t.w[2]), "=&v"(t.w[3]), "=&v"(t.w[4]),
          "=&v"(t.w[5]), "=&v"(t.w[6]), "=&v"(t.w[7]), "=&s"(m)
        : "v"(b.w[0]), "v"(b.w[1]), "v"(b.w[2]), "v"(b.w[3]), "v"(b.w[4]), "v"(b.w[5]), "v"(b.w[6]),
          "v"(b.w[7]), "v"(Prm::P[0]), "v"(Prm::P[1]), "v"(Prm::P[2]), "v"(Prm::P[3]), "v"(Prm::P[4]),
          "v"(Prm::P[5]), "v"(Prm::P[6]), "v"(Prm::P[7])
        : "vcc");
    return s;
  }
  __device__ __forceinline__ static U256 reduce_once(const U256& a) {
    // a - p unless that borrows (a < 2p)
    U256 d;
    asm(
        "v_subrev_co_u32_e32 %0, vcc, %16, %8\n\t"
        "s_nop 1\n\t"
        "v_subbrev_co_u32_e32 %1, vcc, %17, %9, vcc\n\t"
        "s_nop 1\n\t"
        "v_subbrev_co_u32_e32 %2, vcc, %18, %10, vcc\n\t"
        "s_nop 1\n\t"
        "v_subbrev_co_u32_e32 %3, vcc, %19, %11, vcc\n\t"
        "s_nop 1\n\t"
        "v_subbrev_co_u32_e32 %4, vcc, %20, %12, vcc\n\t"
        "s_nop 1\n\t"
        "v_subbrev_co_u32_e32 %5, vcc, %21, %13, vcc\n\t"
        "s_nop 1\n\t"
        "v_subbrev_co_u32_e32 %6, vcc, %22, %14, vcc\n\t"
        "s_nop 1\n\t"
        "v_subbrev_co_u32_e32 %7, vcc, %23, %15, vcc\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e32 %0, %0, %8, vcc\n\t"
        "v_cndmask_b32_e32 %1, %1, %9, vcc\n\t"
        "v_cndmask_b32_e32 %2, %2, %10, vcc\n\t"
        "v_cndmask_b32_e32 %3, %3, %11, vcc\n\t"
        "v_cndmask_b32_e32 %4, %4, %12, vcc\n\t"
        "v_cndmask_b32_e32 %5, %5, %13, vcc\n\t"
        "v_cndmask_b32_e32 %6, %6, %14, vcc\n\t"
        "v_cndmask_b32_e32 %7, %7, %15, vcc"
        : "=&v"(d.w[0]), "=&v"(d.w[1]), "=&v"(d.w[2]), "=&v"(d.w[3]), "=&v"(d.w[4]), "=&v"(d.w[5]),
          "=&v"(d.w[6]), "=&v"(d.w[7])
        : "v"(a.w[0]), "v"(a.w[1]), "v"(a.w[2]), "v"(a.w[3]), "v"(a.w[4]), "v"(a.w[5]), "v"(a.w[6]),
          "v"(a.w[7]), "v"(Prm::P[0]), "v"(Prm::P[1]), "v"(Prm::P[2]), "v"(Prm::P[3]), "v"(Prm::P[4]),
          "v"(Prm::P[5]), "v"(Prm::P[6]), "v"(Prm::P[7])
        : "vcc");
    return d;
  }
#else
  __host__ __device__ __forceinline__ static U256 add(const U256& a, const U256& b, const FieldArgs& = FieldArgs{}) {
    U256 s;
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint64_t t = (uint64_t)a.w[i] + b.w[i] + c;
      s.w[i] = (uint32_t)t;
      c = t >> 32;
    }
    // a, b < p < 2^254: no carry out of 256 bits
    return reduce_once(s);
  }
  __host__ __device__ __forceinline__ static U256 sub(const U256& a, const U256& b, const FieldArgs& = FieldArgs{}) {
    U256 d;
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint64_t t = (uint64_t)a.w[i] - b.w[i] - borrow;
      d.w[i] = (uint32_t)t;
      borrow = (t >> 63) & 1;
    }
    if (borrow) {  // d + p
      uint64_t c = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint64_t t = (uint64_t)d.w[i] + Prm::P[i] + c;
        d.w[i] = (uint32_t)t;
        c = t >> 32;
      }
    }
    return d;
  }
  // a - p if a >= p, else a (a < 2p): one borrow chain and a select, no branches
  __host__ __device__ __forceinline__ static U256 reduce_once(const U256& a) {
    U256 d;
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t t = (uint64_t)a.w[i] - Prm::P[i] - borrow;
      d.w[i] = (uint32_t)t;
      borrow = (t >> 63) & 1;
    }
    U256 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = borrow ? a.w[i] : d.w[i];
    return r;
  }
#endif
#if defined(__HIP_DEVICE_COMPILE__)
  // Accumulators are 96-bit: c0 (64) + c1 (32) * 2^64. v_mad_u64_u32 returns the carry out
  // of its 64-bit sum in an SGPR pair, which a v_addc folds into c1. On gfx950 a VALU SGPR
  // write read as a carry by the next VALU needs 2 wait states: two independent chains
  // are interleaved so the pad is one s_nop 0 per two products.
  __device__ __forceinline__ static void mac2(uint64_t& a0, uint32_t& a1, uint32_t xa, uint32_t ya, uint64_t& b0,
                                              uint32_t& b1, uint32_t xb, uint32_t yb) {
    uint64_t ca, cb;
    asm("v_mad_u64_u32 %0, %2, %6, %7, %0\n\t"
        "v_mad_u64_u32 %1, %3, %8, %9, %1\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32_e64 %4, %2, %4, 0, %2\n\t"
        "v_addc_co_u32_e64 %5, %3, %5, 0, %3"
        : "+v"(a0), "+v"(b0), "=&s"(ca), "=&s"(cb), "+v"(a1), "+v"(b1)
        : "v"(xa), "v"(ya), "v"(xb), "v"(yb));
  }
  __device__ __forceinline__ static void mac1(uint64_t& a0, uint32_t& a1, uint32_t x, uint32_t y) {
    uint64_t c;
    asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
        "s_nop 1\n\t"
        "v_addc_co_u32_e64 %2, %1, %2, 0, %1"
        : "+v"(a0), "=&s"(c), "+v"(a1)
        : "v"(x), "v"(y));
  }
  // Montgomery product a*b*2^-256 mod p by finely integrated product scanning: column k
  // accumulates every a_i b_j and m_i p_j with i + j = k, one v_mad_u64_u32 plus one
  // carry add per product and no carry chains between limbs (the row-wise CIOS form
  // rebuilds a 64-bit addend around every product).
  __device__ __forceinline__ static U256 mul(const U256& a, const U256& b, const FieldArgs& = FieldArgs{}) {
    uint32_t m[8];
    U256 r;
    uint64_t c0 = 0;
    uint32_t c1 = 0;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
      // the column's products: a_i b_(k-i), then m_i p_(k-i) (i < k for k < 8)
      const int lo = k < 8 ? 0 : k - 7, hi = k < 8 ? k : 7;
      const int na = hi - lo + 1, nm = k < 8 ? k : 8 - lo;
      uint32_t xs[16], ys[16];
      int n = 0;
#pragma unroll
      for (int i = lo; i <= hi; ++i) { xs[n] = a.w[i]; ys[n] = b.w[k - i]; ++n; }
#pragma unroll
      for (int i = lo; i < lo + nm; ++i) { xs[n] = m[i]; ys[n] = Prm::P[k - i]; ++n; }
      (void)na;
      uint64_t d0 = 0;
      uint32_t d1 = 0;
#pragma unroll
      for (int t = 0; t + 1 < n; t += 2) mac2(c0, c1, xs[t], ys[t], d0, d1, xs[t + 1], ys[t + 1]);
      if (n & 1) mac1(c0, c1, xs[n - 1], ys[n - 1]);
      const uint64_t s0 = c0 + d0;
      c1 = c1 + d1 + (s0 < c0 ? 1u : 0u);
      c0 = s0;
      if (k < 8) {
        m[k] = (uint32_t)c0 * Prm::NP;
        mac1(c0, c1, m[k], Prm::P[0]);  // the column's low 32 bits become 0
      } else {
        r.w[k - 8] = (uint32_t)c0;
      }
      c0 = (c0 >> 32) | ((uint64_t)c1 << 32);
      c1 = 0;
    }
    r.w[7] = (uint32_t)c0;  // the result is < 2p < 2^256: nothing above
    return reduce_once(r);
  }
  // The same product with ONE accumulation chain per column, for throughput-bound kernels
  // (the MSM accumulation: four waves per SIMD fill each carry fold's wait states): no second
  // chain to merge and zero at every column, ~40 fewer VALU per product than mul.
  __device__ __forceinline__ static U256 mul_tp(const U256& a, const U256& b) {
    uint32_t m[8];
    U256 r;
    uint64_t c0 = 0;
    uint32_t c1 = 0;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
      const int lo = k < 8 ? 0 : k - 7, hi = k < 8 ? k : 7;
      const int nm = k < 8 ? k : 8 - lo;
#pragma unroll
      for (int i = lo; i <= hi; ++i) mac1(c0, c1, a.w[i], b.w[k - i]);
#pragma unroll
      for (int i = lo; i < lo + nm; ++i) mac1(c0, c1, m[i], Prm::P[k - i]);
      if (k < 8) {
        m[k] = (uint32_t)c0 * Prm::NP;
        mac1(c0, c1, m[k], Prm::P[0]);
      } else {
        r.w[k - 8] = (uint32_t)c0;
      }
      c0 = (c0 >> 32) | ((uint64_t)c1 << 32);
      c1 = 0;
    }
    r.w[7] = (uint32_t)c0;
    return reduce_once(r);
  }
  // Two chains of each of two products: four independent v_mad_u64_u32, then their four
  // carry folds -- each carry is read three instructions after its write, so no wait-state
  // pad (mac2 needs one s_nop per pair, mac1 two).
  __device__ __forceinline__ static void mac4(uint64_t& a0, uint32_t& a1, uint32_t xa, uint32_t ya, uint64_t& b0,
                                              uint32_t& b1, uint32_t xb, uint32_t yb, uint64_t& c0, uint32_t& c1,
                                              uint32_t xc, uint32_t yc, uint64_t& d0, uint32_t& d1, uint32_t xd,
                                              uint32_t yd) {
    uint64_t ca, cb, cc, cd;
    asm("v_mad_u64_u32 %0, %4, %12, %13, %0\n\t"
        "v_mad_u64_u32 %1, %5, %14, %15, %1\n\t"
        "v_mad_u64_u32 %2, %6, %16, %17, %2\n\t"
        "v_mad_u64_u32 %3, %7, %18, %19, %3\n\t"
        "v_addc_co_u32_e64 %8, %4, %8, 0, %4\n\t"
        "v_addc_co_u32_e64 %9, %5, %9, 0, %5\n\t"
        "v_addc_co_u32_e64 %10, %6, %10, 0, %6\n\t"
        "v_addc_co_u32_e64 %11, %7, %11, 0, %7"
        : "+v"(a0), "+v"(b0), "+v"(c0), "+v"(d0), "=&s"(ca), "=&s"(cb), "=&s"(cc), "=&s"(cd), "+v"(a1), "+v"(b1),
          "+v"(c1), "+v"(d1)
        : "v"(xa), "v"(ya), "v"(xb), "v"(yb), "v"(xc), "v"(yc), "v"(xd), "v"(yd));
  }
  // Two independent Montgomery products (*r = a b, *s = c d) by one interleaved column scan:
  // bit-identical to two mul() calls, for code whose time is one wave's instruction stream
  // (the MSM's reduction trees, single-lane point chains): the two products' chains fill each
  // other's carry wait states, so the stream carries no s_nop pads.
  __device__ __forceinline__ static void mul2(const U256& a, const U256& b, const U256& c, const U256& d, U256* r,
                                              U256* s) {
    uint32_t m[8], n[8];
    U256 ra, rb;
    uint64_t A0 = 0, B0 = 0;
    uint32_t A1 = 0, B1 = 0;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
      const int lo = k < 8 ? 0 : k - 7, hi = k < 8 ? k : 7;
      const int nm = k < 8 ? k : 8 - lo;
      uint32_t xa[16], ya[16], xb[16], yb[16];
      int cnt = 0;
#pragma unroll
      for (int i = lo; i <= hi; ++i) {
        xa[cnt] = a.w[i]; ya[cnt] = b.w[k - i];
        xb[cnt] = c.w[i]; yb[cnt] = d.w[k - i];
        ++cnt;
      }
#pragma unroll
      for (int i = lo; i < lo + nm; ++i) {
        xa[cnt] = m[i]; ya[cnt] = Prm::P[k - i];
        xb[cnt] = n[i]; yb[cnt] = Prm::P[k - i];
        ++cnt;
      }
      uint64_t A2 = 0, B2 = 0;
      uint32_t A3 = 0, B3 = 0;
#pragma unroll
      for (int t = 0; t + 1 < cnt; t += 2)
        mac4(A0, A1, xa[t], ya[t], B0, B1, xb[t], yb[t], A2, A3, xa[t + 1], ya[t + 1], B2, B3, xb[t + 1], yb[t + 1]);
      if (cnt & 1) mac2(A0, A1, xa[cnt - 1], ya[cnt - 1], B0, B1, xb[cnt - 1], yb[cnt - 1]);
      const uint64_t sa = A0 + A2, sb = B0 + B2;
      A1 = A1 + A3 + (sa < A0 ? 1u : 0u);
      B1 = B1 + B3 + (sb < B0 ? 1u : 0u);
      A0 = sa;
      B0 = sb;
      if (k < 8) {
        m[k] = (uint32_t)A0 * Prm::NP;
        n[k] = (uint32_t)B0 * Prm::NP;
        mac2(A0, A1, m[k], Prm::P[0], B0, B1, n[k], Prm::P[0]);
      } else {
        ra.w[k - 8] = (uint32_t)A0;
        rb.w[k - 8] = (uint32_t)B0;
      }
      A0 = (A0 >> 32) | ((uint64_t)A1 << 32);
      B0 = (B0 >> 32) | ((uint64_t)B1 << 32);
      A1 = 0;
      B1 = 0;
    }
    ra.w[7] = (uint32_t)A0;
    rb.w[7] = (uint32_t)B0;
    *r = reduce_once(ra);
    *s = reduce_once(rb);
  }
  // Three independent chains: three v_mad_u64_u32, then their carry folds -- each carry is
  // read two instructions after its write (the two wait states it needs, no pad).
  __device__ __forceinline__ static void mac3(uint64_t& a0, uint32_t& a1, uint32_t xa, uint32_t ya, uint64_t& b0,
                                              uint32_t& b1, uint32_t xb, uint32_t yb, uint64_t& c0, uint32_t& c1,
                                              uint32_t xc, uint32_t yc) {
    uint64_t ca, cb, cc;
    asm("v_mad_u64_u32 %0, %3, %9, %10, %0\n\t"
        "v_mad_u64_u32 %1, %4, %11, %12, %1\n\t"
        "v_mad_u64_u32 %2, %5, %13, %14, %2\n\t"
        "v_addc_co_u32_e64 %6, %3, %6, 0, %3\n\t"
        "v_addc_co_u32_e64 %7, %4, %7, 0, %4\n\t"
        "v_addc_co_u32_e64 %8, %5, %8, 0, %5"
        : "+v"(a0), "+v"(b0), "+v"(c0), "=&s"(ca), "=&s"(cb), "=&s"(cc), "+v"(a1), "+v"(b1), "+v"(c1)
        : "v"(xa), "v"(ya), "v"(xb), "v"(yb), "v"(xc), "v"(yc));
  }
  // N = 3 or 4 independent Montgomery products out[j] = x[j] y[j] by one interleaved column
  // scan, one accumulator per chain (mac3 / mac4: no wait-state pads): bit-identical to N
  // mul() calls. Point additions on single-lane latency chains group their independent
  // products into these (ec_bn254.hpp add2 / dbl2): 4 dependent steps per addition instead of 7.
  template <int N>
  __device__ __forceinline__ static void mulN(const U256* const* x, const U256* const* y, U256* const* out) {
    static_assert(N == 3 || N == 4, "mulN: 3 or 4 chains");
    uint32_t m[N][8];
    U256 res[N];
    uint64_t c0[N];
    uint32_t c1[N];
#pragma unroll
    for (int j = 0; j < N; ++j) { c0[j] = 0; c1[j] = 0; }
#pragma unroll
    for (int k = 0; k < 15; ++k) {
      const int lo = k < 8 ? 0 : k - 7, hi = k < 8 ? k : 7;
      const int nm = k < 8 ? k : 8 - lo;
#pragma unroll
      for (int i = lo; i <= hi; ++i) {
        if constexpr (N == 4)
          mac4(c0[0], c1[0], x[0]->w[i], y[0]->w[k - i], c0[1], c1[1], x[1]->w[i], y[1]->w[k - i], c0[2], c1[2],
               x[2]->w[i], y[2]->w[k - i], c0[3], c1[3], x[3]->w[i], y[3]->w[k - i]);
        else
          mac3(c0[0], c1[0], x[0]->w[i], y[0]->w[k - i], c0[1], c1[1], x[1]->w[i], y[1]->w[k - i], c0[2], c1[2],
               x[2]->w[i], y[2]->w[k - i]);
      }
#pragma unroll
      for (int i = lo; i < lo + nm; ++i) {
        if constexpr (N == 4)
          mac4(c0[0], c1[0], m[0][i], Prm::P[k - i], c0[1], c1[1], m[1][i], Prm::P[k - i], c0[2], c1[2], m[2][i],
               Prm::P[k - i], c0[3], c1[3], m[3][i], Prm::P[k - i]);
        else
          mac3(c0[0], c1[0], m[0][i], Prm::P[k - i], c0[1], c1[1], m[1][i], Prm::P[k - i], c0[2], c1[2], m[2][i],
               Prm::P[k - i]);
      }
      if (k < 8) {
#pragma unroll
        for (int j = 0; j < N; ++j) m[j][k] = (uint32_t)c0[j] * Prm::NP;
        if constexpr (N == 4)
          mac4(c0[0], c1[0], m[0][k], Prm::P[0], c0[1], c1[1], m[1][k], Prm::P[0], c0[2], c1[2], m[2][k], Prm::P[0],
               c0[3], c1[3], m[3][k], Prm::P[0]);
        else
          mac3(c0[0], c1[0], m[0][k], Prm::P[0], c0[1], c1[1], m[1][k], Prm::P[0], c0[2], c1[2], m[2][k], Prm::P[0]);
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) res[j].w[k - 8] = (uint32_t)c0[j];
      }
#pragma unroll
      for (int j = 0; j < N; ++j) {
        c0[j] = (c0[j] >> 32) | ((uint64_t)c1[j] << 32);
        c1[j] = 0;
      }
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
      res[j].w[7] = (uint32_t)c0[j];
      *out[j] = reduce_once(res[j]);
    }
  }
#else
  // -p^-1 mod 2^64 from the 32-bit constant's modulus by Newton's iteration (x <- x(2 - p x)
  // doubles the correct low bits; p is odd so x = p is right mod 2^3)
  static constexpr uint64_t np64() {
    const uint64_t p0 = (uint64_t)Prm::P[0] | ((uint64_t)Prm::P[1] << 32);
    uint64_t x = p0;
    for (int i = 0; i < 6; ++i) x *= 2 - p0 * x;
    return 0 - x;
  }
  // host pass of device code that names the single-chain product: the same product
  static U256 mul_tp(const U256& a, const U256& b) { return mul(a, b); }
  // CIOS Montgomery product a*b*2^-256 mod p (host) over 4 x 64-bit limbs with 128-bit
  // products: the MSM's host Horner over the window sums (~2600 products per MSM) runs
  // ~2.3x faster than over 8 x 32-bit limbs (mul_cios32, kept as the cross-check;
  // tests/native/fp256_host_check.hip).
  static U256 mul(const U256& a, const U256& b, const FieldArgs& = FieldArgs{}) {
    typedef unsigned __int128 u128;
    constexpr uint64_t NP = np64();
    uint64_t x[4], y[4], p[4], t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
      x[i] = (uint64_t)a.w[2 * i] | ((uint64_t)a.w[2 * i + 1] << 32);
      y[i] = (uint64_t)b.w[2 * i] | ((uint64_t)b.w[2 * i + 1] << 32);
      p[i] = (uint64_t)Prm::P[2 * i] | ((uint64_t)Prm::P[2 * i + 1] << 32);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      u128 s;
      uint64_t C = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s = (u128)x[j] * y[i] + t[j] + C;
        t[j] = (uint64_t)s;
        C = (uint64_t)(s >> 64);
      }
      s = (u128)t[4] + C;
      t[4] = (uint64_t)s;
      t[5] = (uint64_t)(s >> 64);
      const uint64_t m = t[0] * NP;
      s = (u128)m * p[0] + t[0];
      C = (uint64_t)(s >> 64);
#pragma unroll
      for (int j = 1; j < 4; ++j) {
        s = (u128)m * p[j] + t[j] + C;
        t[j - 1] = (uint64_t)s;
        C = (uint64_t)(s >> 64);
      }
      s = (u128)t[4] + C;
      t[3] = (uint64_t)s;
      t[4] = t[5] + (uint64_t)(s >> 64);
    }
    // t < 2p: subtract p once unless that borrows (branch-free select)
    uint64_t d[4], br = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u128 v = (u128)t[i] - p[i] - br;
      d[i] = (uint64_t)v;
      br = (uint64_t)(v >> 64) & 1;
    }
    U256 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t o = br ? t[i] : d[i];
      r.w[2 * i] = (uint32_t)o;
      r.w[2 * i + 1] = (uint32_t)(o >> 32);
    }
    return r;
  }
  static void mul2(const U256& a, const U256& b, const U256& c, const U256& d, U256* r, U256* s) {
    *r = mul(a, b);
    *s = mul(c, d);
  }
  template <int N>
  static void mulN(const U256* const* x, const U256* const* y, U256* const* out) {
    U256 t[N];
    for (int j = 0; j < N; ++j) t[j] = mul(*x[j], *y[j]);  // inputs may alias outputs
    for (int j = 0; j < N; ++j) *out[j] = t[j];
  }
  // CIOS Montgomery product over 8 x 32-bit limbs (host cross-check of mul)
  static U256 mul_cios32(const U256& a, const U256& b) {
    uint32_t t[10];
    for (int i = 0; i < 10; ++i) t[i] = 0;
    for (int i = 0; i < 8; ++i) {
      uint64_t C = 0;
      for (int j = 0; j < 8; ++j) {
        uint64_t s = (uint64_t)a.w[j] * b.w[i] + t[j] + C;
        t[j] = (uint32_t)s;
        C = s >> 32;
      }
      uint64_t s = (uint64_t)t[8] + C;
      t[8] = (uint32_t)s;
      t[9] = (uint32_t)(s >> 32);
      const uint32_t m = t[0] * Prm::NP;
      s = (uint64_t)m * Prm::P[0] + t[0];
      C = s >> 32;
      for (int j = 1; j < 8; ++j) {
        s = (uint64_t)m * Prm::P[j] + t[j] + C;
        t[j - 1] = (uint32_t)s;
        C = s >> 32;
      }
      s = (uint64_t)t[8] + C;
      t[7] = (uint32_t)s;
      t[8] = t[9] + (uint32_t)(s >> 32);
    }
    U256 r;
    for (int i = 0; i < 8; ++i) r.w[i] = t[i];
    return geq_p(r) ? sub_p(r) : r;
  }
#endif
  __host__ __device__ __forceinline__ static U256 r2() {
    U256 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v.w[i] = Prm::R2[i];
    return v;
  }
  __host__ __device__ __forceinline__ static U256 one_plain() {
    U256 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v.w[i] = i == 0 ? 1u : 0u;
    return v;
  }
  // canonical <-> Montgomery (the ABI never sees Montgomery form)
  __host__ __device__ __forceinline__ static U256 to_mont(const U256& a) { return mul(a, r2()); }
  __host__ __device__ __forceinline__ static U256 from_mont(const U256& a) { return mul(a, one_plain()); }
  __host__ __device__ __forceinline__ static bool is_zero(const U256& a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= a.w[i];
    return o == 0;
  }
  __host__ __device__ __forceinline__ static bool eq(const U256& a, const U256& b) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= a.w[i] ^ b.w[i];
    return o == 0;
  }
};

// 4 x uint64_t little-endian (the ABI layout) <-> 8 x uint32_t limbs
__host__ __device__ inline U256 u256_from_u64(const uint64_t* l) {
  U256 r;
  for (int i = 0; i < 4; ++i) {
    r.w[2 * i] = (uint32_t)l[i];
    r.w[2 * i + 1] = (uint32_t)(l[i] >> 32);
  }
  return r;
}
__host__ __device__ inline void u256_to_u64(const U256& a, uint64_t* l) {
  for (int i = 0; i < 4; ++i) l[i] = (uint64_t)a.w[2 * i] | ((uint64_t)a.w[2 * i + 1] << 32);
}

typedef Fp256<Bn254FrParams> Fr;
typedef Fp256<Bn254FqParams> Fq;

}  // namespace pbf
