// 29-bit-limb lazy arithmetic for the BN254-Fr NTT passes (gfx950; round 6).
//
// The Fr pass kernels (ntt256.hip) are VALU-bound on the Fr product: the 32-bit single-chain
// Montgomery product costs ~1.39x the 29-bit one of the MSM (msm_l29.hpp: nine 29-bit limbs,
// R' = 2^261, no carry folds; profiles/r04/fr_mul29.log), and a canonical 256-bit add or sub is
// a 24-instruction carry chain of 4-cycle operations. ntt256l_pass_kernel keeps its elements in
// nine 29-bit limbs between the load and the store of a pass: sums are nine plain 32-bit adds,
// differences add a multiple of r in redundant limbs first (no borrows), products take lazily
// reduced inputs, and one quotient-estimate reduction per element and radix-4 stage bounds
// everything again before the LDS exchange. Values enter canonical (< r) and leave canonical,
// so the pass's output is the same integer as the 32-bit kernel's.
//
// Twiddles are stored as w 2^261 mod r (canonical, normalised limbs): mul(x, w 2^261) = x w.
// Bounds (tests/test_fr29_bounds.py propagates them as intervals and checks every step): stage
// inputs are normalised and below 2r + 2^234; the radix-4 DIF's sums and differences stay below
// 13 r with every limb below 2^32; the product's 64-bit columns hold for the operands the stage
// gives it (normalised, or one redundant difference: limbs below 1.5 x 2^30), its output is
// normalised and below a b / 2^261 + r; reduce() brings a stage output back under the stage-input
// bound; canon() maps a normalised value below 3 r to [0, r).
#pragma once
#include <stdint.h>
#include "ec_bn254.hpp"  // fp256.hpp, and the types msm_l29.hpp uses
#include "msm_l29.hpp"

namespace pbf {
namespace fr29 {
using l29::L29;

// scripts/gen_l29_constants.py (fr section; tests/test_fr29_bounds.py checks this block)
constexpr uint32_t R29[9] = {0x10000001u, 0x1f0fac9fu, 0x0e5c2450u, 0x07d090f3u, 0x1585d283u, 0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
constexpr uint32_t NR29 = 0x0fffffffu;
constexpr uint32_t QC = 0x0000054au;  // floor(2^264 / r)
constexpr uint32_t B4R[9] = {0x20000004u, 0x3c3eb27du, 0x39709142u, 0x3f4243ccu, 0x36174a0bu, 0x2b6d0301u, 0x229b8503u, 0x397098cfu, 0x00c19138u};
constexpr uint32_t B8R[9] = {0x40000008u, 0x587d64fau, 0x52e12285u, 0x5e848799u, 0x4c2e9417u, 0x56da0603u, 0x45370a06u, 0x52e1319eu, 0x01832271u};
constexpr uint32_t B2R[9] = {0x20000002u, 0x3e1f593eu, 0x3cb848a0u, 0x2fa121e5u, 0x2b0ba505u, 0x25b68180u, 0x214dc281u, 0x3cb84c67u, 0x0060c89bu};
constexpr uint32_t MASK = l29::MASK;

// a b 2^-261 (mod r) by product scanning (l29::mul with r): normalised output below
// a b / 2^261 + r
__device__ __forceinline__ L29 mul(const L29& a, const L29& b) {
  uint32_t m[9];
  L29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    const int lo = k < 9 ? 0 : k - 8, hi = k < 9 ? k : 8;
#pragma unroll
    for (int i = lo; i <= hi; ++i) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = lo; i < (k < 9 ? k : 9); ++i) acc += (uint64_t)m[i] * R29[k - i];
    if (k < 9) {
      m[k] = ((uint32_t)acc * NR29) & MASK;
      acc += (uint64_t)m[k] * R29[0];
    } else {
      r.l[k - 9] = (uint32_t)acc & MASK;
    }
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}
__device__ __forceinline__ L29 add(const L29& a, const L29& b) {
  L29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = a.l[i] + b.l[i];
  return r;
}
// a + B - b for B a multiple of r in redundant limbs, each at least b's limb
__device__ __forceinline__ L29 sub(const L29& a, const L29& b, const uint32_t* B) {
  L29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = a.l[i] + (B[i] - b.l[i]);
  return r;
}
// a - q r with q = floor(t QC / 2^32), t = a's top limb plus the carry its neighbour holds (q
// never exceeds floor(a / r)); one signed carry pass leaves the limbs normalised
__device__ __forceinline__ L29 reduce(const L29& a) {
  const uint32_t t = a.l[8] + (a.l[7] >> 29);
  const uint32_t q = __umulhi(t, QC);
  L29 r;
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    acc += (int64_t)a.l[i] - (int64_t)((uint64_t)q * R29[i]);
    if (i < 8) {
      r.l[i] = (uint32_t)acc & MASK;
      acc >>= 29;
    }
  }
  r.l[8] = (uint32_t)acc;
  return r;
}
// a - r if a >= r (a normalised)
__device__ __forceinline__ L29 csub(const L29& a) {
  L29 d;
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int32_t x = (int32_t)a.l[i] - (int32_t)R29[i] - borrow;
    borrow = x < 0 ? 1 : 0;
    d.l[i] = i < 8 ? ((uint32_t)x & MASK) : (uint32_t)x;
  }
  L29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = borrow ? a.l[i] : d.l[i];
  return r;
}
// canonical 8 x 32-bit value of a normalised a below 3 r (two conditional subtractions)
__device__ __forceinline__ U256 canon(const L29& a) { return l29::to_u256(csub(csub(a))); }

}  // namespace fr29
}  // namespace pbf
