// Device field arithmetic for the u64 NTT path (gfx950).
//
// Two element types, both one uint64_t per element at rest in HBM (the layout of
// the reference's U64Field<M>, src/utils/u64field.rs:27-28), canonical in [0, M):
//   Goldilocks  p = 2^64 - 2^32 + 1   (BASELINE config 2 field)
//   Mod32       any odd M < 2^32      (the range where the reference's
//                                      `(a*b) % M` in u64 is exact, u64field.rs:177)
// Results are canonical after every op, so GPU outputs are bit-identical to the
// reference formulas (add u64field.rs:107-112, sub = add(neg) :147-165, mul :174-179).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbf {

struct FieldArgs {
  uint64_t m;   // modulus
  uint64_t mu;  // Mod32 only: floor(2^64 / m)
};

struct Goldilocks {
  static constexpr uint64_t P = 0xFFFFFFFF00000001ull;
  static constexpr uint64_t EPS = 0xFFFFFFFFull;  // 2^64 mod p = 2^32 - 1

  // The corrections below add or subtract a select of EPS (a 32-bit value) instead of
  // selecting between two 64-bit candidates: one v_cndmask instead of two per result.
  __host__ __device__ __forceinline__ static uint64_t add(uint64_t a, uint64_t b, const FieldArgs&) {
    uint64_t s;
    const bool wrap = __builtin_add_overflow(a, b, &s);
    // wrap: the true sum is s + 2^64 = s + EPS (mod p), and s + EPS cannot wrap again
    // (a + b - 2^64 < p - 2^32); s >= p: s - p = s + EPS (mod 2^64). Never both.
    return s + ((wrap || s >= P) ? EPS : 0);
  }
  __host__ __device__ __forceinline__ static uint64_t sub(uint64_t a, uint64_t b, const FieldArgs&) {
#ifdef __HIP_DEVICE_COMPILE__
    // 32-bit borrow chain: the borrow comes straight out of v_subb_co_u32 (the 64-bit
    // __builtin_sub_overflow form re-derived it with a v_cmp_gt_u64: one VALU more)
    unsigned c1, c2;
    const unsigned lo = __builtin_subc((unsigned)a, (unsigned)b, 0u, &c1);
    const unsigned hi = __builtin_subc((unsigned)(a >> 32), (unsigned)(b >> 32), c1, &c2);
    const uint64_t d = ((uint64_t)hi << 32) | lo;
    return d - (c2 ? EPS : 0);  // d + p (mod 2^64); d > EPS when borrowing
#else
    uint64_t d;
    const bool borrow = __builtin_sub_overflow(a, b, &d);
    return d - (borrow ? EPS : 0);
#endif
  }
  // 128-bit value lo + hi*2^64 reduced with 2^64 = 2^32 - 1 and 2^96 = -1 (mod p).
  __host__ __device__ __forceinline__ static uint64_t reduce128(uint64_t lo, uint64_t hi) {
    const uint64_t hh = hi >> 32, hl = (uint32_t)hi;
    uint64_t t0;
    const bool br = __builtin_sub_overflow(lo, hh, &t0);
    t0 -= br ? EPS : 0;                   // borrow: + p (cannot wrap: t0 >= 2^64 - 2^32 here)
    uint64_t r;
    const bool c = __builtin_add_overflow(t0, hl * EPS, &r);
    r += c ? EPS : 0;                     // wrap: + 2^64 = + EPS (cannot wrap again)
    return r >= P ? r - P : r;
  }
  // 64x64 -> 128 from four v_mad_u64_u32 (the carries ride in the 64-bit addends).
  __host__ __device__ __forceinline__ static uint64_t mul(uint64_t a, uint64_t b, const FieldArgs&) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p00 = (uint64_t)a0 * b0;
    const uint64_t t = (uint64_t)a0 * b1 + (p00 >> 32);
    const uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;
    const uint64_t v = (uint64_t)a1 * b1 + (t >> 32);
    return reduce128((u << 32) | (uint32_t)p00, v + (u >> 32));
  }
  // lo + t (mod p) for any lo < 2^64 and t <= (2^32-1)*EPS: one wrap/one
  // conditional subtraction suffice (see DESIGN.md "Goldilocks arithmetic").
  __host__ __device__ __forceinline__ static uint64_t add_small(uint64_t lo, uint64_t t) {
    uint64_t s;
    const bool wrap = __builtin_add_overflow(lo, t, &s);
    return s + ((wrap || s >= P) ? EPS : 0);
  }
  // x * 2^S (mod p) for a compile-time 0 <= S < 96, x canonical.
  template <int S>
  __host__ __device__ __forceinline__ static uint64_t mul_pow2(uint64_t x) {
    static_assert(S >= 0 && S < 96, "shift out of range");
    if constexpr (S == 0) {
      return x;
    } else if constexpr (S <= 32) {
      // x*2^S = lo + hi*2^64 with hi < 2^S <= 2^32, and hi*2^64 = hi*EPS (mod p)
      const uint64_t hi = x >> (64 - S);
      const uint64_t lo = x << S;
      return add_small(lo, (hi << 32) - hi);
    } else if constexpr (S < 64) {
      return reduce128(x << S, x >> (64 - S));
    } else {
      // 2^S = 2^(S-64) * 2^64 and 2^64 = 2^32 - 1 (mod p)
      const uint64_t y = mul_pow2<S - 64>(x);
      const uint64_t z = mul_pow2<32>(y);
      const uint64_t d = z - y;
      return (z < y) ? d - EPS : d;
    }
  }
};

// x * 2^-K (mod p) for a compile-time 1 <= K <= 32, x canonical: with m = -x mod 2^K,
// x + m*p is divisible by 2^K (p = 1 mod 2^32), and (x + m*p) / 2^K
//   = ((x + m) >> K) + (m << (32-K)) * (2^32 - 1)      (x + m < 2^64 for canonical x)
// -- two shifts, one v_mad_u64_u32 and one add_small, against ~25 instructions for the
// equivalent x * 2^(96-K) * (-1) through mul_pow2 (DESIGN.md "Goldilocks arithmetic").
template <int K>
__host__ __device__ __forceinline__ uint64_t gl_div_pow2(uint64_t x) {
  static_assert(K >= 1 && K <= 32, "division by 2^1 .. 2^32");
  const uint32_t mask = K == 32 ? 0xFFFFFFFFu : ((1u << (K & 31)) - 1u);
  const uint32_t m = (0u - (uint32_t)x) & mask;
  const uint64_t q = (x + m) >> K;
  const uint32_t mp = K == 32 ? m : (m << ((32 - K) & 31));
  return Goldilocks::add_small(q, (uint64_t)mp * Goldilocks::EPS);
}

struct Mod32 {
  __device__ __forceinline__ static uint64_t add(uint64_t a, uint64_t b, const FieldArgs& f) {
    uint64_t s = a + b;  // < 2^33
    return s >= f.m ? s - f.m : s;
  }
  __device__ __forceinline__ static uint64_t sub(uint64_t a, uint64_t b, const FieldArgs& f) {
    return a >= b ? a - b : a + f.m - b;
  }
  // Barrett: x < 2^64, q = floor(x * mu / 2^64) <= floor(x / m), remainder < 3m.
  __device__ __forceinline__ static uint64_t mul(uint64_t a, uint64_t b, const FieldArgs& f) {
    uint64_t x = a * b;
    uint64_t q = __umul64hi(x, f.mu);
    uint64_t r = x - q * f.m;
    if (r >= f.m) r -= f.m;
    if (r >= f.m) r -= f.m;
    return r;
  }
};

}  // namespace pbf
