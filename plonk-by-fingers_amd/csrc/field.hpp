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

#ifdef __HIP_DEVICE_COMPILE__
// ---- carry-exact device primitives for Goldilocks reductions (gfx950) -------------------
// One instruction per asm statement, register operands only: the compiler allocates, and
// its hazard recognizer sees the SGPR lane-mask def/use of each statement (it inserts the
// wait states a VALU-written carry needs before a VALU reads it). What the compiler cannot
// express by itself is the carry-out of v_mad_u64_u32, so a reduction that would otherwise
// recompute carries with 64-bit compares uses it directly.
struct GlMadC {
  uint64_t v;  // low 64 bits of a*b + c
  uint64_t c;  // lane mask: a*b + c >= 2^64
};
__device__ __forceinline__ GlMadC gl_mad_c(uint32_t a, uint32_t b, uint64_t c) {
  GlMadC r;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r.v), "=s"(r.c) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t gl_sub_co(uint32_t a, uint32_t b, uint64_t* borrow) {
  uint32_t r;
  asm("v_sub_co_u32_e64 %0, %1, %2, %3" : "=v"(r), "=s"(*borrow) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t gl_subb0(uint32_t a, uint64_t bin, uint64_t* borrow) {
  uint32_t r;
  asm("v_subbrev_co_u32_e64 %0, %1, 0, %2, %3" : "=v"(r), "=s"(*borrow) : "v"(a), "s"(bin));
  return r;
}
__device__ __forceinline__ uint64_t gl_ge_p(uint64_t r) {  // lane mask: r >= p
  uint64_t m;
  asm("v_cmp_lt_u64_e64 %0, %1, %2" : "=s"(m) : "s"(0xFFFFFFFF00000000ull), "v"(r));
  return m;
}
template <uint32_t K>
__device__ __forceinline__ uint32_t gl_selk(uint32_t a, uint64_t m) {  // m ? K : a
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %3, %2" : "=v"(r) : "v"(a), "s"(m), "i"(K));
  return r;
}
// a - b (mod p), canonical, for canonical a, b: 4 VALU. d = a - b over a 32-bit borrow chain;
// a borrow means d + p = d - EPS = d - 2^32 + 1 (d > EPS then), applied as lo + 1 (carry c)
// and hi - (borrow & !c): the correction's carries ride in SGPR masks (one SALU andn2)
// instead of a selected 64-bit addend (two v_cndmask + a 64-bit add).
__device__ __forceinline__ uint64_t gl_sub_chain(uint64_t a, uint64_t b) {
  uint64_t bo, c;
  uint32_t lo, hi, lo2, hi2;
  asm("v_sub_co_u32_e64 %0, %1, %2, %3" : "=v"(lo), "=s"(bo) : "v"((uint32_t)a), "v"((uint32_t)b));
  asm("v_subb_co_u32_e64 %0, %1, %2, %3, %4"
      : "=v"(hi), "=s"(bo)
      : "v"((uint32_t)(a >> 32)), "v"((uint32_t)(b >> 32)), "s"(bo));
  asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(lo2), "=s"(c) : "v"(lo), "s"(bo));
  const uint64_t m = bo & ~c;
  asm("v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(hi2), "=s"(c) : "v"(hi), "s"(m));
  return ((uint64_t)hi2 << 32) | lo2;
}
// lo + h*(2^32-1) (mod p), canonical; lo < 2^64, h < 2^32. With the carry c of the 64-bit
// sum r, the value is r + c*EPS: c = 1 leaves r < 2^64 - 2^33, so r + EPS is canonical;
// c = 0 and r >= p gives r - p = r + EPS (mod 2^64). 6 VALU.
__device__ __forceinline__ uint64_t gl_addmul_eps(uint64_t lo, uint32_t h) {
  const GlMadC m = gl_mad_c(h, 0xFFFFFFFFu, lo);
  const uint32_t a0 = gl_selk<0xFFFFFFFFu>(0u, m.c | gl_ge_p(m.v));
  return m.v + a0;
}
// lo + h0*2^64 + h1*2^96 = lo + h0*EPS - h1 (mod p), canonical; lo < 2^64, h0, h1 < 2^32.
// r = lo + h0*EPS with carry c1 (+EPS), then r -= h1 with borrow c2 (-EPS). c1 without c2
// leaves r < 2^64 - 2^33 (r + EPS canonical); c2 without c1 leaves r >= 2^64 - 2^32 (r - EPS
// canonical); both or neither: r, minus p when r >= p. One 64-bit addend per case:
// +EPS = {2^32-1, 0}, -EPS = {1, 2^32-1} (mod 2^64). 9 VALU against 15-17 for the compiler's
// compare-derived carries.
__device__ __forceinline__ uint64_t gl_red96(uint64_t lo, uint32_t h0, uint32_t h1) {
  const GlMadC m = gl_mad_c(h0, 0xFFFFFFFFu, lo);
  uint64_t c2;
  const uint32_t r0 = gl_sub_co((uint32_t)m.v, h1, &c2);
  const uint32_t r1 = gl_subb0((uint32_t)(m.v >> 32), c2, &c2);
  const uint64_t r = ((uint64_t)r1 << 32) | r0;
  const uint64_t plus = (m.c & ~c2) | (gl_ge_p(r) & ~(m.c ^ c2));
  const uint64_t minus = c2 & ~m.c;
  // +EPS = lo - 1, hi + 1 - borrow; -EPS = lo + 1, hi - 1 + carry (plus, minus exclusive):
  // four carry-chain VALU, the lane masks combined on the SALU (a selected 64-bit addend
  // took three v_cndmask, a v_mov and two 64-bit adds as compiled)
  uint64_t c3, c4, c5;
  uint32_t l1, l2, u1, u2;
  asm("v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(l1), "=s"(c3) : "v"(r0), "s"(plus));
  asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(l2), "=s"(c4) : "v"(l1), "s"(minus));
  const uint64_t up = plus & ~c3, dn = minus & ~c4;
  asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(u1), "=s"(c5) : "v"(r1), "s"(up));
  asm("v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(u2), "=s"(c5) : "v"(u1), "s"(dn));
  return ((uint64_t)u2 << 32) | l2;
}
#endif

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
    return gl_sub_chain(a, b);
#else
    uint64_t d;
    const bool borrow = __builtin_sub_overflow(a, b, &d);
    return d - (borrow ? EPS : 0);
#endif
  }
  // 128-bit value lo + hi*2^64 reduced with 2^64 = 2^32 - 1 and 2^96 = -1 (mod p).
  __host__ __device__ __forceinline__ static uint64_t reduce128(uint64_t lo, uint64_t hi) {
#ifdef __HIP_DEVICE_COMPILE__
    return gl_red96(lo, (uint32_t)hi, (uint32_t)(hi >> 32));
#else
    const uint64_t hh = hi >> 32, hl = (uint32_t)hi;
    uint64_t t0;
    const bool br = __builtin_sub_overflow(lo, hh, &t0);
    t0 -= br ? EPS : 0;                   // borrow: + p (cannot wrap: t0 >= 2^64 - 2^32 here)
    uint64_t r;
    const bool c = __builtin_add_overflow(t0, hl * EPS, &r);
    r += c ? EPS : 0;                     // wrap: + 2^64 = + EPS (cannot wrap again)
    return r >= P ? r - P : r;
#endif
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
  // lo + h*EPS (mod p), canonical, for any lo < 2^64 and h < 2^32.
  __host__ __device__ __forceinline__ static uint64_t add_mul_eps(uint64_t lo, uint32_t h) {
#ifdef __HIP_DEVICE_COMPILE__
    return gl_addmul_eps(lo, h);
#else
    return add_small(lo, (uint64_t)h * EPS);
#endif
  }
  // x * 2^S (mod p) for a compile-time 0 <= S < 96, x canonical.
  template <int S>
  __host__ __device__ __forceinline__ static uint64_t mul_pow2(uint64_t x) {
    static_assert(S >= 0 && S < 96, "shift out of range");
    if constexpr (S == 0) {
      return x;
    } else if constexpr (S <= 32) {
      // x*2^S = lo + hi*2^64 with hi < 2^S <= 2^32, and hi*2^64 = hi*EPS (mod p)
      return add_mul_eps(x << S, (uint32_t)(x >> (64 - S)));
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
  return Goldilocks::add_mul_eps(q, mp);
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
