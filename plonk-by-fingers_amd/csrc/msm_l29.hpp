// 29-bit-limb Montgomery arithmetic for the MSM accumulation (BN254 Fq, gfx950; round 3).
//
// The 32-bit-limb product (fp256.hpp) folds the carry of every v_mad_u64_u32 into a third
// accumulator word: 128 of its 319 VALU are those folds. With nine 29-bit limbs a partial
// product is < 2^58, so a column of up to 18 of them plus the carry-in stays below 2^63 and
// NO carry is ever folded: 162 v_mad_u64_u32, 17 column shifts and the 9 Montgomery digits,
// ~205 VALU per product (R = 2^261).
//
// Domains: msm_chunk_acc_l29 keeps its XYZZ accumulator as X, Y = x 2^261 and ZZ, ZZZ = x 2^266
// (mod p) while the points arrive in the library's 32-bit Montgomery form (x 2^256): then
// every product of madd-2008-s lands in the domain its consumer expects (U2 = x ZZ 2^(256+266
// -261) = x ZZ 2^261, ZZ3 = ZZ PP 2^(266+261-261), ...), and only the first point of a run and
// the flushed bucket sums change domain (products by 2^266, 2^271, 2^256, 2^251 mod p).
// Values stay lazily reduced: products of normalised inputs below 17.3p are below 3.3p (R is
// 128x p), differences are taken as a + M - b with M = 8p or 16p in redundant limbs (every
// limb but the top >= 2^31 - 4: no borrows), and the accumulator is bounded by 11.3p (X; Y below
// 3.8p since round 6's mulsub), all
// derived in DESIGN.md §3.5. Results are exact group elements: bit-identical after the
// canonical conversion at the flush.
#pragma once
#include <stdint.h>

namespace pbf {
namespace l29 {

// scripts/gen_l29_constants.py (tests/test_l29_constants.py checks this block)
constexpr uint32_t P29[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u, 0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
constexpr uint32_t NP29 = 0x04866389u;
constexpr uint32_t M8P[9] = {0x83e7ea38u, 0x882305b2u, 0x83951a74u, 0x96a91683u, 0x8c2ecbbcu, 0x96da0601u, 0x85370a04u, 0x92e1319cu, 0x0183226fu};
constexpr uint32_t M16P[9] = {0x87cfd470u, 0x90460b68u, 0x872a34ecu, 0x8d522d0au, 0x985d977du, 0x8db40c06u, 0x8a6e140du, 0x85c2633cu, 0x030644e3u};
constexpr uint32_t C266[9] = {0x13349ca1u, 0x1a5d84a8u, 0x0a3e5cacu, 0x100249e0u, 0x12b951e8u, 0x0e92d304u, 0x14cb95b3u, 0x041b9d3du, 0x00058003u};
constexpr uint32_t C271[9] = {0x1d1c9c4bu, 0x08a372eeu, 0x1273abadu, 0x17c9d397u, 0x1698b0a7u, 0x09c89e50u, 0x177e12abu, 0x185f3518u, 0x001ed378u};
constexpr uint32_t C256[9] = {0x058f0d9du, 0x1aea1c6eu, 0x11c2cf74u, 0x11d651ebu, 0x1462c0a7u, 0x11b7bc3cu, 0x1cbd99bau, 0x183340fbu, 0x000e0a77u};
constexpr uint32_t C251[9] = {0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00080000u};
constexpr uint32_t P12[9] = {0x05dbdf54u, 0x0c348891u, 0x155fa7b4u, 0x01fda1cau, 0x024631a1u, 0x02470908u, 0x07d28f0du, 0x0c51ca70u, 0x0244b3adu};
constexpr uint32_t P4[9] = {0x01f3f51cu, 0x041182dbu, 0x11ca8d3cu, 0x0b548b43u, 0x161765e0u, 0x0b6d0302u, 0x029b8504u, 0x197098d0u, 0x00c19139u};

constexpr uint32_t MASK = (1u << 29) - 1;

struct L29 {
  uint32_t l[9];
};

__device__ __forceinline__ L29 from_u256(const U256& a) {  // re-limb a < 2^256
  L29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int b = 29 * i, w = b >> 5, s = b & 31;
    uint32_t v = a.w[w] >> s;
    if (s > 3 && w + 1 < 8) v |= a.w[w + 1] << (32 - s);
    r.l[i] = v & MASK;
  }
  return r;
}
__device__ __forceinline__ U256 to_u256(const L29& a) {  // a normalised and < 2^256
  U256 r;
#pragma unroll
  for (int w = 0; w < 8; ++w) {
    const int b = 32 * w, i = b / 29, s = b % 29;
    uint32_t v = a.l[i] >> s;
    if (i + 1 < 9) v |= a.l[i + 1] << (29 - s);
    if (s > 29 - 32 + 29 && i + 2 < 9) v |= a.l[i + 2] << (58 - s);
    r.w[w] = v;
  }
  return r;
}
// Montgomery product a b 2^-261 (mod p) by product scanning, one 64-bit accumulator and no
// carry folds; normalised output. Inputs: limbs < 2^29 (values < 2^261).
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
    for (int i = lo; i < (k < 9 ? k : 9); ++i) acc += (uint64_t)m[i] * P29[k - i];
    if (k < 9) {
      m[k] = ((uint32_t)acc * NP29) & MASK;
      acc += (uint64_t)m[k] * P29[0];  // the column's low 29 bits become 0
    } else {
      r.l[k - 9] = (uint32_t)acc & MASK;
    }
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}
// (a b - c d) 2^-261 + p (mod p) by ONE product scan (round 6): the c d terms enter the same
// columns through -c (v_mad_i64_i32), the accumulator is signed with arithmetic carries, and
// p 2^261 is added at columns 9..17 so that the total is positive; one Montgomery reduction
// instead of two products' and the lazy difference's (~150 fewer VALU per mixed addition).
// Column bound: the a b and m p terms are below 18 x 2^58, the c d terms above -9 x 2^58, so
// every column fits a signed 64-bit word. For madd-2008-s's Y3 (a b = R (Q - X3) below
// (17.3 p)^2, c d = Y PPP below 11.3 p x 3.3 p < p 2^261) the output is normalised and in
// (0.78 p, 3.8 p) (tests/test_l29_constants.py::test_mulsub_matches_montgomery restates it).
__device__ __forceinline__ L29 mulsub(const L29& a, const L29& b, const L29& c, const L29& d) {
  uint32_t m[9], nc[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) nc[i] = 0u - c.l[i];
  L29 r;
  uint64_t acc = 0;  // a signed value in two's complement
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    const int lo = k < 9 ? 0 : k - 8, hi = k < 9 ? k : 8;
#pragma unroll
    for (int i = lo; i <= hi; ++i) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = lo; i <= hi; ++i) acc += (uint64_t)((int64_t)(int32_t)nc[i] * (int64_t)d.l[k - i]);
#pragma unroll
    for (int i = lo; i < (k < 9 ? k : 9); ++i) acc += (uint64_t)m[i] * P29[k - i];
    if (k < 9) {
      m[k] = ((uint32_t)acc * NP29) & MASK;
      acc += (uint64_t)m[k] * P29[0];
    } else {
      acc += P29[k - 9];
      r.l[k - 9] = (uint32_t)acc & MASK;
    }
    acc = (uint64_t)((int64_t)acc >> 29);
  }
  r.l[8] = (uint32_t)acc + P29[8];
  return r;
}
// a b 2^-261 + E - f (mod p) by one product scan (round 6): E (a constant multiple of p) and f
// (a normalised value) enter at 2^261, i.e. their limbs at columns 9..17, into a signed
// accumulator; the difference madd-2008-s takes after its first two products (P = U2 - X,
// R = S2 - Y) then needs no separate a + M - b and carry normalisation. With E = 12p for
// f = X < 11.3p and E = 4p for f = Y < 3.8p the output is normalised and below 13.1p / 5.1p
// (tests/test_l29_constants.py::test_mul_shift_sub_matches_montgomery).
__device__ __forceinline__ L29 mul_shift_sub(const L29& a, const L29& b, const uint32_t* E, const L29& f) {
  uint32_t m[9];
  L29 r;
  uint64_t acc = 0;  // signed from column 9 on
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    const int lo = k < 9 ? 0 : k - 8, hi = k < 9 ? k : 8;
#pragma unroll
    for (int i = lo; i <= hi; ++i) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = lo; i < (k < 9 ? k : 9); ++i) acc += (uint64_t)m[i] * P29[k - i];
    if (k < 9) {
      m[k] = ((uint32_t)acc * NP29) & MASK;
      acc += (uint64_t)m[k] * P29[0];
      acc >>= 29;  // nonnegative so far
    } else {
      acc += (uint64_t)(int64_t)((int32_t)E[k - 9] - (int32_t)f.l[k - 9]);
      r.l[k - 9] = (uint32_t)acc & MASK;
      acc = (uint64_t)((int64_t)acc >> 29);
    }
  }
  r.l[8] = (uint32_t)acc + E[8] - f.l[8];
  return r;
}
// mul(a, a) with the square's symmetric column terms taken once, doubled (a_i (2 a_j), i < j:
// 45 instead of 81 products for a a; 2 a_j < 2^30, so a column of <= 4 doubled terms, a square,
// 9 m p terms and the carry stays below 18 x 2^58, the bound of mul's columns). The column sums
// are the same integers as mul's, so the Montgomery digits and the result are identical.
__device__ __forceinline__ L29 sqr(const L29& a) {
  uint32_t m[9], a2[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) a2[i] = a.l[i] << 1;
  L29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    const int lo = k < 9 ? 0 : k - 8;
#pragma unroll
    for (int i = lo; i < k - i; ++i) acc += (uint64_t)a.l[i] * a2[k - i];
    if ((k & 1) == 0) acc += (uint64_t)a.l[k / 2] * a.l[k / 2];
#pragma unroll
    for (int i = lo; i < (k < 9 ? k : 9); ++i) acc += (uint64_t)m[i] * P29[k - i];
    if (k < 9) {
      m[k] = ((uint32_t)acc * NP29) & MASK;
      acc += (uint64_t)m[k] * P29[0];
    } else {
      r.l[k - 9] = (uint32_t)acc & MASK;
    }
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}
// carry-normalise limbs < 2^32 (value < 2^261)
__device__ __forceinline__ L29 norm(L29 a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a.l[i + 1] += a.l[i] >> 29;
    a.l[i] &= MASK;
  }
  return a;
}
// a + M - b (limb-wise, no borrows: M's limbs exceed b's), normalised
__device__ __forceinline__ L29 sub(const L29& a, const L29& b, const uint32_t* M) {
  L29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = a.l[i] + M[i] - b.l[i];
  return norm(r);
}
// value == 0 or == p (a normalised, < 2p)
__device__ __forceinline__ bool zero_mod_p(const L29& a) {
  uint32_t z = 0, q = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    z |= a.l[i];
    q |= a.l[i] ^ P29[i];
  }
  return z == 0 || q == 0;
}
// canonical value of a normalised a < 2p
__device__ __forceinline__ L29 canon(const L29& a) {
  bool ge = true;  // a >= p, compared from the top limb
#pragma unroll
  for (int i = 8; i >= 0; --i) {
    if (a.l[i] != P29[i]) {
      ge = a.l[i] > P29[i];
      break;
    }
  }
  if (!ge) return a;
  L29 r;
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int32_t d = (int32_t)a.l[i] - (int32_t)P29[i] - borrow;
    borrow = d < 0 ? 1 : 0;
    r.l[i] = (uint32_t)(d + (borrow << 29));
  }
  return r;
}
__device__ __forceinline__ L29 konst(const uint32_t* c) {
  L29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = c[i];
  return r;
}

// XYZZ accumulator in the mixed domains above; `id` marks the identity
struct Acc {
  L29 X, Y, ZZ, ZZZ;
  bool id;
};

// Xyzz (32-bit Montgomery, canonical, not the identity) -> Acc
__device__ __forceinline__ Acc from_xyzz(const Xyzz& p) {
  Acc r;
  r.X = mul(from_u256(p.X), konst(C266));
  r.Y = mul(from_u256(p.Y), konst(C266));
  r.ZZ = mul(from_u256(p.ZZ), konst(C271));
  r.ZZZ = mul(from_u256(p.ZZZ), konst(C271));
  r.id = false;
  return r;
}
// Acc -> Xyzz (32-bit Montgomery, canonical)
__device__ __forceinline__ Xyzz to_xyzz(const Acc& a) {
  if (a.id) return G1::identity();
  Xyzz r;
  r.X = to_u256(canon(mul(a.X, konst(C256))));
  r.Y = to_u256(canon(mul(a.Y, konst(C256))));
  r.ZZ = to_u256(canon(mul(a.ZZ, konst(C251))));
  r.ZZZ = to_u256(canon(mul(a.ZZZ, konst(C251))));
  return r;
}

// x 2^5 (mod p) of a normalised x < p, below 1.0001 p: the shift, then q = floor(y_8 / (P29[8] + 1))
// (<= floor(32 x / p), so 32 x - q p >= 0, and 32 x - q p < (P29[8] + q + 1) 2^232) subtracted
// with signed carries. ~50 VALU instead of a product by 2^266 (the domain change of a run's
// first point: x 2^256 -> x 2^261).
__device__ __forceinline__ L29 times32(const L29& x) {
  uint32_t y[9];
  y[0] = (x.l[0] << 5) & MASK;
#pragma unroll
  for (int i = 1; i < 9; ++i) y[i] = ((x.l[i] << 5) | (x.l[i - 1] >> 24)) & MASK;
  const uint32_t q = y[8] / (P29[8] + 1);
  L29 r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int64_t v = (int64_t)y[i] - (int64_t)q * P29[i] + c;
    r.l[i] = (uint32_t)v & MASK;
    c = v >> 29;  // arithmetic: the borrow (0 after the top limb: the result is positive)
  }
  return r;
}

// a run's first point: X, Y = x 2^261, y 2^261 (the points' x 2^256 times 2^5, below 1.0001 p:
// within the bounds of a product's output), ZZ = ZZZ = 1 in the x 2^266 domain
__device__ __forceinline__ void start_run(Acc& a, const L29& x, const L29& y) {
  a.X = times32(x);
  a.Y = times32(y);
  a.ZZ = konst(C266);
  a.ZZZ = konst(C266);
  a.id = false;
}
// The raw accumulator (36 u32: X, Y, ZZ, ZZZ limbs; ZZ all zero for the identity), stored at a
// flush instead of the converted point: the conversion (4 products) then runs once per stored
// sum in a separate, divergence-free kernel (msm.hip msm_l29_finish) rather than inside the
// accumulation loop, where a wave pays it whenever any of its lanes flushes.
__device__ __forceinline__ void store_raw(const Acc& a, uint32_t* dst) {
  uint32_t w[36];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    w[i] = a.X.l[i];
    w[9 + i] = a.Y.l[i];
    w[18 + i] = a.id ? 0u : a.ZZ.l[i];
    w[27 + i] = a.ZZZ.l[i];
  }
  uint4* d = (uint4*)dst;
#pragma unroll
  for (int i = 0; i < 9; ++i) d[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}
__device__ __forceinline__ Xyzz raw_to_xyzz(const uint32_t* src) {
  const uint4* s4 = (const uint4*)src;
  uint32_t w[36];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint4 v = s4[i];
    w[4 * i] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
  Acc a;
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    a.X.l[i] = w[i];
    a.Y.l[i] = w[9 + i];
    a.ZZ.l[i] = w[18 + i];
    a.ZZZ.l[i] = w[27 + i];
    z |= w[18 + i];
  }
  a.id = z == 0;
  return to_xyzz(a);
}

// acc += (x, y) (affine point, 29-bit limbs of its 32-bit Montgomery coordinates):
// madd-2008-s. Returns true in the exceptional case P + P (the caller replaces acc by the
// doubled point): P == 0 is detected through ZZ3 = ZZ PP == 0 (PP == 0 iff P == 0, ZZ != 0),
// then R == 0 tells P + P from P + (-P) (the identity). Products are ordered so that every
// input dies as early as it can (the accumulation kernel is register-bound).
__device__ __forceinline__ bool madd(Acc& a, const L29& x, const L29& y) {
  if (a.id) {
    start_run(a, x, y);
    return false;
  }
  // P = U2 - X, R = S2 - Y with the differences inside the products' reductions (round 6)
  const L29 P = mul_shift_sub(x, a.ZZ, P12, a.X);
  const L29 R = mul_shift_sub(y, a.ZZZ, P4, a.Y);
  const L29 PP = sqr(P);
  const L29 ZZ3 = mul(a.ZZ, PP);
  if (zero_mod_p(ZZ3)) {  // P == 0: doubling (R == 0) or the identity
    L29 one{};
    one.l[0] = 1;
    if (zero_mod_p(mul(R, one))) return true;
    a.id = true;
    return false;
  }
  const L29 PPP = mul(P, PP);
  a.ZZZ = mul(a.ZZZ, PPP);
  const L29 Q = mul(a.X, PP);
  const L29 RR = sqr(R);
  L29 X3;
#pragma unroll
  for (int i = 0; i < 9; ++i) X3.l[i] = RR.l[i] + M8P[i] - PPP.l[i] - 2 * Q.l[i];
  X3 = norm(X3);
  // Y3 = R (Q - X3) - Y PPP under one reduction (round 6; round 5: two products and a + 8p - b)
  a.Y = mulsub(R, sub(Q, X3, M16P), a.Y, PPP);
  a.X = X3;
  a.ZZ = ZZ3;
  return false;
}

}  // namespace l29
}  // namespace pbf
