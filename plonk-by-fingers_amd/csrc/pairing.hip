// BN254 optimal-ate pairing on gfx950 (BASELINE config 4 "pairing check"; the BN254
// instance of the reference's Pairing::pairing, src/ec.rs:87-93 / src/pbh/pairing.rs:12-47,
// which Plonk::verify calls twice, src/plonk.rs:646-647).
//
//   e(P, Q) = ( f_{6u+2,Q}(P) * l_{T,pi(Q)}(P) * l_{T',-pi^2(Q)}(P) )^((q^12-1)/r)
//
// Tower: Fq2 = Fq[u]/(u^2+1), xi = 9+u, Fq12 = Fq2[w]/(w^6 - xi) (= Fq6[w]/(w^2-v) with
// v = w^2, Fq6 = Fq2[v]/(v^3-xi)); G2 on the D-type twist y^2 = x^3 + 3/xi.
//
// One wave (one 64-thread workgroup) per pairing, Fq12 values in LDS in the flat w-basis
// g[k] = coefficient of w^k. A product of two Fq12 is 36 Fq2 products, one per lane,
// and 6 lanes summing them (x xi for the wrapped terms): the latency of one Fq2 product
// instead of 54 dependent Fq products on one thread. T runs in homogeneous projective
// coordinates (no inversions in the Miller loop); its formulas are split into stages of
// independent Fq2 products, one per lane. Lines are scaled by Fq2 factors
// (doubling: 2 Y Z^2, addition: xQ Z - X), which the final exponentiation removes
// ((q^12-1)/r is a multiple of q^2-1), so every pairing value is the reduced pairing
// itself, bit-identical to oracle/bn254_pairing.py.
//
// Final exponentiation: easy part f^(q^6-1) (conjugate times inverse; one Fq inversion
// by binary extended Euclid), f^(q^2+1) (Frobenius); hard part EXACTLY
// (q^4-q^2+1)/r = l0 + l1 q + l2 q^2 + q^3 with l2 = 6u^2+1, l1 = -36u^3-18u^2-12u+1,
// l0 = -36u^3-30u^2-18u-2 (an identity of integers, checked in
// tests/test_bn254_pairing_oracle.py): three exponentiations by u, a few small powers,
// Frobenius maps, and conjugation for the negative coefficients (the input of the hard
// part lies in the cyclotomic subgroup, where inversion is conjugation).
//
// Fq elements in Montgomery form inside kernels; the ABI carries canonical little-endian
// limbs (GT: 12 Fq in tower order c0.a0, c0.a1, c0.a2, c1.a0, c1.a1, c1.a2 = w^0, w^2,
// w^4, w^1, w^3, w^5).
#include <vector>
#include "../../include/pbf.h"
#include "ec_bn254.hpp"
#include "internal.hpp"

namespace pbf {

// ---------------------------------------------------------------- constants
// Generated from q and u alone by scripts/gen_pairing_constants.py (canonical, little-endian):
//   FROB1[k] = xi^(k(q-1)/6) (Fq2, k = 0..5): w^k -> w^(kq) = FROB1[k] w^k
//   GX = FROB1[2], GY = FROB1[3] (twist Frobenius pi(x, y) = (conj(x) GX, conj(y) GY))
//   FROB2[k] = xi^(k(q^2-1)/6) (in Fq), R3 = 2^768 mod q, ATE = 6u+2, BN_U = u
struct PairingConsts {
  U256 frob1[6][2];         // Montgomery
  U256 frob2[6];            // Montgomery
  U256 one;                 // Montgomery 1
  U256 r3;                  // plain 2^768 mod q (binary-Euclid inverse -> Montgomery)
  uint64_t ate;             // low 64 bits of 6u+2 (bit 64 is set too)
};

static const uint64_t K_FROB1[6][2][4] = {
    {{0x0000000000000001ull, 0x0000000000000000ull, 0x0000000000000000ull, 0x0000000000000000ull},
     {0x0000000000000000ull, 0x0000000000000000ull, 0x0000000000000000ull, 0x0000000000000000ull}},
    {{0xd60b35dadcc9e470ull, 0x5c521e08292f2176ull, 0xe8b99fdd76e68b60ull, 0x1284b71c2865a7dfull},
     {0xca5cf05f80f362acull, 0x747992778eeec7e5ull, 0xa6327cfe12150b8eull, 0x246996f3b4fae7e6ull}},
    {{0x99e39557176f553dull, 0xb78cc310c2c3330cull, 0x4c0bec3cf559b143ull, 0x2fb347984f7911f7ull},
     {0x1665d51c640fcba2ull, 0x32ae2a1d0b7c9dceull, 0x4ba4cc8bd75a0794ull, 0x16c9e55061ebae20ull}},
    {{0xdc54014671a0135aull, 0xdbaae0eda9c95998ull, 0xdc5ec698b6e2f9b9ull, 0x063cf305489af5dcull},
     {0x82d37f632623b0e3ull, 0x21807dc98fa25bd2ull, 0x0704b5a7ec796f2bull, 0x07c03cbcac41049aull}},
    {{0x848a1f55921ea762ull, 0xd33365f7be94ec72ull, 0x80f3c0b75a181e84ull, 0x05b54f5e64eea801ull},
     {0xc13b4711cd2b8126ull, 0x3685d2ea1bdec763ull, 0x9f3a80b03b0b1c92ull, 0x2c145edbe7fd8aeeull}},
    {{0x2ea2c810eab7692full, 0x425c459b55aa1bd3ull, 0xe93a3661a4353ff4ull, 0x0183c1e74f798649ull},
     {0x24c6b8ee6e0c2c4bull, 0xb080cb99678e2ac0ull, 0xa27fb246c7729f7dull, 0x12acf2ca76fd0675ull}}};
static const uint64_t K_FROB2[6][4] = {
    {0x0000000000000001ull, 0, 0, 0},
    {0xe4bd44e5607cfd49ull, 0xc28f069fbb966e3dull, 0x5e6dd9e7e0acccb0ull, 0x30644e72e131a029ull},
    {0xe4bd44e5607cfd48ull, 0xc28f069fbb966e3dull, 0x5e6dd9e7e0acccb0ull, 0x30644e72e131a029ull},
    {0x3c208c16d87cfd46ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
    {0x5763473177fffffeull, 0xd4f263f1acdb5c4full, 0x59e26bcea0d48bacull, 0x0000000000000000ull},
    {0x5763473177ffffffull, 0xd4f263f1acdb5c4full, 0x59e26bcea0d48bacull, 0x0000000000000000ull}};
static const uint64_t K_R3[4] = {0xb1cd6dafda1530dfull, 0x62f210e6a7283db6ull, 0xef7f0b0c0ada0afbull,
                                 0x20fd6e902d592544ull};
static const uint64_t K_ATE_LO = 0x9d797039be763ba8ull;  // 6u+2 = 2^64 + K_ATE_LO
constexpr uint64_t K_BN_U = 0x44e992b44a6909f1ull;  // u = 4965661367192848881

// ---------------------------------------------------------------- Fq / Fq2 (one lane)
struct Fq2 {
  U256 c0, c1;
};

__device__ __forceinline__ Fq2 f2_add(const Fq2& a, const Fq2& b) { return {Fq::add(a.c0, b.c0), Fq::add(a.c1, b.c1)}; }
__device__ __forceinline__ Fq2 f2_sub(const Fq2& a, const Fq2& b) { return {Fq::sub(a.c0, b.c0), Fq::sub(a.c1, b.c1)}; }
__device__ __forceinline__ Fq2 f2_neg(const Fq2& a) { return {Fq::sub(u256_zero(), a.c0), Fq::sub(u256_zero(), a.c1)}; }
__device__ __forceinline__ Fq2 f2_dbl(const Fq2& a) { return f2_add(a, a); }
__device__ __forceinline__ Fq2 f2_conj(const Fq2& a) { return {a.c0, Fq::sub(u256_zero(), a.c1)}; }
__device__ __forceinline__ Fq2 f2_muls(const Fq2& a, const U256& s) { return {Fq::mul(a.c0, s), Fq::mul(a.c1, s)}; }
__device__ __forceinline__ Fq2 f2_mul(const Fq2& a, const Fq2& b) {
  // Karatsuba: (a0 b0 - a1 b1) + ((a0 + a1)(b0 + b1) - a0 b0 - a1 b1) u
  const U256 t0 = Fq::mul(a.c0, b.c0), t1 = Fq::mul(a.c1, b.c1);
  const U256 t2 = Fq::mul(Fq::add(a.c0, a.c1), Fq::add(b.c0, b.c1));
  return {Fq::sub(t0, t1), Fq::sub(Fq::sub(t2, t0), t1)};
}
__device__ __forceinline__ Fq2 f2_sqr(const Fq2& a) {
  // (a0 + a1)(a0 - a1) + 2 a0 a1 u
  const U256 t = Fq::mul(a.c0, a.c1);
  return {Fq::mul(Fq::add(a.c0, a.c1), Fq::sub(a.c0, a.c1)), Fq::add(t, t)};
}
// (9 + u)(a0 + a1 u) = (9 a0 - a1) + (a0 + 9 a1) u
__device__ __forceinline__ Fq2 f2_mul_xi(const Fq2& a) {
  auto nine = [](const U256& x) {
    const U256 x2 = Fq::add(x, x), x4 = Fq::add(x2, x2), x8 = Fq::add(x4, x4);
    return Fq::add(x8, x);
  };
  return {Fq::sub(nine(a.c0), a.c1), Fq::add(a.c0, nine(a.c1))};
}
__device__ __forceinline__ bool f2_eq(const Fq2& a, const Fq2& b) { return Fq::eq(a.c0, b.c0) && Fq::eq(a.c1, b.c1); }
__device__ __forceinline__ bool f2_is_zero(const Fq2& a) { return Fq::is_zero(a.c0) && Fq::is_zero(a.c1); }

__device__ __forceinline__ bool u256_is_one(const U256& a) {
  uint32_t o = a.w[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < 8; ++i) o |= a.w[i];
  return o == 0;
}
__device__ __forceinline__ bool u256_geq(const U256& a, const U256& b) {
#pragma unroll
  for (int i = 7; i >= 0; --i)
    if (a.w[i] != b.w[i]) return a.w[i] > b.w[i];
  return true;
}
__device__ __forceinline__ void u256_shr1(U256& a) {
#pragma unroll
  for (int i = 0; i < 7; ++i) a.w[i] = (a.w[i] >> 1) | (a.w[i + 1] << 31);
  a.w[7] >>= 1;
}
__device__ __forceinline__ U256 u256_sub_raw(const U256& a, const U256& b) {
  U256 d;
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t t = (uint64_t)a.w[i] - b.w[i] - borrow;
    d.w[i] = (uint32_t)t;
    borrow = (t >> 63) & 1;
  }
  return d;
}
// x / 2 mod q for canonical x (x odd: (x + q) / 2 < q, no overflow since q < 2^254)
__device__ __forceinline__ void fq_half(U256& x) {
  if (x.w[0] & 1) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t t = (uint64_t)x.w[i] + Bn254FqParams::P[i] + c;
      x.w[i] = (uint32_t)t;
      c = t >> 32;
    }
  }
  u256_shr1(x);
}
// Montgomery inverse (aR)^-1 -> a^-1 R: binary extended Euclid on the representative, then
// one Montgomery product with R^3 ((aR)^-1 R^3 R^-1 = a^-1 R). a != 0.
__device__ __noinline__ U256 fq_inv(const U256& am, const PairingConsts& k) {
  U256 u = am, v, x1 = u256_zero(), x2 = u256_zero();
#pragma unroll
  for (int i = 0; i < 8; ++i) v.w[i] = Bn254FqParams::P[i];
  x1.w[0] = 1;
  if (Fq::is_zero(am)) return u256_zero();  // no inverse (callers never pass 0)
  // gcd(a, q) = 1: each round removes >= 1 bit from u or v, so <= 2 * 256 rounds; the cap
  // only guards the exit
  for (int round = 0; round < 1024 && !u256_is_one(u) && !u256_is_one(v); ++round) {
    while (!(u.w[0] & 1)) { u256_shr1(u); fq_half(x1); }
    while (!(v.w[0] & 1)) { u256_shr1(v); fq_half(x2); }
    if (u256_geq(u, v)) {
      u = u256_sub_raw(u, v);
      x1 = Fq::sub(x1, x2);
    } else {
      v = u256_sub_raw(v, u);
      x2 = Fq::sub(x2, x1);
    }
  }
  return Fq::mul(u256_is_one(u) ? x1 : x2, k.r3);
}
__device__ __forceinline__ Fq2 f2_inv(const Fq2& a, const PairingConsts& k) {
  const U256 ni = fq_inv(Fq::add(Fq::mul(a.c0, a.c0), Fq::mul(a.c1, a.c1)), k);
  return {Fq::mul(a.c0, ni), Fq::sub(u256_zero(), Fq::mul(a.c1, ni))};
}

// ---------------------------------------------------------------- wave-cooperative Fq12
// Every function below is called by all 64 lanes of the (single-wave) workgroup and ends
// with a barrier; operands and results are flat Fq12 (6 Fq2) in LDS and may alias.
// Miller-step slots: T = (X : Y : Z), the affine point added (xq, yq), P as Fq2 (xp, 0),
// (yp, 0), the line's w^0, w^1, w^3 coefficients, temporaries from SL_T
enum { SL_X, SL_Y, SL_Z, SL_XQ, SL_YQ, SL_XP, SL_YP, SL_L0, SL_L1, SL_L3, SL_T };

struct PairLds {
  Fq2 prod[36];    // partial products
  Fq2 reg[14][6];  // Fq12 registers
  Fq2 sl[32];      // Miller-step slots (SL_* above)
  Fq2 Qa[3][2];    // Q, pi(Q), -pi^2(Q) affine
  Fq2 frob1[6];    // the lane-indexed constants (a lane-indexed kernel argument would be
  U256 frob2[6];   // copied to scratch)
};

// constants -> LDS with compile-time indices
__device__ __forceinline__ void load_consts(const PairingConsts& k, PairLds& L, int lane) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    if (lane == i) {
      L.frob1[i] = Fq2{k.frob1[i][0], k.frob1[i][1]};
      L.frob2[i] = k.frob2[i];
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void wsync() { __syncthreads(); }

// dst = x * y: 36 Fq2 products (one per lane, x xi for the wrapped terms), then 6 lanes
// sum them (a three-level Karatsuba split into 54 Fq products measured slower: its operand
// selection diverges across lanes and adds three reconstruction stages)
__device__ __forceinline__ void w12_mul(Fq2* dst, const Fq2* x, const Fq2* y, PairLds& L, int lane) {
  if (lane < 36) {
    const int i = lane / 6, j = lane - 6 * (lane / 6);
    // one f2_mul for every lane (a separate squaring path for the diagonal would only
    // serialise two code paths across the wave)
    Fq2 p = f2_mul(x[i], y[j]);
    if (i + j >= 6) p = f2_mul_xi(p);
    L.prod[lane] = p;
  }
  wsync();
  if (lane < 6) {
    Fq2 s = L.prod[lane];  // i = 0, j = lane
#pragma unroll
    for (int i = 1; i < 6; ++i) {
      const int j = lane - i < 0 ? lane - i + 6 : lane - i;
      s = f2_add(s, L.prod[6 * i + j]);
    }
    dst[lane] = s;
  }
  wsync();
}
// f *= line (coefficients at w^0, w^1, w^3)
__device__ __forceinline__ void w12_mul_line(Fq2* f, PairLds& L, int lane) {
  if (lane < 18) {
    const int i = lane / 3, jj = lane - 3 * (lane / 3);
    const int j = jj == 2 ? 3 : jj;
    Fq2 p = f2_mul(f[i], L.sl[SL_L0 + jj]);
    if (i + j >= 6) p = f2_mul_xi(p);
    L.prod[6 * i + j] = p;
  }
  wsync();
  if (lane < 6) {
    Fq2 s;
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      const int j = jj == 2 ? 3 : jj;
      const int i = lane - j < 0 ? lane - j + 6 : lane - j;
      s = jj == 0 ? L.prod[6 * i + j] : f2_add(s, L.prod[6 * i + j]);
    }
    f[lane] = s;
  }
  wsync();
}
__device__ __forceinline__ void w12_copy(Fq2* dst, const Fq2* x, int lane) {
  if (lane < 6) dst[lane] = x[lane];
  wsync();
}
// x^(q^6): w -> -w
__device__ __forceinline__ void w12_conj(Fq2* dst, const Fq2* x, int lane) {
  if (lane < 6) dst[lane] = (lane & 1) ? f2_neg(x[lane]) : x[lane];
  wsync();
}
// x^q: g_k -> conj(g_k) FROB1[k]
__device__ __forceinline__ void w12_frob1(Fq2* dst, const Fq2* x, PairLds& L, int lane) {
  if (lane < 6) dst[lane] = lane == 0 ? f2_conj(x[0]) : f2_mul(f2_conj(x[lane]), L.frob1[lane]);
  wsync();
}
// x^(q^2): g_k -> g_k FROB2[k]
__device__ __forceinline__ void w12_frob2(Fq2* dst, const Fq2* x, PairLds& L, int lane) {
  if (lane < 6) dst[lane] = lane == 0 ? x[0] : f2_muls(x[lane], L.frob2[lane]);
  wsync();
}
__device__ __forceinline__ void w12_one(Fq2* dst, const PairingConsts& k, int lane) {
  if (lane < 6) dst[lane] = Fq2{lane == 0 ? k.one : u256_zero(), u256_zero()};
  wsync();
}
// In-place inverse of the Fq6 element n0 + n1 v + n2 v^2 held at flat slots 0, 2, 4 of n
// (one lane; one Fq inversion)
__device__ __noinline__ void fq6_inv_flat(Fq2* n, const PairingConsts& k) {
  const Fq2 n0 = n[0], n1 = n[2], n2 = n[4];
  const Fq2 t0 = f2_sub(f2_sqr(n0), f2_mul_xi(f2_mul(n1, n2)));
  const Fq2 t1 = f2_sub(f2_mul_xi(f2_sqr(n2)), f2_mul(n0, n1));
  const Fq2 t2 = f2_sub(f2_sqr(n1), f2_mul(n0, n2));
  const Fq2 den = f2_add(f2_mul(n0, t0), f2_mul_xi(f2_add(f2_mul(n2, t1), f2_mul(n1, t2))));
  const Fq2 di = f2_inv(den, k);
  const Fq2 z{u256_zero(), u256_zero()};
  n[0] = f2_mul(t0, di);
  n[1] = z;
  n[2] = f2_mul(t1, di);
  n[3] = z;
  n[4] = f2_mul(t2, di);
  n[5] = z;
}

// The final exponentiation as a program over the LDS Fq12 registers, run by one
// interpreter loop: one inlined copy of each wave primitive and no calls (a call would
// save and restore the callee's VGPRs through scratch every time).
enum : uint8_t { FE_MUL, FE_CONJ, FE_FROB1, FE_FROB2, FE_COPY, FE_INVN };
struct FeOp {
  uint8_t op, dst, a, b;
};
constexpr int FE_MAX = 320;
struct FeProg {
  FeOp ops[FE_MAX];
  int n;
};
// registers: 0 f (in/out), 1 a = f^u, 2 b = f^u^2, 3 c = f^u^3, 4..11 temporaries, 12, 13 inverse
constexpr FeProg make_fe_prog() {
  FeProg p{};
  int n = 0;
  auto op = [&](uint8_t o, int d, int a, int b) { p.ops[n++] = FeOp{o, (uint8_t)d, (uint8_t)a, (uint8_t)b}; };
  auto mul = [&](int d, int a, int b) { op(FE_MUL, d, a, b); };
  auto powu = [&](int d, int x) {  // d = x^u, u = K_BN_U (63 bits)
    op(FE_COPY, d, x, 0);
    for (int bit = 61; bit >= 0; --bit) {
      mul(d, d, d);
      if ((K_BN_U >> bit) & 1) mul(d, d, x);
    }
  };
  // easy part: f^(q^6-1) = conj(f) / f (f^-1 = conj(f) * (f conj(f))^-1), then ^(q^2+1)
  op(FE_CONJ, 12, 0, 0);
  mul(13, 0, 12);
  op(FE_INVN, 13, 0, 0);
  mul(4, 12, 13);          // f^-1
  mul(0, 12, 4);           // conj(f) f^-1
  op(FE_FROB2, 4, 0, 0);
  mul(0, 4, 0);
  // hard part: l0 + l1 q + l2 q^2 + q^3 (see file header)
  powu(1, 0);
  powu(2, 1);
  powu(3, 2);
  mul(7, 3, 3); mul(7, 7, 7);                   // c^4
  mul(4, 7, 7); mul(4, 4, 4); mul(4, 4, 4);     // c^32
  mul(4, 4, 7);                                 // c^36
  mul(7, 2, 2); mul(10, 7, 7); mul(10, 10, 7);  // b^2, b^4, b^6
  mul(8, 10, 10); mul(9, 8, 10);                // b^12, b^18
  mul(8, 8, 8); mul(8, 8, 10);                  // b^24, b^30
  mul(7, 1, 1); mul(11, 7, 7); mul(11, 11, 7);  // a^2, a^4, a^6
  mul(7, 11, 11); mul(11, 7, 11);               // a^12, a^18
  mul(5, 4, 9); mul(5, 5, 7); op(FE_CONJ, 5, 5, 0); mul(5, 5, 0);  // f^l1
  mul(6, 10, 0);                                                  // f^l2
  mul(4, 4, 8); mul(4, 4, 11); mul(7, 0, 0); mul(4, 4, 7); op(FE_CONJ, 4, 4, 0);  // f^l0
  op(FE_FROB1, 7, 5, 0); mul(4, 4, 7);
  op(FE_FROB2, 7, 6, 0); mul(4, 4, 7);
  op(FE_FROB1, 7, 0, 0); op(FE_FROB2, 8, 7, 0); mul(0, 4, 8);
  p.n = n;
  return p;
}
__constant__ FeProg c_fe_prog = make_fe_prog();
static_assert(make_fe_prog().n <= FE_MAX, "program size");

// result = f^((q^12-1)/r), f in L.reg[0]; result in L.reg[0]
__device__ __forceinline__ void final_exp_w(const PairingConsts& k, PairLds& L, int lane) {
  const int n = c_fe_prog.n;
  for (int pc = 0; pc < n; ++pc) {
    const FeOp o = c_fe_prog.ops[pc];
    Fq2* d = L.reg[o.dst];
    const Fq2* a = L.reg[o.a];
    switch (o.op) {
      case FE_MUL: w12_mul(d, a, L.reg[o.b], L, lane); break;
      case FE_CONJ: w12_conj(d, a, lane); break;
      case FE_FROB1: w12_frob1(d, a, L, lane); break;
      case FE_FROB2: w12_frob2(d, a, L, lane); break;
      case FE_COPY: w12_copy(d, a, lane); break;
      default:  // FE_INVN
        if (lane == 0) fq6_inv_flat(d, k);
        wsync();
        break;
    }
  }
}

// ---------------------------------------------------------------- Miller loop (wave)
// T = (X : Y : Z) homogeneous on the twist, P = (xp, yp) affine in G1 (Montgomery).
// Doubling: w = 3X^2, s = 2YZ, R = Ys, B = (X+R)^2 - X^2 - R^2, h = w^2 - 2B,
//   X3 = h s, Y3 = w (B - h) - 2 R^2, Z3 = s^3;
//   line * s Z: (s Z) yp - (w Z) xp w + (w X - R) v w   (v w = w^3)
// Mixed addition T += (xq, yq): N = yq Z - Y, D = xq Z - X,
//   A = N^2 Z - D^3 - 2 D^2 X, X3 = D A, Y3 = N (D^2 X - A) - D^3 Y, Z3 = D^3 Z;
//   line * D: D yp - N xp w + (N xq - D yq) v w
// Both steps are micro-op programs over the slot file: a MULS group is up to 6
// independent Fq2 products, one per lane (one inlined f2_mul for the whole wave); a LIN
// group is a short run of additions on lane 0; F12 ops update f. One interpreter loop
// runs them, so the kernel holds one copy of each primitive (I-cache, registers).
enum : uint8_t { U_MULS, U_LIN, U_F12SQR, U_F12LINE, L_ADD, L_SUB, L_DBL, L_TRP, L_NEG, L_COPY, U_MUL };
struct Uop {
  uint8_t code, d, a, b;
};
#define MUL(d, a, b) Uop{U_MUL, (uint8_t)(d), (uint8_t)(a), (uint8_t)(b)}
#define LIN(c, d, a, b) Uop{c, (uint8_t)(d), (uint8_t)(a), (uint8_t)(b)}
#define GRP(c, n) Uop{c, (uint8_t)(n), 0, 0}
constexpr int T0 = SL_T;
__constant__ Uop c_dbl_prog[] = {
    GRP(U_MULS, 2), MUL(T0 + 0, SL_X, SL_X), MUL(T0 + 1, SL_Y, SL_Z),                // X^2, YZ
    GRP(U_LIN, 2), LIN(L_TRP, T0 + 2, T0 + 0, 0), LIN(L_DBL, T0 + 3, T0 + 1, 0),    // w, s
    GRP(U_MULS, 6), MUL(T0 + 4, T0 + 3, T0 + 3), MUL(T0 + 5, SL_Y, T0 + 3),          // s^2, R
    MUL(T0 + 6, T0 + 3, SL_Z), MUL(T0 + 7, T0 + 2, SL_Z),                            // sZ, wZ
    MUL(T0 + 8, T0 + 2, SL_X), MUL(T0 + 9, T0 + 2, T0 + 2),                          // wX, w^2
    GRP(U_LIN, 1), LIN(L_ADD, T0 + 10, SL_X, T0 + 5),                                // X + R
    GRP(U_MULS, 5), MUL(T0 + 11, T0 + 3, T0 + 4), MUL(T0 + 12, T0 + 5, T0 + 5),      // s^3, R^2
    MUL(T0 + 13, T0 + 10, T0 + 10), MUL(SL_L0, T0 + 6, SL_YP), MUL(T0 + 14, T0 + 7, SL_XP),
    GRP(U_LIN, 9), LIN(L_NEG, SL_L1, T0 + 14, 0), LIN(L_SUB, SL_L3, T0 + 8, T0 + 5),
    LIN(L_SUB, T0 + 15, T0 + 13, T0 + 0), LIN(L_SUB, T0 + 15, T0 + 15, T0 + 12),     // B
    LIN(L_DBL, T0 + 16, T0 + 15, 0), LIN(L_SUB, T0 + 16, T0 + 9, T0 + 16),           // h
    LIN(L_SUB, T0 + 17, T0 + 15, T0 + 16), LIN(L_DBL, T0 + 18, T0 + 12, 0),          // B - h, 2R^2
    LIN(L_COPY, SL_Z, T0 + 11, 0),                                                    // Z3
    GRP(U_MULS, 2), MUL(SL_X, T0 + 16, T0 + 3), MUL(T0 + 19, T0 + 2, T0 + 17),         // X3, w(B-h)
    GRP(U_LIN, 1), LIN(L_SUB, SL_Y, T0 + 19, T0 + 18),                                // Y3
    GRP(U_F12SQR, 0), GRP(U_F12LINE, 0)};
__constant__ Uop c_add_prog[] = {
    GRP(U_MULS, 2), MUL(T0 + 0, SL_YQ, SL_Z), MUL(T0 + 1, SL_XQ, SL_Z),
    GRP(U_LIN, 2), LIN(L_SUB, T0 + 2, T0 + 0, SL_Y), LIN(L_SUB, T0 + 3, T0 + 1, SL_X),  // N, D
    GRP(U_MULS, 6), MUL(T0 + 4, T0 + 2, T0 + 2), MUL(T0 + 5, T0 + 3, T0 + 3),         // N^2, D^2
    MUL(T0 + 6, T0 + 2, SL_XQ), MUL(T0 + 7, T0 + 3, SL_YQ),                           // N xq, D yq
    MUL(SL_L0, T0 + 3, SL_YP), MUL(T0 + 8, T0 + 2, SL_XP),                            // D yp, N xp
    GRP(U_LIN, 2), LIN(L_NEG, SL_L1, T0 + 8, 0), LIN(L_SUB, SL_L3, T0 + 6, T0 + 7),
    GRP(U_MULS, 3), MUL(T0 + 9, T0 + 3, T0 + 5), MUL(T0 + 10, T0 + 5, SL_X),          // D^3, D^2 X
    MUL(T0 + 11, T0 + 4, SL_Z),                                                       // N^2 Z
    GRP(U_LIN, 4), LIN(L_SUB, T0 + 12, T0 + 11, T0 + 9), LIN(L_DBL, T0 + 13, T0 + 10, 0),
    LIN(L_SUB, T0 + 12, T0 + 12, T0 + 13), LIN(L_SUB, T0 + 14, T0 + 10, T0 + 12),    // A, D^2X - A
    GRP(U_MULS, 4), MUL(T0 + 15, T0 + 3, T0 + 12), MUL(T0 + 16, T0 + 9, SL_Z),
    MUL(T0 + 17, T0 + 2, T0 + 14), MUL(T0 + 18, T0 + 9, SL_Y),
    GRP(U_LIN, 3), LIN(L_COPY, SL_X, T0 + 15, 0), LIN(L_COPY, SL_Z, T0 + 16, 0),
    LIN(L_SUB, SL_Y, T0 + 17, T0 + 18),
    GRP(U_F12LINE, 0)};
#undef MUL
#undef LIN
#undef GRP
constexpr int DBL_LEN = sizeof(c_dbl_prog) / sizeof(Uop), ADD_LEN = sizeof(c_add_prog) / sizeof(Uop);
static_assert(SL_T + 20 <= 32, "slot file");

__device__ __forceinline__ void run_uops(const Uop* prog, int len, Fq2* f, PairLds& L, int lane) {
  Fq2* sl = L.sl;
  for (int pc = 0; pc < len;) {
    const Uop u = prog[pc];
    if (u.code == U_MULS) {
      if (lane < u.d) {
        const Uop m = prog[pc + 1 + lane];
        sl[m.d] = f2_mul(sl[m.a], sl[m.b]);
      }
      wsync();
      pc += 1 + u.d;
    } else if (u.code == U_LIN) {
      if (lane == 0) {
        for (int i = 0; i < u.d; ++i) {
          const Uop m = prog[pc + 1 + i];
          const Fq2 a = sl[m.a], b = sl[m.b];
          Fq2 r;
          switch (m.code) {
            case L_ADD: r = f2_add(a, b); break;
            case L_SUB: r = f2_sub(a, b); break;
            case L_DBL: r = f2_dbl(a); break;
            case L_TRP: r = f2_add(f2_dbl(a), a); break;
            case L_NEG: r = f2_neg(a); break;
            default: r = a; break;  // L_COPY
          }
          sl[m.d] = r;
        }
      }
      wsync();
      pc += 1 + u.d;
    } else if (u.code == U_F12SQR) {
      w12_mul(f, f, f, L, lane);
      ++pc;
    } else {  // U_F12LINE
      w12_mul_line(f, L, lane);
      ++pc;
    }
  }
}

// ---------------------------------------------------------------- ABI <-> device layouts
__device__ inline U256 ld_mont(const uint64_t* p) { return Fq::to_mont(u256_from_u64(p)); }
__device__ inline void st_canon(uint64_t* p, const U256& a) { u256_to_u64(Fq::from_mont(a), p); }
__device__ inline bool all_zero(const uint64_t* p, int n) {
  uint64_t o = 0;
  for (int i = 0; i < n; ++i) o |= p[i];
  return o == 0;
}
// flat index k (w^k) -> ABI tower slot: c0.a0 c0.a1 c0.a2 c1.a0 c1.a1 c1.a2 = w^0 w^2 w^4 w^1 w^3 w^5
__device__ __forceinline__ int tower_slot(int k) { return (k & 1) ? 3 + (k >> 1) : (k >> 1); }

// Miller value of pair i into f (all lanes); identity inputs -> 1
__device__ __forceinline__ void miller_w(Fq2* f, const uint64_t* g1, const uint64_t* g2, size_t i,
                                         const PairingConsts& k, PairLds& L, int lane) {
  const uint64_t* p = g1 + 8 * i;
  const uint64_t* q = g2 + 16 * i;
  w12_one(f, k, lane);
  if (all_zero(p, 8) || all_zero(q, 16)) return;  // uniform across the wave
  if (lane == 0) {
    const Fq2 xq{ld_mont(q), ld_mont(q + 4)}, yq{ld_mont(q + 8), ld_mont(q + 12)};
    L.Qa[0][0] = xq;
    L.Qa[0][1] = yq;
    L.sl[SL_X] = xq;
    L.sl[SL_Y] = yq;
    L.sl[SL_Z] = Fq2{k.one, u256_zero()};
    L.sl[SL_XQ] = xq;
    L.sl[SL_YQ] = yq;
    L.sl[SL_XP] = Fq2{ld_mont(p), u256_zero()};
    L.sl[SL_YP] = Fq2{ld_mont(p + 4), u256_zero()};
    // pi(Q) = (conj(x) GX, conj(y) GY), -pi^2(Q) = (conj(x1) GX, -conj(y1) GY)
    const Fq2 gx = L.frob1[2], gy = L.frob1[3];
    const Fq2 x1 = f2_mul(f2_conj(xq), gx), y1 = f2_mul(f2_conj(yq), gy);
    L.Qa[1][0] = x1;
    L.Qa[1][1] = y1;
    L.Qa[2][0] = f2_mul(f2_conj(x1), gx);
    L.Qa[2][1] = f2_neg(f2_mul(f2_conj(y1), gy));
  }
  wsync();
  // bits 63..0 of 6u+2 below its leading bit: double, and add Q on a one; then T + pi(Q)
  // and T - pi^2(Q). One run_uops call site (one inlined copy of the step code).
  int b = 63;
  bool dbl = true;
  while (b >= -2) {
    if (!dbl && b < 0) {
      if (lane == 0) {
        L.sl[SL_XQ] = L.Qa[b == -1 ? 1 : 2][0];
        L.sl[SL_YQ] = L.Qa[b == -1 ? 1 : 2][1];
      }
      wsync();
    }
    run_uops(dbl ? c_dbl_prog : c_add_prog, dbl ? DBL_LEN : ADD_LEN, f, L, lane);
    // next step: after a doubling at bit b, the addition if bit b is set; else the next bit
    if (dbl && ((k.ate >> b) & 1)) {
      dbl = false;
    } else {
      --b;
      dbl = b >= 0;
    }
  }
}

__device__ __forceinline__ void store_f12_canon(uint64_t* out, const Fq2* f, int lane) {
  if (lane < 6) {
    const int s = tower_slot(lane);
    st_canon(out + 8 * s, f[lane].c0);
    st_canon(out + 8 * s + 4, f[lane].c1);
  }
}

// one pairing per workgroup (one wave)
__global__ void __launch_bounds__(64) pairing_kernel(const uint64_t* g1, const uint64_t* g2, size_t n, uint64_t* out,
                                                     PairingConsts k) {
  __shared__ PairLds L;
  const int lane = threadIdx.x;
  const size_t i = blockIdx.x;
  if (i >= n) return;
  load_consts(k, L, lane);
  miller_w(L.reg[0], g1, g2, i, k, L, lane);
  final_exp_w(k, L, lane);
  store_f12_canon(out + 48 * i, L.reg[0], lane);
}

// Miller value of pair i, raw Montgomery flat Fq12 (scratch layout)
__global__ void __launch_bounds__(64) miller_kernel(const uint64_t* g1, const uint64_t* g2, size_t n, uint64_t* acc,
                                                    PairingConsts k) {
  __shared__ PairLds L;
  const int lane = threadIdx.x;
  const size_t i = blockIdx.x;
  if (i >= n) return;
  load_consts(k, L, lane);
  miller_w(L.reg[0], g1, g2, i, k, L, lane);
  if (lane < 6) {
    u256_to_u64(L.reg[0][lane].c0, acc + 48 * i + 8 * lane);
    u256_to_u64(L.reg[0][lane].c1, acc + 48 * i + 8 * lane + 4);
  }
}

// product of the n Miller values, final exponentiation, compare with 1
__global__ void __launch_bounds__(64) pairing_check_final(const uint64_t* acc, size_t n, int* ok, PairingConsts k) {
  __shared__ PairLds L;
  const int lane = threadIdx.x;
  Fq2* f = L.reg[0];
  Fq2* g = L.reg[12];
  load_consts(k, L, lane);
  w12_one(f, k, lane);
  for (size_t i = 0; i < n; ++i) {
    if (lane < 6) {
      g[lane].c0 = u256_from_u64(acc + 48 * i + 8 * lane);
      g[lane].c1 = u256_from_u64(acc + 48 * i + 8 * lane + 4);
    }
    wsync();
    w12_mul(f, f, g, L, lane);
  }
  final_exp_w(k, L, lane);
  if (lane == 0) {
    bool eq = Fq::eq(f[0].c0, k.one) && Fq::is_zero(f[0].c1);
    for (int j = 1; j < 6; ++j) eq = eq && f2_is_zero(f[j]);
    *ok = eq ? 1 : 0;
  }
}

// ---------------------------------------------------------------- G2 scalar multiplication
struct G2A {
  Fq2 x, y;
};


// out_i = s_i * Q_i (affine double-and-add, LSB first like the reference's G2P::mul,
// src/pbh/g2.rs:82-101; identity and P + (-P) handled). Used for the SRS's [s]G2.
__global__ void __launch_bounds__(64) g2_mul_kernel(const uint64_t* pts, const uint64_t* sc, size_t n, uint64_t* out,
                                                    PairingConsts k) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t* q = pts + 16 * i;
  bool base_inf = all_zero(q, 16);
  G2A b{{ld_mont(q), ld_mont(q + 4)}, {ld_mont(q + 8), ld_mont(q + 12)}};
  G2A acc = b;
  bool acc_inf = true;
  const U256 three = Fq::add(Fq::add(k.one, k.one), k.one);
  auto add = [&](G2A& r, bool& rinf, const G2A& p, bool pinf) {
    if (pinf) return;
    if (rinf) { r = p; rinf = false; return; }
    Fq2 lam;
    if (f2_eq(r.x, p.x)) {
      if (!f2_eq(r.y, p.y) || f2_is_zero(p.y)) { rinf = true; return; }  // P + (-P)
      lam = f2_mul(f2_muls(f2_sqr(p.x), three), f2_inv(f2_dbl(p.y), k));
    } else {
      lam = f2_mul(f2_sub(p.y, r.y), f2_inv(f2_sub(p.x, r.x), k));
    }
    const Fq2 x3 = f2_sub(f2_sub(f2_sqr(lam), r.x), p.x);
    r.y = f2_sub(f2_mul(lam, f2_sub(r.x, x3)), r.y);
    r.x = x3;
  };
  for (int w = 0; w < 4; ++w) {
    const uint64_t s = sc[4 * i + w];
    for (int bit = 0; bit < 64; ++bit) {
      if ((s >> bit) & 1) add(acc, acc_inf, b, base_inf);
      G2A b2 = b;
      bool b2inf = base_inf;
      add(b, base_inf, b2, b2inf);
    }
  }
  uint64_t* o = out + 16 * i;
  if (acc_inf) {
    for (int j = 0; j < 16; ++j) o[j] = 0;
  } else {
    st_canon(o, acc.x.c0); st_canon(o + 4, acc.x.c1); st_canon(o + 8, acc.y.c0); st_canon(o + 12, acc.y.c1);
  }
}

static PairingConsts make_consts() {
  PairingConsts k;
  for (int i = 0; i < 6; ++i)
    for (int c = 0; c < 2; ++c) k.frob1[i][c] = Fq::to_mont(u256_from_u64(K_FROB1[i][c]));
  for (int i = 0; i < 6; ++i) k.frob2[i] = Fq::to_mont(u256_from_u64(K_FROB2[i]));
  k.one = Fq::to_mont(Fq::one_plain());
  k.r3 = u256_from_u64(K_R3);
  k.ate = K_ATE_LO;
  return k;
}

// canonical-input validation on the host (x, y < q for every coordinate)
static bool canonical_fq(const uint64_t* l) {
  static const uint64_t QL[4] = {0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull,
                                 0x30644e72e131a029ull};
  for (int i = 3; i >= 0; --i) {
    if (l[i] != QL[i]) return l[i] < QL[i];
  }
  return false;
}

}  // namespace pbf

using namespace pbf;

static int check_coords(const uint64_t* v, size_t count) {
  for (size_t i = 0; i < count; ++i)
    if (!canonical_fq(v + 4 * i)) return fail(1, "coordinate not canonical (>= q)");
  return 0;
}

extern "C" int pbf_pairing_bn254(pbf_ctx* ctx, const uint64_t* g1, const uint64_t* g2, size_t n, uint64_t* out) {
  if (!ctx || (n && (!g1 || !g2 || !out))) return fail(1, "null argument");
  if (n == 0) return 0;
  if (n > 0x7fffffffu) return fail(1, "batch too large");
  int rc = check_coords(g1, 2 * n);
  if (!rc) rc = check_coords(g2, 4 * n);
  if (rc) return rc;
  hipStream_t s = ctx->host_stream();
  if ((rc = ctx->io0.ensure(n * 64)) || (rc = ctx->io1.ensure(n * 128)) || (rc = ctx->io2.ensure(n * 384))) return rc;
  PBF_HIP(hipMemcpyAsync(ctx->io0.p, g1, n * 64, hipMemcpyHostToDevice, s));
  PBF_HIP(hipMemcpyAsync(ctx->io1.p, g2, n * 128, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(pairing_kernel, dim3(n), dim3(64), 0, s, (const uint64_t*)ctx->io0.p,
                     (const uint64_t*)ctx->io1.p, n, (uint64_t*)ctx->io2.p, make_consts());
  PBF_HIP(hipGetLastError());
  PBF_HIP(hipMemcpyAsync(out, ctx->io2.p, n * 384, hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  return 0;
}

extern "C" int pbf_pairing_bn254_dev(pbf_ctx* ctx, const uint64_t* d_g1, const uint64_t* d_g2, size_t n,
                                     uint64_t* d_out, void* stream) {
  if (!ctx) return fail(1, "null context");
  if (n == 0) return 0;
  if (n > 0x7fffffffu) return fail(1, "batch too large");
  hipLaunchKernelGGL(pairing_kernel, dim3(n), dim3(64), 0, pbf_ctx::pick(stream), d_g1, d_g2, n, d_out,
                     make_consts());
  PBF_HIP(hipGetLastError());
  return 0;
}

// The pairing check on an explicit stream (host g1 / g2, synchronous): used by
// pbf_pairing_check_bn254 (context host stream) and Plonk::verify's `_dev` entry (its
// caller's stream).
int pbf::pairing_check_on_stream(pbf_ctx* ctx, const uint64_t* g1, const uint64_t* g2, size_t n, int* ok,
                                 hipStream_t s) {
  if (!ctx || !ok || (n && (!g1 || !g2))) return fail(1, "null argument");
  *ok = 0;
  if (n == 0) {
    *ok = 1;  // empty product
    return 0;
  }
  if (n > 0x7fffffffu) return fail(1, "batch too large");
  int rc = check_coords(g1, 2 * n);
  if (!rc) rc = check_coords(g2, 4 * n);
  if (rc) return rc;
  PBF_HIP(hipSetDevice(ctx->device));
  DevBuf &b1 = ctx->buf("pc.g1"), &b2 = ctx->buf("pc.g2"), &b3 = ctx->buf("pc.acc");
  if ((rc = b1.ensure(n * 64)) || (rc = b2.ensure(n * 128)) || (rc = b3.ensure(n * 384 + 64))) return rc;
  PBF_HIP(hipMemcpyAsync(b1.p, g1, n * 64, hipMemcpyHostToDevice, s));
  PBF_HIP(hipMemcpyAsync(b2.p, g2, n * 128, hipMemcpyHostToDevice, s));
  const PairingConsts k = make_consts();
  uint64_t* acc = (uint64_t*)b3.p;
  int* d_ok = (int*)(acc + 48 * n);
  hipLaunchKernelGGL(miller_kernel, dim3(n), dim3(64), 0, s, (const uint64_t*)b1.p, (const uint64_t*)b2.p, n, acc, k);
  PBF_HIP(hipGetLastError());
  hipLaunchKernelGGL(pairing_check_final, dim3(1), dim3(64), 0, s, (const uint64_t*)acc, n, d_ok, k);
  PBF_HIP(hipGetLastError());
  PBF_HIP(hipMemcpyAsync(ok, d_ok, sizeof(int), hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  return 0;
}

extern "C" int pbf_pairing_check_bn254(pbf_ctx* ctx, const uint64_t* g1, const uint64_t* g2, size_t n, int* ok) {
  if (!ctx) return fail(1, "null argument");
  return pairing_check_on_stream(ctx, g1, g2, n, ok, ctx->host_stream());
}

extern "C" int pbf_g2_bn254_mul(pbf_ctx* ctx, const uint64_t* pts, const uint64_t* scalars, size_t n,
                                uint64_t* out) {
  if (!ctx || (n && (!pts || !scalars || !out))) return fail(1, "null argument");
  if (n == 0) return 0;
  int rc = check_coords(pts, 4 * n);
  if (rc) return rc;
  hipStream_t s = ctx->host_stream();
  if ((rc = ctx->io0.ensure(n * 128)) || (rc = ctx->io1.ensure(n * 32)) || (rc = ctx->io2.ensure(n * 128))) return rc;
  PBF_HIP(hipMemcpyAsync(ctx->io0.p, pts, n * 128, hipMemcpyHostToDevice, s));
  PBF_HIP(hipMemcpyAsync(ctx->io1.p, scalars, n * 32, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(g2_mul_kernel, dim3((n + 63) / 64), dim3(64), 0, s, (const uint64_t*)ctx->io0.p,
                     (const uint64_t*)ctx->io1.p, n, (uint64_t*)ctx->io2.p, make_consts());
  PBF_HIP(hipGetLastError());
  PBF_HIP(hipMemcpyAsync(out, ctx->io2.p, n * 128, hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  return 0;
}
