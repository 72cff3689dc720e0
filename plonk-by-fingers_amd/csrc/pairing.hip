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
#include <cstring>
#include <mutex>
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

// a + b without the reduction (< 2q for canonical a, b): a Montgomery product accepts operands
// below 2q (their product is below q R, so the result stays below 2q before its subtraction)
__device__ __forceinline__ U256 u256_add_raw(const U256& a, const U256& b) {
  U256 r;
  unsigned c = 0;
#pragma unroll
  for (int l = 0; l < 8; ++l) r.w[l] = __builtin_addc(a.w[l], b.w[l], c, &c);
  return r;
}
// Montgomery inverse (aR)^-1 -> a^-1 R by Kaliski's almost-inverse (round 5; binary extended
// Euclid with one halving mod q per bit before, ~400 k cycles on one lane, now ~1/4 of that):
// u = q, v = aR, r = 0, s = 1 keep u s + v r = q; every step subtracts the smaller odd value
// from the larger, adds r and s, and strips the difference's trailing zeros at once (the
// other of r, s doubled as many times), counting them in k (254 <= k <= 508). It ends with
// x = q - r = (aR)^-1 2^k mod q, and one Montgomery product with 2^-k R^3 (g_inv2k, filled by
// the host from K_R3) gives a^-1 R. a != 0.
__device__ U256 g_inv2k[512];  // 2^-k R^3 mod q (plain), k < 512

__device__ __forceinline__ bool u256_zero_p(const U256& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.w[i];
  return o == 0;
}
__device__ __forceinline__ int u256_ctz(const U256& a) {  // a != 0
  uint32_t w = a.w[7];
  int base = 224;
#pragma unroll
  for (int l = 6; l >= 0; --l) {
    if (a.w[l] != 0) { w = a.w[l]; base = 32 * l; }
  }
  return base + __builtin_ctz(w);
}
__device__ __forceinline__ void u256_shr(U256& a, int t) {  // 0 <= t < 256
  while (t >= 32) {
#pragma unroll
    for (int l = 0; l < 7; ++l) a.w[l] = a.w[l + 1];
    a.w[7] = 0;
    t -= 32;
  }
  if (t) {
#pragma unroll
    for (int l = 0; l < 7; ++l) a.w[l] = __builtin_amdgcn_alignbit(a.w[l + 1], a.w[l], (uint32_t)t);
    a.w[7] >>= t;
  }
}
__device__ __forceinline__ void u256_shl(U256& a, int t) {  // no bits lost (a 2^t < 2^256)
  while (t >= 32) {
#pragma unroll
    for (int l = 7; l > 0; --l) a.w[l] = a.w[l - 1];
    a.w[0] = 0;
    t -= 32;
  }
  if (t) {
#pragma unroll
    for (int l = 7; l > 0; --l) a.w[l] = __builtin_amdgcn_alignbit(a.w[l], a.w[l - 1], (uint32_t)(32 - t));
    a.w[0] <<= t;
  }
}
// a - b mod 2^256; returns the borrow out
__device__ __forceinline__ unsigned u256_subb(U256& d, const U256& a, const U256& b) {
  unsigned c = 0;
#pragma unroll
  for (int l = 0; l < 8; ++l) d.w[l] = __builtin_subc(a.w[l], b.w[l], c, &c);
  return c;
}
__device__ __noinline__ U256 fq_inv(const U256& am, const PairingConsts&) {
  if (Fq::is_zero(am)) return u256_zero();  // no inverse (callers never pass 0)
  U256 u, v = am, r = u256_zero(), s = u256_zero(), d;
#pragma unroll
  for (int i = 0; i < 8; ++i) u.w[i] = Bn254FqParams::P[i];
  s.w[0] = 1;
  int k = u256_ctz(v);
  u256_shr(v, k);
  u256_shl(r, k);  // r = 0: a no-op, kept for the invariant's reading
  for (int guard = 0; guard < 1024; ++guard) {  // u, v odd here; <= 2 x 254 bits to strip
    if (u256_subb(d, u, v) == 0 && !u256_zero_p(d)) {  // u > v: u = (u - v) / 2^t, r += s, s <<= t
      const int t = u256_ctz(d);
      u256_shr(d, t);
      u = d;
      r = u256_add_raw(r, s);
      u256_shl(s, t);
      k += t;
    } else {  // v = (v - u) / 2^t, s += r, r <<= t
      u256_subb(d, v, u);
      s = u256_add_raw(s, r);
      if (u256_zero_p(d)) {  // u = v = 1: done
        u256_shl(r, 1);
        ++k;
        break;
      }
      const int t = u256_ctz(d);
      u256_shr(d, t);
      v = d;
      u256_shl(r, t);
      k += t;
    }
  }
  U256 q;
#pragma unroll
  for (int i = 0; i < 8; ++i) q.w[i] = Bn254FqParams::P[i];
  r = Fq::reduce_once(r);  // r < 2q
  u256_subb(d, q, r);      // x = q - r
  return Fq::mul(d, g_inv2k[k & 511]);
}
__device__ __forceinline__ Fq2 f2_inv(const Fq2& a, const PairingConsts& k) {
  const U256 ni = fq_inv(Fq::add(Fq::mul(a.c0, a.c0), Fq::mul(a.c1, a.c1)), k);
  return {Fq::mul(a.c0, ni), Fq::sub(u256_zero(), Fq::mul(a.c1, ni))};
}

// ---------------------------------------------------------------- lane-parallel Fq12 engine
// A pairing product runs in one workgroup of PT threads (four waves on four SIMDs). Fq12
// values live in LDS in the flat w-basis (g[k] = coefficient of w^k, an Fq2); a register
// holds g[0..5] and, in slots 6..11, xi g[0..5]. On gfx950 a lone wave's Fq product costs
// ~2250 cycles (136 v_mad_u64_u32 at ~16 cycles each, scripts/ubench/pairing_lat.hip) whatever
// the lanes hold, so the engine puts ONE Fq product on each lane per round: an Fq12 product is
//   round 1  the 108 Fq products of 36 Karatsuba Fq2 products x_i y_j, one per lane; where
//            i + j >= 6 (w^6 = xi) the lane takes xi x_i from the register's second half, so
//            no product is multiplied by xi afterwards;
//   round 2  18 lanes (k, c) sum the Karatsuba parts t_c of the six products of output
//            coefficient k, S_c, in 288-bit accumulators without reductions;
//   round 3  lane k of wave (h, c) forms component c of g_k (h = 0) or of xi g_k (h = 1) as a
//            small integer combination of S_0, S_1, S_2 and reduces it once,
// where the form before round 5 (Karatsuba recombination and a product by xi per Fq2
// product, then sums of reduced Fq2) paid ~10 reduced Fq additions in sequence (round 2 +
// round 3: 4.2 k cycles; now ~2.4-3.2 k, scripts/ubench/r2lat.hip). A sparse line (w^0, w^1,
// w^3) is the same with 18 pairs.
// Every function is called by all PT threads and ends with a barrier; operands are LDS
// Fq12 registers (12 Fq2) and may alias the result.
constexpr int PT = 256;

// Lazy sums: 9 x 32-bit limbs (< 2^288) through __builtin_addc / __builtin_subc carry chains
// (v_add_co / v_addc with SGPR-pair carries; the compiler interleaves independent chains and
// places the carry wait states).
struct L9 {
  uint32_t w[9];
};
__device__ __forceinline__ L9 l9_of(const U256& x) {
  L9 r;
#pragma unroll
  for (int l = 0; l < 8; ++l) r.w[l] = x.w[l];
  r.w[8] = 0;
  return r;
}
__device__ __forceinline__ void l9_add(L9& a, const U256& x) {
  unsigned c = 0;
#pragma unroll
  for (int l = 0; l < 8; ++l) a.w[l] = __builtin_addc(a.w[l], x.w[l], c, &c);
  a.w[8] += c;
}
__device__ __forceinline__ void l9_add(L9& a, const L9& b) {
  unsigned c = 0;
#pragma unroll
  for (int l = 0; l < 9; ++l) a.w[l] = __builtin_addc(a.w[l], b.w[l], c, &c);
}
__device__ __forceinline__ void l9_sub(L9& a, const L9& b) {  // requires a >= b
  unsigned c = 0;
#pragma unroll
  for (int l = 0; l < 9; ++l) a.w[l] = __builtin_subc(a.w[l], b.w[l], c, &c);
}
template <int S>
__device__ __forceinline__ L9 l9_shl(const L9& a) {  // a << S (no overflow for our bounds)
  L9 r;
  r.w[0] = a.w[0] << S;
#pragma unroll
  for (int l = 1; l < 9; ++l) r.w[l] = (a.w[l] << S) | (a.w[l - 1] >> (32 - S));
  return r;
}
// K q in 9 limbs, compile time
struct L9c {
  uint32_t w[9];
};
constexpr L9c l9_kq(uint32_t K) {
  L9c r{};
  uint64_t c = 0;
  for (int l = 0; l < 8; ++l) {
    const uint64_t p = (uint64_t)K * Bn254FqParams::P[l] + c;
    r.w[l] = (uint32_t)p;
    c = p >> 32;
  }
  r.w[8] = (uint32_t)c;
  return r;
}
template <uint32_t K>
__device__ __forceinline__ void l9_add_kq(L9& a) {
  constexpr L9c k = l9_kq(K);
  unsigned c = 0;
#pragma unroll
  for (int l = 0; l < 9; ++l) a.w[l] = __builtin_addc(a.w[l], k.w[l], c, &c);
}
// x mod q for x < 2^262 (x < 340 q): d = floor(x / q) estimated from x's top 96 bits in double
// (relative error < 2^-50, so x / q - est < 1e-12 for x < 340 q) minus a 1e-9 margin, so that
// d is floor(x / q) or one less: x - d q < 2q, one conditional subtraction.
__device__ __forceinline__ U256 l9_reduce(L9 x) {
  const double top = ((double)x.w[8] * 18446744073709551616.0 + (double)x.w[7] * 4294967296.0) + (double)x.w[6];
  const double est = top * (1.0 / 3486998266802970666.0) - 1e-9;  // q / 2^192 = 0x30644e72e131a029.b8...
  const uint32_t d = est > 0.0 ? (uint32_t)est : 0u;
  L9 m;
  uint64_t c = 0;
#pragma unroll
  for (int l = 0; l < 8; ++l) {
    const uint64_t p = (uint64_t)d * Bn254FqParams::P[l] + c;
    m.w[l] = (uint32_t)p;
    c = p >> 32;
  }
  m.w[8] = (uint32_t)c;
  l9_sub(x, m);
  U256 r;
#pragma unroll
  for (int l = 0; l < 8; ++l) r.w[l] = x.w[l];  // < 2q < 2^255: limb 8 is 0
  return Fq::reduce_once(r);
}
// 16-byte LDS accesses (ds_read_b128 / ds_write_b128: PL is 16-byte aligned and every member
// a multiple of 16 bytes; U256's own alignment is 4, so the compiler would split them)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ U256 ld16_u256(const U256* p) {
  const u32x4* v = (const u32x4*)__builtin_assume_aligned(p, 16);
  const u32x4 a = v[0], b = v[1];
  return U256{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
}
__device__ __forceinline__ void st16_u256(U256* p, const U256& x) {
  u32x4* v = (u32x4*)__builtin_assume_aligned(p, 16);
  v[0] = u32x4{x.w[0], x.w[1], x.w[2], x.w[3]};
  v[1] = u32x4{x.w[4], x.w[5], x.w[6], x.w[7]};
}
__device__ __forceinline__ Fq2 ld16_fq2(const Fq2* p) { return Fq2{ld16_u256(&p->c0), ld16_u256(&p->c1)}; }
struct alignas(16) L9s {  // an L9 in LDS, padded to 48 bytes
  uint32_t w[12];
};
__device__ __forceinline__ void st16_l9(L9s* p, const L9& x) {
  u32x4* v = (u32x4*)p;
  v[0] = u32x4{x.w[0], x.w[1], x.w[2], x.w[3]};
  v[1] = u32x4{x.w[4], x.w[5], x.w[6], x.w[7]};
  v[2] = u32x4{x.w[8], 0u, 0u, 0u};
}
__device__ __forceinline__ L9 ld16_l9(const L9s* p) {
  const u32x4* v = (const u32x4*)p;
  const u32x4 a = v[0], b = v[1], c = v[2];
  return L9{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x}};
}
__device__ __forceinline__ U256 kara_raw(const Fq2& a, int r) {
  return u256_add_raw(r == 1 ? a.c1 : a.c0, r == 2 ? a.c1 : u256_zero());
}

// Miller-step slots: T = (X : Y : Z), the affine point added (xq, yq), the line's w^3
// coefficient, temporaries from SL_T
enum { SL_X, SL_Y, SL_Z, SL_XQ, SL_YQ, SL_L3, SL_T };
constexpr int SL_N = SL_T + 20;

// the Miller schedule of 6u+2 = 2^64 + K_ATE_LO: a doubling per bit below the top one, an
// addition of Q after it where the bit is set, then T + pi(Q) and T - pi^2(Q)
constexpr int ATE_ADDS = __builtin_popcountll(K_ATE_LO);
constexpr int NSTEP = 64 + ATE_ADDS + 2;
enum : uint8_t { ST_DBL, ST_ADD_Q, ST_ADD_PI, ST_ADD_PI2 };
struct StepTable {
  uint8_t kind[NSTEP];
};
constexpr StepTable make_steps() {
  StepTable t{};
  int n = 0;
  for (int b = 63; b >= 0; --b) {
    t.kind[n++] = ST_DBL;
    if ((K_ATE_LO >> b) & 1) t.kind[n++] = ST_ADD_Q;
  }
  t.kind[n++] = ST_ADD_PI;
  t.kind[n++] = ST_ADD_PI2;
  return t;
}
__constant__ StepTable c_steps = make_steps();
static_assert(make_steps().kind[NSTEP - 1] == ST_ADD_PI2, "step count");

// A prepared line: l(P) = a yp + (b xp) w + c w^3, Fq2 each (Montgomery); the identity Q
// is flagged separately and contributes 1.
struct PrepLine {
  Fq2 a, b, c;
};

constexpr int LCHUNK = 2;  // pairs whose evaluated lines sit in LDS at once
constexpr int NREG = 32;   // Fq12 registers (the final exponentiation's program names them)
constexpr int LB = PT / 27;  // steps per batch of pair_line_products
struct alignas(16) PL {
  U256 t[PT];          // round-1 Fq products
  L9s acc[2][6][3];    // round-2 sums (two products: w_mul_dual)
  Fq2 pp[9 * LB];      // Fq2 products of pair_line_products
  Fq2 reg[NREG][12];   // Fq12 registers: g[0..5], xi g[0..5]
  Fq2 sl[SL_N];        // Miller-step slots
  Fq2 Qa[3][2];        // Q, pi(Q), -pi^2(Q) affine
  Fq2 frob1[12];       // lane-indexed constants: FROB1[k], xi FROB1[k] (a lane-indexed kernel
  U256 frob2[6];       // argument would be copied to scratch)
  U256 px[LCHUNK], py[LCHUNK];
  // per step: the lines evaluated at P, pair p's (w^0, w^1, w^3) at [3p .. 3p + 2]; for two pairs
  // then their product as a register: w^0..w^4 at [0..4], 0 at [5], xi times them at [6..11]
  Fq2 le[NSTEP][12];
  int skip[LCHUNK];
};

__device__ __forceinline__ void load_consts(const PairingConsts& k, PL& L, int tid) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    if (tid == i) {
      const Fq2 f{k.frob1[i][0], k.frob1[i][1]};
      L.frob1[i] = f;
      L.frob1[6 + i] = f2_mul_xi(f);
      L.frob2[i] = k.frob2[i];
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void bsync() { __syncthreads(); }

// Operand of a Karatsuba product: role 0 -> a.c0, 1 -> a.c1, 2 -> a.c0 + a.c1 (one uniform
// addition for every lane, no divergence)
__device__ __forceinline__ U256 kara_operand(const Fq2& a, int r) {
  return Fq::add(r == 1 ? a.c1 : a.c0, r == 2 ? a.c1 : u256_zero());
}
__device__ __forceinline__ Fq2 kara_combine(const U256& t0, const U256& t1, const U256& t2) {
  return Fq2{Fq::sub(t0, t1), Fq::sub(t2, Fq::add(t0, t1))};
}
__device__ __forceinline__ int line_j(int jj) { return jj == 2 ? 3 : jj; }

// y's nonzero coefficients: W_DENSE all six; W_LINE w^0, w^1, w^3 (as y[0], y[1], y[2]);
// W_FIVE w^0..w^4 (the product of two lines)
enum { W_DENSE, W_LINE, W_FIVE };
template <int MODE>
struct WShape {
  static constexpr int NJ = MODE == W_DENSE ? 6 : (MODE == W_LINE ? 3 : 5);
  __device__ __forceinline__ static int j(int jj) { return MODE == W_LINE ? line_j(jj) : jj; }
};

// dst = x * y (x a register: its xi half feeds the wrapped products; y: NJ coefficients).
// Karatsuba parts of x_i y_j: t0 = x0 y0, t1 = x1 y1, t2 = (x0 + x1)(y0 + y1), the product
// (t0 - t1) + (t2 - t0 - t1) u and xi times it (10 t0 - 8 t1 - t2) + (9 t2 - 8 t0 - 10 t1) u.
// Sums of at most six canonical t are < 6q, so the offsets 6q, 12q, 54q, 108q keep every
// combination non-negative and below 162 q. The three rounds are split out so that two
// independent products can share them (w_mul_dual).
//
// round 1 on `lane` < 3 NP: t[lane]; NEGY: y's odd coefficients negated (x conj(y)): the
// product of a pair with odd j changes sign, so each of its three parts does
template <int MODE, bool NEGY>
__device__ __forceinline__ void wm_r1(const Fq2* x, const Fq2* y, U256* t, int lane) {
  using Sh = WShape<MODE>;
  constexpr int NJ = Sh::NJ, NP = 6 * NJ;
  if (lane < 3 * NP) {
    const int q = lane / 3, r = lane - 3 * q, i = q / NJ, jj = q - NJ * i, j = Sh::j(jj);
    const Fq2 xa = ld16_fq2(x + i + (i + j >= 6 ? 6 : 0)), ya = ld16_fq2(y + jj);
    U256 v = Fq::mul(kara_raw(xa, r), kara_raw(ya, r));
    if (NEGY && (j & 1)) v = Fq::sub(u256_zero(), v);
    st16_u256(t + lane, v);
  }
}
// round 2 on `lane` < 18: S_c of output k, lane (k, c)
template <int MODE>
__device__ __forceinline__ void wm_r2(const U256* t, L9s (*acc)[3], int lane) {
  using Sh = WShape<MODE>;
  constexpr int NJ = Sh::NJ;
  if (lane < 18) {
    const int k = lane / 3, c = lane - 3 * k;
    L9 s;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      const int j = Sh::j(jj);
      const int i = k - j < 0 ? k - j + 6 : k - j;
      const U256 v = ld16_u256(t + 3 * (i * NJ + jj) + c);
      if (jj == 0) s = l9_of(v);
      else l9_add(s, v);
    }
    st16_l9(&acc[k][c], s);
  }
}
// round 3 for output k < 6 in wave wv = (h, c): component c of g_k (h = 0) or of xi g_k (h = 1)
__device__ __forceinline__ void wm_r3(Fq2* dst, L9s (*acc)[3], int wv, int k) {
  L9 s[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) s[c] = ld16_l9(&acc[k][c]);
  L9 v;
  if (wv == 0) {  // t0 - t1
    v = s[0];
    l9_add_kq<6>(v);
    l9_sub(v, s[1]);
  } else if (wv == 1) {  // t2 - t0 - t1
    v = s[2];
    l9_add_kq<12>(v);
    l9_sub(v, s[0]);
    l9_sub(v, s[1]);
  } else if (wv == 2) {  // 10 t0 - 8 t1 - t2
    L9 f = l9_shl<2>(s[0]);
    l9_add(f, s[0]);
    v = l9_shl<1>(f);
    l9_add_kq<54>(v);
    l9_sub(v, l9_shl<3>(s[1]));
    l9_sub(v, s[2]);
  } else {  // 9 t2 - 8 t0 - 10 t1
    v = l9_shl<3>(s[2]);
    l9_add(v, s[2]);
    l9_add_kq<108>(v);
    L9 u = s[0];
    l9_add(u, s[1]);
    l9_sub(v, l9_shl<3>(u));
    l9_sub(v, l9_shl<1>(s[1]));
  }
  const U256 r = l9_reduce(v);
  Fq2* d = dst + k + (wv >> 1) * 6;
  st16_u256((wv & 1) ? &d->c1 : &d->c0, r);
}
template <int MODE>
__device__ __forceinline__ void w_mul(Fq2* dst, const Fq2* x, const Fq2* y, PL& L, int tid) {
  wm_r1<MODE, false>(x, y, L.t, tid);
  bsync();
  wm_r2<MODE>(L.t, L.acc[0], tid);
  bsync();
  const int wv = tid >> 6, k = tid & 63;
  if (k < 6) wm_r3(dst, L.acc[0], wv, k);
  bsync();
}
// Two independent dense products in the same three rounds (216 of the 256 lanes in round 1):
// dA = xA yA and dB = xB yB (NEGB: xB conj(yB)). Either destination may alias any operand:
// round 1 reads every operand before round 3 writes.
template <bool NEGB>
__device__ __forceinline__ void w_mul_dual(Fq2* dA, const Fq2* xA, const Fq2* yA, Fq2* dB, const Fq2* xB, const Fq2* yB,
                                           PL& L, int tid) {
  if (tid < 128) wm_r1<W_DENSE, false>(xA, yA, L.t, tid);
  else wm_r1<W_DENSE, NEGB>(xB, yB, L.t + 128, tid - 128);
  bsync();
  const int wv = tid >> 6, k = tid & 63;
  if (wv == 0) wm_r2<W_DENSE>(L.t, L.acc[0], k);
  else if (wv == 1) wm_r2<W_DENSE>(L.t + 128, L.acc[1], k);
  bsync();
  if ((k & 31) < 6) {  // lanes 0..5: product A, 32..37: product B (one code path)
    const bool b = k >= 32;
    wm_r3(b ? dB : dA, L.acc[b ? 1 : 0], wv, k & 31);
  }
  bsync();
}

// the xi half of a register from its first half (after a value was written by one lane)
__device__ __forceinline__ void w_fill_xi(Fq2* d, int tid) {
  if (tid < 6) d[6 + tid] = f2_mul_xi(d[tid]);
  bsync();
}
__device__ __forceinline__ void w_copy(Fq2* dst, const Fq2* x, int tid) {
  if (tid < 12) dst[tid] = x[tid];
  bsync();
}
// x^(q^6): w -> -w (the xi half likewise)
__device__ __forceinline__ void w_conj(Fq2* dst, const Fq2* x, int tid) {
  if (tid < 12) dst[tid] = (tid & 1) ? f2_neg(x[tid]) : x[tid];
  bsync();
}
// x^q: g_k -> conj(g_k) FROB1[k], and xi times it = conj(g_k) (xi FROB1[k]); lane (h, k, role)
// computes one Karatsuba product
__device__ __forceinline__ void w_frob1(Fq2* dst, const Fq2* x, PL& L, int tid) {
  if (tid < 36) {
    const int q = tid / 3, r = tid - 3 * q, k = q % 6;
    L.t[tid] = Fq::mul(kara_operand(f2_conj(x[k]), r), kara_operand(L.frob1[q], r));
  }
  bsync();
  if (tid < 12) dst[tid] = kara_combine(L.t[3 * tid], L.t[3 * tid + 1], L.t[3 * tid + 2]);
  bsync();
}
// x^(q^2): g_k -> g_k FROB2[k] (FROB2 in Fq, so the xi half scales the same way)
__device__ __forceinline__ void w_frob2(Fq2* dst, const Fq2* x, PL& L, int tid) {
  if (tid < 24) {
    const int e = tid >> 1;
    const U256 v = Fq::mul((tid & 1) ? x[e].c1 : x[e].c0, L.frob2[e % 6]);
    if (tid & 1) dst[e].c1 = v; else dst[e].c0 = v;
  }
  bsync();
}
__device__ __forceinline__ void w_one(Fq2* dst, const PairingConsts& k, int tid) {
  if (tid < 12) dst[tid] = Fq2{tid == 0 ? k.one : u256_zero(), u256_zero()};
  bsync();
  if (tid == 0) dst[6] = f2_mul_xi(dst[0]);
  bsync();
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
// interpreter loop: one inlined copy of each primitive and no calls (a call would save and
// restore the callee's VGPRs through scratch every time). FE_DUAL runs two independent
// products in one set of rounds (w_mul_dual): the program pairs them wherever the chain allows.
enum : uint8_t { FE_MUL, FE_DUAL, FE_CONJ, FE_FROB1, FE_FROB2, FE_COPY, FE_INVN, FE_CSQR };
struct FeOp {
  uint8_t op, dst, a, b;      // FE_MUL / FE_DUAL product A: dst = a b
  uint8_t dst2, a2, b2, neg;  // FE_DUAL product B: dst2 = a2 b2 (neg: a2 conj(b2))
};
constexpr int FE_MAX = 320;
struct FeProg {
  FeOp ops[FE_MAX];
  int n, products;  // ops; product rounds (FE_MUL + FE_DUAL)
};
struct FeMul {  // a product waiting for a slot
  int d, a, b;
};
// Registers (all distinct, so that products of independent chains can share rounds):
enum : int {
  R_F, R_A, R_B, R_C, R_S,                     // f, a = f^u, b = a^u, c = b^u, a power's running square
  R_E1, R_E2, R_E3, R_E4,                      // easy part
  R_A2, R_A4, R_A6, R_A12, R_A18,              // a^2 .. a^18
  R_B2, R_B4, R_B6, R_B12, R_B18, R_B24, R_B30,  // b^2 .. b^30
  R_C2, R_C4, R_C36, R_F2, R_L2, R_X5, R_X4, R_T7, R_FQ1, R_FQ3, R_Y, R_COUNT
};
static_assert(R_COUNT <= NREG, "register file");
constexpr FeProg make_fe_prog() {
  FeProg p{};
  int n = 0, np = 0;
  auto op = [&](uint8_t o, int d, int a, int b) {
    p.ops[n++] = FeOp{o, (uint8_t)d, (uint8_t)a, (uint8_t)b, 0, 0, 0, 0};
  };
  auto mul = [&](int d, int a, int b) { op(FE_MUL, d, a, b); ++np; };
  auto dual = [&](int d, int a, int b, int d2, int a2, int b2, bool neg) {
    p.ops[n++] = FeOp{FE_DUAL, (uint8_t)d, (uint8_t)a, (uint8_t)b, (uint8_t)d2, (uint8_t)a2, (uint8_t)b2, (uint8_t)neg};
    ++np;
  };
  // d = x^u, right to left over the NAF of u (x^-1 = conj x in the cyclotomic subgroup): the
  // running square S and the product d read the same S in each round, so the squaring and the
  // multiplication share it; rounds without a multiplication take the next of `side` (a
  // dependent chain of products on values ready before this power starts), in order.
  auto powu = [&](int d, int x, const FeMul* side, int ns) {
    int8_t naf[66] = {};
    int len = 0;
    for (uint64_t e = K_BN_U; e; e >>= 1) {
      int8_t z = 0;
      if (e & 1) {
        z = (int8_t)(2 - (int)(e & 3));
        e = z > 0 ? e - 1 : e + 1;
      }
      naf[len++] = z;
    }
    int si = 0;
    bool have = false;
    op(FE_COPY, R_S, x, 0);
    for (int i = 0; i < len; ++i) {
      const int z = naf[i];
      if (i == len - 1) {  // the top digit (+1): d = d S
        if (si < ns) {
          dual(d, d, R_S, side[si].d, side[si].a, side[si].b, false);
          ++si;
        } else {
          mul(d, d, R_S);
        }
        break;
      }
      const bool m = z != 0 && have;
      if (z != 0 && !have) {  // the lowest digit: d = S^z, no product
        op(z > 0 ? FE_COPY : FE_CONJ, d, R_S, 0);
        have = true;
      }
      if (m) {
        dual(R_S, R_S, R_S, d, d, R_S, z < 0);
      } else if (si < ns) {
        dual(R_S, R_S, R_S, side[si].d, side[si].a, side[si].b, false);
        ++si;
      } else {
        mul(R_S, R_S, R_S);
      }
    }
    for (; si < ns; ++si) mul(side[si].d, side[si].a, side[si].b);  // (never: enough free rounds)
  };
  // easy part: f^(q^6-1) = conj(f)^2 / (f conj(f)), then ^(q^2+1)
  op(FE_CONJ, R_E1, R_F, 0);
  dual(R_E2, R_F, R_E1, R_E3, R_E1, R_E1, false);  // N = f conj(f) (in Fq6); conj(f)^2
  op(FE_INVN, R_E2, 0, 0);
  mul(R_F, R_E3, R_E2);    // f^(q^6-1)
  op(FE_FROB2, R_E4, R_F, 0);
  mul(R_F, R_E4, R_F);     // f^((q^6-1)(q^2+1)): the hard part's base, in the cyclotomic subgroup
  // hard part: f^(l0 + l1 q + l2 q^2 + q^3) (see file header)
  op(FE_FROB1, R_FQ1, R_F, 0);
  op(FE_FROB2, R_FQ3, R_FQ1, 0);  // f^(q^3)
  const FeMul s1[] = {{R_F2, R_F, R_F}};
  powu(R_A, R_F, s1, 1);
  const FeMul s2[] = {{R_A2, R_A, R_A}, {R_A4, R_A2, R_A2}, {R_A6, R_A4, R_A2}, {R_A12, R_A6, R_A6}, {R_A18, R_A12, R_A6}};
  powu(R_B, R_A, s2, 5);
  const FeMul s3[] = {{R_B2, R_B, R_B},     {R_B4, R_B2, R_B2},    {R_B6, R_B4, R_B2},    {R_B12, R_B6, R_B6},
                      {R_B18, R_B12, R_B6}, {R_B24, R_B12, R_B12}, {R_B30, R_B24, R_B6}, {R_L2, R_B6, R_F}};
  powu(R_C, R_B, s3, 8);
  // c^36 = c^32 c^4, beside it Y = frob2(f^l2) f^(q^3)
  op(FE_FROB2, R_T7, R_L2, 0);
  dual(R_C2, R_C, R_C, R_Y, R_T7, R_FQ3, false);
  mul(R_C4, R_C2, R_C2);
  mul(R_C2, R_C4, R_C4);  // c^8
  mul(R_C2, R_C2, R_C2);  // c^16
  mul(R_C2, R_C2, R_C2);  // c^32
  mul(R_C36, R_C2, R_C4);
  // f^l1 = conj(c^36 b^18 a^12) f, f^l0 = conj(c^36 b^30 a^18 f^2)
  dual(R_X5, R_C36, R_B18, R_X4, R_C36, R_B30, false);
  dual(R_X5, R_X5, R_A12, R_X4, R_X4, R_A18, false);
  op(FE_CONJ, R_X5, R_X5, 0);
  dual(R_X5, R_X5, R_F, R_X4, R_X4, R_F2, false);
  op(FE_CONJ, R_X4, R_X4, 0);
  op(FE_FROB1, R_T7, R_X5, 0);
  mul(R_X4, R_X4, R_T7);  // f^l0 frob1(f^l1)
  mul(R_F, R_X4, R_Y);    // times frob2(f^l2) f^(q^3)
  p.n = n;
  p.products = np;
  return p;
}
__constant__ FeProg c_fe_prog = make_fe_prog();
static_assert(make_fe_prog().n <= FE_MAX, "program size");

// The lane engine's program: the same chain as one product per step, left to right over the
// NAF of u, squarings in the hard part marked FE_CSQR (Granger-Scott per lane: 21 Fq products
// instead of 36), 16 registers (the lane engine keeps them in scratch): 0 f (in/out),
// 1 a = f^u, 2 b = f^u^2, 3 c = f^u^3, 4..11 temporaries, 12, 13 inverse, 14 conj of the base
// of a power by u
constexpr FeProg make_fe_seq() {
  FeProg p{};
  int n = 0, np = 0;
  auto op = [&](uint8_t o, int d, int a, int b) {
    p.ops[n++] = FeOp{o, (uint8_t)d, (uint8_t)a, (uint8_t)b, 0, 0, 0, 0};
    if (o == FE_MUL || o == FE_CSQR) ++np;
  };
  auto mul = [&](int d, int a, int b) { op(FE_MUL, d, a, b); };
  auto sqr = [&](int d, int a) { op(FE_CSQR, d, a, 0); };
  auto powu = [&](int d, int x) {
    int8_t naf[66] = {};
    int len = 0;
    for (uint64_t e = K_BN_U; e; e >>= 1) {
      int8_t z = 0;
      if (e & 1) {
        z = (int8_t)(2 - (int)(e & 3));
        e = z > 0 ? e - 1 : e + 1;
      }
      naf[len++] = z;
    }
    op(FE_CONJ, 14, x, 0);
    op(FE_COPY, d, x, 0);  // the top digit is +1
    for (int i = len - 2; i >= 0; --i) {
      sqr(d, d);
      if (naf[i] == 1) mul(d, d, x);
      if (naf[i] == -1) mul(d, d, 14);
    }
  };
  op(FE_CONJ, 12, 0, 0);
  mul(13, 0, 12);
  op(FE_INVN, 13, 0, 0);
  mul(4, 12, 13);          // f^-1
  mul(0, 12, 4);           // conj(f) f^-1
  op(FE_FROB2, 4, 0, 0);
  mul(0, 4, 0);
  powu(1, 0);
  powu(2, 1);
  powu(3, 2);
  sqr(7, 3); sqr(7, 7);                         // c^4
  sqr(4, 7); sqr(4, 4); sqr(4, 4);              // c^32
  mul(4, 4, 7);                                 // c^36
  sqr(7, 2); sqr(10, 7); mul(10, 10, 7);        // b^2, b^4, b^6
  sqr(8, 10); mul(9, 8, 10);                    // b^12, b^18
  sqr(8, 8); mul(8, 8, 10);                     // b^24, b^30
  sqr(7, 1); sqr(11, 7); mul(11, 11, 7);        // a^2, a^4, a^6
  sqr(7, 11); mul(11, 7, 11);                   // a^12, a^18
  mul(5, 4, 9); mul(5, 5, 7); op(FE_CONJ, 5, 5, 0); mul(5, 5, 0);  // f^l1
  mul(6, 10, 0);                                                  // f^l2
  mul(4, 4, 8); mul(4, 4, 11); sqr(7, 0); mul(4, 4, 7); op(FE_CONJ, 4, 4, 0);  // f^l0
  op(FE_FROB1, 7, 5, 0); mul(4, 4, 7);
  op(FE_FROB2, 7, 6, 0); mul(4, 4, 7);
  op(FE_FROB1, 7, 0, 0); op(FE_FROB2, 8, 7, 0); mul(0, 4, 8);
  p.n = n;
  p.products = np;
  return p;
}
constexpr int FE_SEQ_REGS = 16;
__constant__ FeProg c_fe_seq = make_fe_seq();
static_assert(make_fe_seq().n <= FE_MAX, "program size");

// result = f^((q^12-1)/r), f in L.reg[0]; result in L.reg[0]
__device__ __forceinline__ void final_exp_w(const PairingConsts& k, PL& L, int tid) {
  const int n = c_fe_prog.n;
  for (int pc = 0; pc < n; ++pc) {
    const FeOp o = c_fe_prog.ops[pc];
    Fq2* d = L.reg[o.dst];
    const Fq2* a = L.reg[o.a];
    switch (o.op) {
      case FE_MUL: w_mul<W_DENSE>(d, a, L.reg[o.b], L, tid); break;
      case FE_DUAL:
        if (o.neg) w_mul_dual<true>(d, a, L.reg[o.b], L.reg[o.dst2], L.reg[o.a2], L.reg[o.b2], L, tid);
        else w_mul_dual<false>(d, a, L.reg[o.b], L.reg[o.dst2], L.reg[o.a2], L.reg[o.b2], L, tid);
        break;
      case FE_CONJ: w_conj(d, a, tid); break;
      case FE_FROB1: w_frob1(d, a, L, tid); break;
      case FE_FROB2: w_frob2(d, a, L, tid); break;
      case FE_COPY: w_copy(d, a, tid); break;
      default:  // FE_INVN
        if (tid == 0) fq6_inv_flat(d, k);
        bsync();
        w_fill_xi(d, tid);
        break;
    }
  }
}

// ---------------------------------------------------------------- prepared lines of Q
// T = (X : Y : Z) homogeneous on the twist. Doubling: w = 3X^2, s = 2YZ, R = Ys,
//   B = (X+R)^2 - X^2 - R^2, h = w^2 - 2B, X3 = h s, Y3 = w (B - h) - 2 R^2, Z3 = s^3;
//   line * s Z: (s Z) yp - (w Z) xp w + (w X - R) v w   (v w = w^3)
// Mixed addition T += (xq, yq): N = yq Z - Y, D = xq Z - X,
//   A = N^2 Z - D^3 - 2 D^2 X, X3 = D A, Y3 = N (D^2 X - A) - D^3 Y, Z3 = D^3 Z;
//   line * D: D yp - N xp w + (N xq - D yq) v w
// (The line scalings s Z and D are Fq2 factors, removed by the final exponentiation.)
// The steps are micro-op programs over the slot file: a MULS group is up to 6 independent
// Fq2 products (18 Fq products, one per lane, then 6 lanes recombine), a LIN group a short
// run of additions on lane 0, STORE writes the step's (a, b, c).
enum : uint8_t { U_MULS, U_LIN, U_STORE, L_ADD, L_SUB, L_DBL, L_TRP, L_NEG, L_COPY, U_MUL };
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
    GRP(U_MULS, 3), MUL(T0 + 11, T0 + 3, T0 + 4), MUL(T0 + 12, T0 + 5, T0 + 5),      // s^3, R^2
    MUL(T0 + 13, T0 + 10, T0 + 10),                                                  // (X+R)^2
    GRP(U_LIN, 9), LIN(L_NEG, T0 + 14, T0 + 7, 0), LIN(L_SUB, SL_L3, T0 + 8, T0 + 5),
    LIN(L_SUB, T0 + 15, T0 + 13, T0 + 0), LIN(L_SUB, T0 + 15, T0 + 15, T0 + 12),     // B
    LIN(L_DBL, T0 + 16, T0 + 15, 0), LIN(L_SUB, T0 + 16, T0 + 9, T0 + 16),           // h
    LIN(L_SUB, T0 + 17, T0 + 15, T0 + 16), LIN(L_DBL, T0 + 18, T0 + 12, 0),          // B - h, 2R^2
    LIN(L_COPY, SL_Z, T0 + 11, 0),                                                    // Z3
    GRP(U_STORE, 0), Uop{U_STORE, T0 + 6, T0 + 14, SL_L3},                            // (sZ, -wZ, L3)
    GRP(U_MULS, 2), MUL(SL_X, T0 + 16, T0 + 3), MUL(T0 + 19, T0 + 2, T0 + 17),         // X3, w(B-h)
    GRP(U_LIN, 1), LIN(L_SUB, SL_Y, T0 + 19, T0 + 18)};                               // Y3
__constant__ Uop c_add_prog[] = {
    GRP(U_MULS, 2), MUL(T0 + 0, SL_YQ, SL_Z), MUL(T0 + 1, SL_XQ, SL_Z),
    GRP(U_LIN, 2), LIN(L_SUB, T0 + 2, T0 + 0, SL_Y), LIN(L_SUB, T0 + 3, T0 + 1, SL_X),  // N, D
    GRP(U_MULS, 4), MUL(T0 + 4, T0 + 2, T0 + 2), MUL(T0 + 5, T0 + 3, T0 + 3),         // N^2, D^2
    MUL(T0 + 6, T0 + 2, SL_XQ), MUL(T0 + 7, T0 + 3, SL_YQ),                           // N xq, D yq
    GRP(U_LIN, 2), LIN(L_NEG, T0 + 8, T0 + 2, 0), LIN(L_SUB, SL_L3, T0 + 6, T0 + 7),
    GRP(U_STORE, 0), Uop{U_STORE, T0 + 3, T0 + 8, SL_L3},                             // (D, -N, L3)
    GRP(U_MULS, 3), MUL(T0 + 9, T0 + 3, T0 + 5), MUL(T0 + 10, T0 + 5, SL_X),          // D^3, D^2 X
    MUL(T0 + 11, T0 + 4, SL_Z),                                                       // N^2 Z
    GRP(U_LIN, 4), LIN(L_SUB, T0 + 12, T0 + 11, T0 + 9), LIN(L_DBL, T0 + 13, T0 + 10, 0),
    LIN(L_SUB, T0 + 12, T0 + 12, T0 + 13), LIN(L_SUB, T0 + 14, T0 + 10, T0 + 12),    // A, D^2X - A
    GRP(U_MULS, 4), MUL(T0 + 15, T0 + 3, T0 + 12), MUL(T0 + 16, T0 + 9, SL_Z),
    MUL(T0 + 17, T0 + 2, T0 + 14), MUL(T0 + 18, T0 + 9, SL_Y),
    GRP(U_LIN, 3), LIN(L_COPY, SL_X, T0 + 15, 0), LIN(L_COPY, SL_Z, T0 + 16, 0),
    LIN(L_SUB, SL_Y, T0 + 17, T0 + 18)};
#undef MUL
#undef LIN
#undef GRP
constexpr int DBL_LEN = sizeof(c_dbl_prog) / sizeof(Uop), ADD_LEN = sizeof(c_add_prog) / sizeof(Uop);
static_assert(T0 + 20 <= SL_N, "slot file");

__device__ __forceinline__ void run_uops(const Uop* prog, int len, PrepLine* out, PL& L, int tid) {
  Fq2* sl = L.sl;
  for (int pc = 0; pc < len;) {
    const Uop u = prog[pc];
    if (u.code == U_MULS) {
      if (tid < 3 * u.d) {
        const int m = tid / 3, r = tid - 3 * m;
        const Uop o = prog[pc + 1 + m];
        L.t[tid] = Fq::mul(kara_operand(sl[o.a], r), kara_operand(sl[o.b], r));
      }
      bsync();
      if (tid < u.d) {
        const Uop o = prog[pc + 1 + tid];
        sl[o.d] = kara_combine(L.t[3 * tid], L.t[3 * tid + 1], L.t[3 * tid + 2]);
      }
      bsync();
      pc += 1 + u.d;
    } else if (u.code == U_LIN) {
      if (tid == 0) {
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
      bsync();
      pc += 1 + u.d;
    } else {  // U_STORE: the next uop names the (a, b, c) slots
      const Uop m = prog[pc + 1];
      if (tid < 3) {
        const int s = tid == 0 ? m.d : (tid == 1 ? m.a : m.b);
        (&out->a)[tid] = sl[s];
      }
      bsync();
      pc += 2;
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

// The NSTEP prepared lines of Q_i (one workgroup per G2 point); qinf[i] = 1 for the identity
__global__ void __launch_bounds__(PT) prep_lines_kernel(const uint64_t* g2, size_t n, PrepLine* lines,
                                                        uint8_t* qinf, PairingConsts k) {
  __shared__ PL L;
  const int tid = threadIdx.x;
  const size_t i = blockIdx.x;
  if (i >= n) return;
  load_consts(k, L, tid);
  const uint64_t* q = g2 + 16 * i;
  const bool inf = all_zero(q, 16);  // uniform
  if (tid == 0) qinf[i] = inf ? 1 : 0;
  if (inf) return;
  if (tid == 0) {
    const Fq2 xq{ld_mont(q), ld_mont(q + 4)}, yq{ld_mont(q + 8), ld_mont(q + 12)};
    L.Qa[0][0] = xq;
    L.Qa[0][1] = yq;
    L.sl[SL_X] = xq;
    L.sl[SL_Y] = yq;
    L.sl[SL_Z] = Fq2{k.one, u256_zero()};
    // pi(Q) = (conj(x) GX, conj(y) GY), -pi^2(Q) = (conj(x1) GX, -conj(y1) GY)
    const Fq2 gx = L.frob1[2], gy = L.frob1[3];
    const Fq2 x1 = f2_mul(f2_conj(xq), gx), y1 = f2_mul(f2_conj(yq), gy);
    L.Qa[1][0] = x1;
    L.Qa[1][1] = y1;
    L.Qa[2][0] = f2_mul(f2_conj(x1), gx);
    L.Qa[2][1] = f2_neg(f2_mul(f2_conj(y1), gy));
  }
  bsync();
  PrepLine* out = lines + i * NSTEP;
  for (int st = 0; st < NSTEP; ++st) {
    const int kind = c_steps.kind[st];
    if (kind != ST_DBL) {
      if (tid == 0) {
        L.sl[SL_XQ] = L.Qa[kind - ST_ADD_Q][0];
        L.sl[SL_YQ] = L.Qa[kind - ST_ADD_Q][1];
      }
      bsync();
    }
    run_uops(kind == ST_DBL ? c_dbl_prog : c_add_prog, kind == ST_DBL ? DBL_LEN : ADD_LEN, out + st, L, tid);
  }
}

// Lines of pairs [p0, p0 + m) evaluated at their P into L.le (identity pairs: the line 1)
__device__ __forceinline__ void eval_lines(const uint64_t* g1, const PrepLine* lines, const uint8_t* qinf,
                                           size_t p0, int m, const PairingConsts& k, PL& L, int tid) {
  if (tid < m) {
    const uint64_t* p = g1 + 8 * (p0 + tid);
    const bool skip = all_zero(p, 8) || qinf[p0 + tid];
    L.skip[tid] = skip ? 1 : 0;
    L.px[tid] = skip ? u256_zero() : ld_mont(p);
    L.py[tid] = skip ? u256_zero() : ld_mont(p + 4);
  }
  bsync();
  const int jobs = m * NSTEP * 4;
  for (int j = tid; j < jobs; j += PT) {
    const int pp = j / (NSTEP * 4), rem = j - pp * (NSTEP * 4), st = rem >> 2, w = rem & 3;
    const PrepLine& ln = lines[(p0 + pp) * NSTEP + st];
    Fq2* le = L.le[st] + 3 * pp;
    if (L.skip[pp]) {
      const U256 v = w == 0 ? k.one : u256_zero();
      if (w == 0) le[0].c0 = v;
      else if (w == 1) le[0].c1 = v;
      else if (w == 2) le[1].c0 = v;
      else le[1].c1 = v;
      if (w < 2) (w == 0 ? le[2].c0 : le[2].c1) = u256_zero();
    } else {
      const U256 src = w == 0 ? ln.a.c0 : w == 1 ? ln.a.c1 : w == 2 ? ln.b.c0 : ln.b.c1;
      const U256 v = Fq::mul(src, w < 2 ? L.py[pp] : L.px[pp]);
      if (w == 0) le[0].c0 = v;
      else if (w == 1) le[0].c1 = v;
      else if (w == 2) le[1].c0 = v;
      else le[1].c1 = v;
      if (w < 2) (w == 0 ? le[2].c0 : le[2].c1) = w == 0 ? ln.c.c0 : ln.c.c1;
    }
  }
  bsync();
}

// The two lines of every step multiplied together in place (off the Miller loop's critical
// path: all steps are independent): l m = a0 b0 + xi a3 b3 + (a0 b1 + a1 b0) w + a1 b1 w^2
// + (a0 b3 + a3 b0) w^3 + (a1 b3 + a3 b1) w^4, written to le[st][0..4] (the flat w^0..w^4 of a
// W_FIVE operand) with le[st][5] = 0 and xi times them at [6..11]. LB steps per batch.
__device__ __forceinline__ void pair_line_products(PL& L, int tid) {
  // the 9 products (index into l, index into m) and their output coefficient
  constexpr int8_t PA[9] = {0, 2, 0, 1, 1, 0, 2, 1, 2}, PB[9] = {0, 2, 1, 0, 1, 2, 0, 2, 1};
  for (int st0 = 0; st0 < NSTEP; st0 += LB) {
    const int sb = tid / 27, rem = tid - 27 * sb, q = rem / 3, r = rem - 3 * q;
    if (sb < LB && st0 + sb < NSTEP) {
      const Fq2* ln = L.le[st0 + sb];
      const Fq2* mn = L.le[st0 + sb] + 3;
      L.t[tid] = Fq::mul(kara_operand(ln[PA[q]], r), kara_operand(mn[PB[q]], r));
    }
    bsync();
    if (tid < 9 * LB && st0 + tid / 9 < NSTEP) {
      const int qq = tid % 9, base = 27 * (tid / 9) + 3 * qq;
      Fq2 p = kara_combine(L.t[base], L.t[base + 1], L.t[base + 2]);
      if (qq == 1) p = f2_mul_xi(p);  // a3 b3 w^6
      L.pp[tid] = p;
    }
    bsync();
    if (tid < 10 * LB && st0 + tid / 10 < NSTEP) {
      const int sb2 = tid / 10, e = (tid % 10) >> 1, c = tid & 1;
      const Fq2* P = L.pp + 9 * sb2;
      // w^0: p0 + p1, w^1: p2 + p3, w^2: p4, w^3: p5 + p6, w^4: p7 + p8
      const int ia = e == 0 ? 0 : (e == 1 ? 2 : (e == 2 ? 4 : (e == 3 ? 5 : 7)));
      const U256 x0 = c ? P[ia].c1 : P[ia].c0;
      const U256 x1 = e == 2 ? u256_zero() : (c ? P[ia + 1].c1 : P[ia + 1].c0);
      const U256 v = Fq::add(x0, x1);
      Fq2* o = L.le[st0 + sb2] + e;
      if (c) o->c1 = v; else o->c0 = v;
    }
    bsync();
    // the register form's xi half (a line product is the x operand of a merged step's product,
    // pairing_product_kernel) and its zero slot 5
    if (tid < 6 * LB && st0 + tid / 6 < NSTEP) {
      const int sb2 = tid / 6, e = tid % 6;
      Fq2* o = L.le[st0 + sb2];
      const Fq2 v = e == 5 ? Fq2{u256_zero(), u256_zero()} : o[e];
      if (e == 5) o[5] = v;
      o[6 + e] = f2_mul_xi(v);
    }
    bsync();
  }
}

// dA = xA yA (MA) and dB = xB yB (MB) in one set of rounds (w_mul_dual with mixed shapes)
template <int MA, int MB>
__device__ __forceinline__ void w_mul_pair(Fq2* dA, const Fq2* xA, const Fq2* yA, Fq2* dB, const Fq2* xB, const Fq2* yB,
                                           PL& L, int tid) {
  if (tid < 128) wm_r1<MA, false>(xA, yA, L.t, tid);
  else wm_r1<MB, false>(xB, yB, L.t + 128, tid - 128);
  bsync();
  const int wv = tid >> 6, k = tid & 63;
  if (wv == 0) wm_r2<MA>(L.t, L.acc[0], k);
  else if (wv == 1) wm_r2<MB>(L.t + 128, L.acc[1], k);
  bsync();
  if ((k & 31) < 6) {
    const bool b = k >= 32;
    wm_r3(b ? dB : dA, L.acc[b ? 1 : 0], wv, k & 31);
  }
  bsync();
}

// One workgroup multiplies the Miller values of pairs [g per, (g+1) per) (one shared
// squaring per doubling step: f = prod_i f_i exactly) and applies the final
// exponentiation. out_gt: the reduced pairing value of the group (tower order, canonical);
// ok: 1 iff it is one.
__global__ void __launch_bounds__(PT) pairing_product_kernel(const uint64_t* g1, const PrepLine* lines,
                                                             const uint8_t* qinf, size_t n, uint32_t per,
                                                             uint64_t* out_gt, int* ok, PairingConsts k) {
  __shared__ PL L;
  const int tid = threadIdx.x;
  const size_t b0 = (size_t)blockIdx.x * per;
  if (b0 >= n) return;
  const size_t b1 = b0 + per < n ? b0 + per : n;
  load_consts(k, L, tid);
  Fq2* f = L.reg[0];
  Fq2* F = L.reg[NREG - 1];
  for (size_t c = b0; c < b1; c += LCHUNK) {
    const int m = (int)(b1 - c < (size_t)LCHUNK ? b1 - c : (size_t)LCHUNK);
    eval_lines(g1, lines, qinf, c, m, k, L, tid);
    if (m == 2) pair_line_products(L, tid);
    w_one(f, k, tid);
    if (m == 2) {
      // Round 5: a doubling step followed by an addition step multiplies f by the product of the
      // two steps' line products, M = LL(st) LL(st + 1), formed beside the doubling's squaring
      // (w_mul_pair): one dense product per addition step instead of a line product; likewise
      // pi(Q) and -pi^2(Q)'s lines, merged in the first squaring round without an addition
      Fq2* M = L.reg[1];
      Fq2* MP = L.reg[2];
      bool pi_done = false;
      for (int st = 0; st < NSTEP; ++st) {
        const int kind = c_steps.kind[st];
        if (kind == ST_ADD_PI) {  // the last two steps, merged
          if (!pi_done) w_mul<W_FIVE>(MP, L.le[st], L.le[st + 1], L, tid);
          w_mul<W_DENSE>(f, f, MP, L, tid);
          break;
        }
        const bool merge = kind == ST_DBL && st + 1 < NSTEP && c_steps.kind[st + 1] == ST_ADD_Q;
        if (st == 0) {  // f = 1
          if (merge) {
            w_mul<W_FIVE>(M, L.le[0], L.le[1], L, tid);
            w_copy(f, M, tid);
            ++st;
          } else {
            w_mul<W_FIVE>(f, f, L.le[0], L, tid);
          }
          continue;
        }
        if (kind == ST_DBL) {
          if (merge) w_mul_pair<W_DENSE, W_FIVE>(f, f, f, M, L.le[st], L.le[st + 1], L, tid);
          else if (!pi_done) {
            w_mul_pair<W_DENSE, W_FIVE>(f, f, f, MP, L.le[NSTEP - 2], L.le[NSTEP - 1], L, tid);
            pi_done = true;
          } else {
            w_mul<W_DENSE>(f, f, f, L, tid);
          }
        }
        if (merge) {
          w_mul<W_DENSE>(f, f, M, L, tid);
          ++st;
        } else {
          w_mul<W_FIVE>(f, f, L.le[st], L, tid);
        }
      }
    } else {
      for (int st = 0; st < NSTEP; ++st) {
        if (c_steps.kind[st] == ST_DBL && st > 0) w_mul<W_DENSE>(f, f, f, L, tid);  // f = 1 before step 0
        w_mul<W_LINE>(f, f, L.le[st], L, tid);
      }
    }
    if (c == b0) w_copy(F, f, tid);
    else w_mul<W_DENSE>(F, F, f, L, tid);
  }
  w_copy(f, F, tid);
  final_exp_w(k, L, tid);
  if (out_gt && tid < 6) {
    uint64_t* o = out_gt + 48 * blockIdx.x;
    const int s = tower_slot(tid);
    st_canon(o + 8 * s, f[tid].c0);
    st_canon(o + 8 * s + 4, f[tid].c1);
  }
  if (ok && tid == 0) {
    bool eq = Fq::eq(f[0].c0, k.one) && Fq::is_zero(f[0].c1);
    for (int j = 1; j < 6; ++j) eq = eq && f2_is_zero(f[j]);
    *ok = eq ? 1 : 0;
  }
}

// ---------------------------------------------------------------- lane engine (throughput)
// Batched independent pairings (pbf_pairing_bn254_dev at n >= PAIR_LANE_MIN):
// ONE LANE PER PAIRING. The Miller loop's step schedule and the final exponentiation are the
// same for every pairing (fixed 6u+2 and exponent), so the 64 lanes of a wave run one
// instruction stream in lock-step on 64 different pairs -- no cross-lane traffic, no barriers,
// every lane busy -- where the workgroup engine above spends its lanes on one pairing's
// latency. The state (f in Fq12, T, Q, P) is per lane; what does not fit the registers the
// compiler keeps in scratch. Fq12 in the tower Fq6[w]/(w^2 - v), Fq6 = Fq2[v]/(v^3 - xi)
// (flat w^k: c0 = (w^0, w^2, w^4), c1 = (w^1, w^3, w^5), the ABI's tower order); Karatsuba
// products (54 Fq products), complex squaring in the Miller loop (36), the line as a sparse
// operand (a yP at w^0, b xP at w^1, c at w^3: 39), Granger-Scott cyclotomic squaring in the
// hard part (21). Line formulas, step schedule and final-exponentiation chain are the
// workgroup engine's (prep_lines_kernel, make_fe_prog), so every value is the exact reduced
// pairing, bit-identical to oracle/bn254_pairing.py.
struct Fq6 {
  Fq2 c0, c1, c2;
};
struct Fq12 {
  Fq6 c0, c1;
};
__device__ __forceinline__ Fq6 f6_add(const Fq6& a, const Fq6& b) {
  return {f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)};
}
__device__ __forceinline__ Fq6 f6_sub(const Fq6& a, const Fq6& b) {
  return {f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)};
}
__device__ __forceinline__ Fq6 f6_neg(const Fq6& a) { return {f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; }
__device__ __forceinline__ Fq6 f6_mul_v(const Fq6& a) { return {f2_mul_xi(a.c2), a.c0, a.c1}; }
// the Fq6 products are real calls (one copy each): inlined, the engine's code grows past what
// the compiler schedules in reasonable time
__device__ __noinline__ Fq6 f6_mul(const Fq6& a, const Fq6& b) {
  const Fq2 t0 = f2_mul(a.c0, b.c0), t1 = f2_mul(a.c1, b.c1), t2 = f2_mul(a.c2, b.c2);
  const Fq2 u0 = f2_sub(f2_sub(f2_mul(f2_add(a.c1, a.c2), f2_add(b.c1, b.c2)), t1), t2);
  const Fq2 u1 = f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1)), t0), t1);
  const Fq2 u2 = f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c2), f2_add(b.c0, b.c2)), t0), t2);
  return {f2_add(t0, f2_mul_xi(u0)), f2_add(u1, f2_mul_xi(t2)), f2_add(u2, t1)};
}
// a (b0 + b1 v): c0 = a0 b0 + xi a2 b1, c1 = a0 b1 + a1 b0, c2 = a1 b1 + a2 b0
__device__ __noinline__ Fq6 f6_mul_01(const Fq6& a, const Fq2& b0, const Fq2& b1) {
  return {f2_add(f2_mul(a.c0, b0), f2_mul_xi(f2_mul(a.c2, b1))), f2_add(f2_mul(a.c0, b1), f2_mul(a.c1, b0)),
          f2_add(f2_mul(a.c1, b1), f2_mul(a.c2, b0))};
}
__device__ __forceinline__ Fq12 f12_mul(const Fq12& a, const Fq12& b) {
  const Fq6 t0 = f6_mul(a.c0, b.c0), t1 = f6_mul(a.c1, b.c1);
  const Fq6 s = f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1));
  return {f6_add(t0, f6_mul_v(t1)), f6_sub(f6_sub(s, t0), t1)};
}
// (a0 + a1 w)^2 = (a0 + a1)(a0 + v a1) - t - v t + 2 t w, t = a0 a1
__device__ __forceinline__ Fq12 f12_sqr(const Fq12& a) {
  const Fq6 t = f6_mul(a.c0, a.c1);
  const Fq6 s = f6_mul(f6_add(a.c0, a.c1), f6_add(a.c0, f6_mul_v(a.c1)));
  return {f6_sub(f6_sub(s, t), f6_mul_v(t)), f6_add(t, t)};
}
// f * l, l = A0 + (B0 + B1 v) w (the line: A0 = a yP at w^0, B0 = b xP at w^1, B1 = c at w^3)
__device__ __forceinline__ Fq12 f12_mul_line(const Fq12& f, const Fq2& A0, const Fq2& B0, const Fq2& B1) {
  const Fq6 t0 = {f2_mul(f.c0.c0, A0), f2_mul(f.c0.c1, A0), f2_mul(f.c0.c2, A0)};
  const Fq6 t1 = f6_mul_01(f.c1, B0, B1);
  const Fq6 s = f6_mul_01(f6_add(f.c0, f.c1), f2_add(A0, B0), B1);
  return {f6_add(t0, f6_mul_v(t1)), f6_sub(f6_sub(s, t0), t1)};
}
__device__ __forceinline__ Fq12 f12_conj(const Fq12& a) { return {a.c0, f6_neg(a.c1)}; }
// x^q: flat g_k -> conj(g_k) FROB1[k]
__device__ __forceinline__ Fq12 f12_frob1(const Fq12& a, const PairingConsts& k) {
  auto fr = [&](const Fq2& g, int i) { return f2_mul(f2_conj(g), Fq2{k.frob1[i][0], k.frob1[i][1]}); };
  return {{fr(a.c0.c0, 0), fr(a.c0.c1, 2), fr(a.c0.c2, 4)}, {fr(a.c1.c0, 1), fr(a.c1.c1, 3), fr(a.c1.c2, 5)}};
}
// x^(q^2): flat g_k -> g_k FROB2[k]
__device__ __forceinline__ Fq12 f12_frob2(const Fq12& a, const PairingConsts& k) {
  return {{f2_muls(a.c0.c0, k.frob2[0]), f2_muls(a.c0.c1, k.frob2[2]), f2_muls(a.c0.c2, k.frob2[4])},
          {f2_muls(a.c1.c0, k.frob2[1]), f2_muls(a.c1.c1, k.frob2[3]), f2_muls(a.c1.c2, k.frob2[5])}};
}
// Granger-Scott squaring in the cyclotomic subgroup (per lane):
// A_m = g_m + g_(m+3) s (s = w^3, s^2 = xi), A_m^2 = (a^2 + xi b^2) + 2 a b s; flat outputs
// 3 S -/+ 2 g_k
__device__ __noinline__ Fq12 f12_csqr(const Fq12& x) {
  const Fq2 g[6] = {x.c0.c0, x.c1.c0, x.c0.c1, x.c1.c1, x.c0.c2, x.c1.c2};  // flat w^0..w^5
  Fq2 lo[3], hi[3];
  for (int m = 0; m < 3; ++m) {
    const Fq2 a = g[m], b = g[m + 3];
    lo[m] = f2_add(f2_sqr(a), f2_mul_xi(f2_sqr(b)));
    hi[m] = f2_dbl(f2_mul(a, b));
  }
  const Fq2 S[6] = {lo[0], f2_mul_xi(hi[2]), lo[1], hi[0], lo[2], hi[1]};
  Fq2 o[6];
#pragma unroll
  for (int kk = 0; kk < 6; ++kk) {
    const Fq2 s3 = f2_add(f2_dbl(S[kk]), S[kk]), g2 = f2_dbl(g[kk]);
    o[kk] = (kk & 1) ? f2_add(s3, g2) : f2_sub(s3, g2);
  }
  return {{o[0], o[2], o[4]}, {o[1], o[3], o[5]}};
}
__device__ __forceinline__ Fq6 f6_inv(const Fq6& n, const PairingConsts& k) {
  const Fq2 t0 = f2_sub(f2_sqr(n.c0), f2_mul_xi(f2_mul(n.c1, n.c2)));
  const Fq2 t1 = f2_sub(f2_mul_xi(f2_sqr(n.c2)), f2_mul(n.c0, n.c1));
  const Fq2 t2 = f2_sub(f2_sqr(n.c1), f2_mul(n.c0, n.c2));
  const Fq2 den = f2_add(f2_mul(n.c0, t0), f2_mul_xi(f2_add(f2_mul(n.c2, t1), f2_mul(n.c1, t2))));
  const Fq2 di = f2_inv(den, k);
  return {f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di)};
}
// f^((q^12-1)/r): make_fe_prog's chain run by an interpreter over per-lane Fq12 registers (a
// local array: scratch), each primitive inlined once; the hard part's squarings are cyclotomic
// (the value is in the cyclotomic subgroup there, so they are the same field elements)
__device__ __noinline__ void f12_final_exp(Fq12* R, const PairingConsts& k) {
  const Fq2 z{u256_zero(), u256_zero()};
  for (int pc = 0; pc < c_fe_seq.n; ++pc) {
    const FeOp o = c_fe_seq.ops[pc];
    const Fq12 a = R[o.op == FE_INVN ? o.dst : o.a];
    Fq12 d;
    switch (o.op) {
      case FE_MUL: d = f12_mul(a, R[o.b]); break;
      case FE_CSQR: d = f12_csqr(a); break;
      case FE_CONJ: d = f12_conj(a); break;
      case FE_FROB1: d = f12_frob1(a, k); break;
      case FE_FROB2: d = f12_frob2(a, k); break;
      case FE_COPY: d = a; break;
      default: d = Fq12{f6_inv(a.c0, k), {z, z, z}}; break;  // FE_INVN: an Fq6 value (c1 = 0)
    }
    R[o.dst] = d;
  }
}

constexpr size_t PAIR_LANE_MIN = 64;  // batches from this size take the lane engine

// WPE: waves per SIMD the compiler must allow. One lane per pairing puts a batch of 65536 at
// one wave per SIMD, where the unconstrained build (256 VGPRs) is fastest; from two waves per
// SIMD the build held at 2 (more scratch, two waves hiding each other's latency) is faster:
// 262144 pairings 1.89 -> 2.41 M/s, 65536 1.83 -> 1.78 M/s (profiles/r05/lanew_ab.log)
template <int WPE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) pairing_lane_kernel(const uint64_t* g1, const uint64_t* g2, size_t n,
                                                          uint64_t* out, PairingConsts k) {
  const size_t i0 = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t i = i0 < n ? i0 : n - 1;  // surplus lanes repeat the last pair and store nothing
  const uint64_t* p = g1 + 8 * i;
  const uint64_t* q = g2 + 16 * i;
  const bool inf = all_zero(p, 8) || all_zero(q, 16);
  const U256 xp = ld_mont(p), yp = ld_mont(p + 4);
  const Fq2 xq{ld_mont(q), ld_mont(q + 4)}, yq{ld_mont(q + 8), ld_mont(q + 12)};
  // Q, pi(Q), -pi^2(Q) (prep_lines_kernel)
  const Fq2 gx{k.frob1[2][0], k.frob1[2][1]}, gy{k.frob1[3][0], k.frob1[3][1]};
  const Fq2 x1 = f2_mul(f2_conj(xq), gx), y1 = f2_mul(f2_conj(yq), gy);
  const Fq2 x2 = f2_mul(f2_conj(x1), gx), y2 = f2_neg(f2_mul(f2_conj(y1), gy));
  Fq2 X = xq, Y = yq, Z{k.one, u256_zero()};
  const Fq2 zero{u256_zero(), u256_zero()};
  Fq12 f{{Fq2{k.one, u256_zero()}, zero, zero}, {zero, zero, zero}};
  for (int st = 0; st < NSTEP; ++st) {
    const int kind = c_steps.kind[st];
    Fq2 la, lb, lc;  // line: la yP + (lb xP) w + lc w^3
    if (kind == ST_DBL) {
      if (st > 0) f = f12_sqr(f);
      // w = 3X^2, s = 2YZ, R = Y s, B = (X+R)^2 - X^2 - R^2, h = w^2 - 2B,
      // X3 = h s, Y3 = w (B - h) - 2 R^2, Z3 = s^3; line (sZ, -wZ, wX - R)
      const Fq2 xx = f2_sqr(X), w = f2_add(f2_dbl(xx), xx), s = f2_dbl(f2_mul(Y, Z));
      const Fq2 R = f2_mul(Y, s), RR = f2_sqr(R);
      const Fq2 B = f2_sub(f2_sub(f2_sqr(f2_add(X, R)), xx), RR);
      const Fq2 h = f2_sub(f2_sqr(w), f2_dbl(B));
      la = f2_mul(s, Z);
      lb = f2_neg(f2_mul(w, Z));
      lc = f2_sub(f2_mul(w, X), R);
      X = f2_mul(h, s);
      Y = f2_sub(f2_mul(w, f2_sub(B, h)), f2_dbl(RR));
      Z = f2_mul(f2_sqr(s), s);
    } else {
      const Fq2 xa = kind == ST_ADD_Q ? xq : (kind == ST_ADD_PI ? x1 : x2);
      const Fq2 ya = kind == ST_ADD_Q ? yq : (kind == ST_ADD_PI ? y1 : y2);
      // N = yq Z - Y, D = xq Z - X, A = N^2 Z - D^3 - 2 D^2 X, X3 = D A,
      // Y3 = N (D^2 X - A) - D^3 Y, Z3 = D^3 Z; line (D, -N, N xq - D yq)
      const Fq2 N = f2_sub(f2_mul(ya, Z), Y), D = f2_sub(f2_mul(xa, Z), X);
      const Fq2 DD = f2_sqr(D), DDD = f2_mul(D, DD), DDX = f2_mul(DD, X);
      const Fq2 A = f2_sub(f2_sub(f2_mul(f2_sqr(N), Z), DDD), f2_dbl(DDX));
      la = D;
      lb = f2_neg(N);
      lc = f2_sub(f2_mul(N, xa), f2_mul(D, ya));
      X = f2_mul(D, A);
      Y = f2_sub(f2_mul(N, f2_sub(DDX, A)), f2_mul(DDD, Y));
      Z = f2_mul(DDD, Z);
    }
    f = f12_mul_line(f, f2_muls(la, yp), f2_muls(lb, xp), lc);
  }
  Fq12 R[FE_SEQ_REGS];
  R[0] = f;
  f12_final_exp(R, k);
  f = R[0];
  if (inf) f = Fq12{{Fq2{k.one, u256_zero()}, zero, zero}, {zero, zero, zero}};
  if (i0 < n) {
    uint64_t* o = out + 48 * i;
    const Fq2 c[6] = {f.c0.c0, f.c0.c1, f.c0.c2, f.c1.c0, f.c1.c1, f.c1.c2};
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      st_canon(o + 8 * j, c[j].c0);
      st_canon(o + 8 * j + 4, c[j].c1);
    }
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

// g_inv2k on `device` (once per device): 2^-k R^3 mod q for k < 512, plain, from K_R3 and
// Montgomery products by 2^-1 (the host's Fq::mul)
static int ensure_inv2k(int device) {
  static std::mutex mu;
  static bool done[256];
  std::lock_guard<std::mutex> g(mu);
  if (device < 0 || device >= 256) return fail(1, "device index out of range");
  if (done[device]) return 0;
  U256 inv2{};  // (q + 1) / 2
  {
    uint64_t c = 1;
    U256 q1;
    for (int i = 0; i < 8; ++i) {
      const uint64_t t = (uint64_t)Bn254FqParams::P[i] + c;
      q1.w[i] = (uint32_t)t;
      c = t >> 32;
    }
    for (int i = 0; i < 8; ++i) inv2.w[i] = (q1.w[i] >> 1) | (i < 7 ? (q1.w[i + 1] << 31) : 0);
  }
  const U256 inv2m = Fq::to_mont(inv2);
  std::vector<U256> t(512);
  U256 c = u256_from_u64(K_R3);
  for (int k = 0; k < 512; ++k) {
    t[k] = c;
    c = Fq::mul(c, inv2m);  // c 2^-1 R R^-1
  }
  int cur = 0;
  PBF_HIP(hipGetDevice(&cur));
  PBF_HIP(hipSetDevice(device));
  const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_inv2k), t.data(), t.size() * sizeof(U256));
  PBF_HIP(hipSetDevice(cur));
  if (e != hipSuccess) return fail(PBF_EDEVICE, "hipMemcpyToSymbol(g_inv2k) failed");
  done[device] = true;
  return 0;
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

// Enqueue prepared lines of n G2 points (device) into the context's line buffers
static int prep_lines(pbf_ctx* ctx, const uint64_t* d_g2, size_t n, hipStream_t s, const PairingConsts& k,
                      PrepLine** lines, uint8_t** qinf) {
  DevBuf &bl = ctx->buf("pair.lines"), &bq = ctx->buf("pair.qinf");
  int rc;
  if ((rc = bl.ensure(n * NSTEP * sizeof(PrepLine))) || (rc = bq.ensure(n))) return rc;
  *lines = (PrepLine*)bl.p;
  *qinf = (uint8_t*)bq.p;
  hipLaunchKernelGGL(prep_lines_kernel, dim3((uint32_t)n), dim3(PT), 0, s, d_g2, n, *lines, *qinf, k);
  PBF_HIP(hipGetLastError());
  return 0;
}

// e(P_i, Q_i) for every i: from PAIR_LANE_MIN pairs one lane per pairing (pairing_lane_kernel;
// PBF_PAIR_WG=1 keeps the workgroup engine), below that prepared lines, then one workgroup per
// pair (the latency form)
static int pairing_values(pbf_ctx* ctx, const uint64_t* d_g1, const uint64_t* d_g2, size_t n, uint64_t* d_out,
                          hipStream_t s) {
  int rc = ensure_inv2k(ctx->device);
  if (rc) return rc;
  const PairingConsts k = make_consts();
  // option pair.engine = "lane" / "wg" forces an engine (the tests' cross-check)
  const char* eng = ctx->options.get("pair.engine");
  const bool lane = eng ? strcmp(eng, "lane") == 0 : n >= PAIR_LANE_MIN;
  if (lane) {
    const uint32_t waves = (uint32_t)((n + 63) / 64);
    int dev_cus = 0;
    PBF_HIP(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    bool two = waves >= (uint32_t)(8 * dev_cus);  // at least two waves per SIMD (four SIMDs per CU)
    if (const char* w = ctx->options.get("pair.lane_wpe")) two = w[0] == '2';  // option (tests): force a build
    if (two)
      hipLaunchKernelGGL(pairing_lane_kernel<2>, dim3(waves), dim3(64), 0, s, d_g1, d_g2, n, d_out, k);
    else
      hipLaunchKernelGGL(pairing_lane_kernel<1>, dim3(waves), dim3(64), 0, s, d_g1, d_g2, n, d_out, k);
    PBF_HIP(hipGetLastError());
    return 0;
  }
  PrepLine* lines;
  uint8_t* qinf;
  rc = prep_lines(ctx, d_g2, n, s, k, &lines, &qinf);
  if (rc) return rc;
  hipLaunchKernelGGL(pairing_product_kernel, dim3((uint32_t)n), dim3(PT), 0, s, d_g1, (const PrepLine*)lines,
                     (const uint8_t*)qinf, n, 1u, d_out, (int*)nullptr, k);
  PBF_HIP(hipGetLastError());
  return 0;
}

extern "C" int pbf_pairing_bn254(pbf_ctx* ctx, const uint64_t* g1, const uint64_t* g2, size_t n, uint64_t* out) {
  if (!ctx || (n && (!g1 || !g2 || !out))) return fail(1, "null argument");
  if (n == 0) return 0;
  if (n > 0x7fffffffu) return fail(1, "batch too large");
  int rc = check_coords(g1, 2 * n);
  if (!rc) rc = check_coords(g2, 4 * n);
  if (rc) return rc;
  PBF_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->host_stream();
  if ((rc = ctx->io0.ensure(n * 64)) || (rc = ctx->io1.ensure(n * 128)) || (rc = ctx->io2.ensure(n * 384))) return rc;
  PBF_HIP(hipMemcpyAsync(ctx->io0.p, g1, n * 64, hipMemcpyHostToDevice, s));
  PBF_HIP(hipMemcpyAsync(ctx->io1.p, g2, n * 128, hipMemcpyHostToDevice, s));
  if ((rc = pairing_values(ctx, (const uint64_t*)ctx->io0.p, (const uint64_t*)ctx->io1.p, n, (uint64_t*)ctx->io2.p,
                           s)))
    return rc;
  PBF_HIP(hipMemcpyAsync(out, ctx->io2.p, n * 384, hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  return 0;
}

extern "C" int pbf_pairing_bn254_dev(pbf_ctx* ctx, const uint64_t* d_g1, const uint64_t* d_g2, size_t n,
                                     uint64_t* d_out, void* stream) {
  if (!ctx) return fail(1, "null context");
  if (n == 0) return 0;
  if (n > 0x7fffffffu) return fail(1, "batch too large");
  return pairing_values(ctx, d_g1, d_g2, n, d_out, pbf_ctx::pick(stream));
}

// The pairing check on an explicit stream (host g1 / g2, synchronous): used by
// pbf_pairing_check_bn254 (context host stream) and Plonk::verify's `_dev` entry (its
// caller's stream). The G2 side's prepared lines are kept in the context and reused while
// the G2 inputs are the same bytes (a verifier checks against the same [1]G2, [s]G2 every
// time): only the G1 side is then evaluated, multiplied and exponentiated.
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
  DevBuf &b1 = ctx->buf("pc.g1"), &b2 = ctx->buf("pc.g2"), &b3 = ctx->buf("pc.ok");
  DevBuf &cl = ctx->buf("pc.lines"), &cq = ctx->buf("pc.qinf");
  if ((rc = b1.ensure(n * 64)) || (rc = b2.ensure(n * 128)) || (rc = b3.ensure(64))) return rc;
  if ((rc = ensure_inv2k(ctx->device))) return rc;
  const PairingConsts k = make_consts();
  auto& key = ctx->pair_g2_key;
  const bool hit = key.size() == 16 * n && memcmp(key.data(), g2, n * 128) == 0 && cl.p && cq.p;
  if (!hit) {
    key.clear();  // the lines are rewritten below; a failure in between must not leave a stale hit
    if ((rc = cl.ensure(n * NSTEP * sizeof(PrepLine))) || (rc = cq.ensure(n))) return rc;
    PBF_HIP(hipMemcpyAsync(b2.p, g2, n * 128, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(prep_lines_kernel, dim3((uint32_t)n), dim3(PT), 0, s, (const uint64_t*)b2.p, n,
                       (PrepLine*)cl.p, (uint8_t*)cq.p, k);
    PBF_HIP(hipGetLastError());
    key.assign(g2, g2 + 16 * n);
  }
  PBF_HIP(hipMemcpyAsync(b1.p, g1, n * 64, hipMemcpyHostToDevice, s));
  int* d_ok = (int*)b3.p;
  hipLaunchKernelGGL(pairing_product_kernel, dim3(1), dim3(PT), 0, s, (const uint64_t*)b1.p,
                     (const PrepLine*)cl.p, (const uint8_t*)cq.p, n, (uint32_t)n, (uint64_t*)nullptr, d_ok, k);
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
  if (!rc) rc = ensure_inv2k(ctx->device);
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
