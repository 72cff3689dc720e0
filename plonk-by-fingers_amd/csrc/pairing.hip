// BN254 optimal-ate pairing on gfx950 (BASELINE config 4 "pairing check"; the BN254
// instance of the reference's Pairing::pairing, src/ec.rs:87-93 / src/pbh/pairing.rs:12-47,
// which Plonk::verify calls twice, src/plonk.rs:646-647).
//
//   e(P, Q) = ( f_{6u+2,Q}(P) * l_{T,pi(Q)}(P) * l_{T',-pi^2(Q)}(P) )^((q^12-1)/r)
//
// Tower: Fq2 = Fq[u]/(u^2+1), Fq6 = Fq2[v]/(v^3-xi), xi = 9+u, Fq12 = Fq6[w]/(w^2-v);
// G2 on the D-type twist y^2 = x^3 + 3/xi. Miller loop over the bits of 6u+2 with affine
// T (one Fq2 inversion per step), lines l = yP - lam*xP*w + (lam*xT - yT)*v*w (vertical
// parts dropped: they lie in Fq6 and die in the final exponentiation). Final
// exponentiation: easy part f^(q^6-1) (conjugate / inverse) and f^(q^2+1) (Frobenius
// constants), hard part a plain square-and-multiply by (q^4-q^2+1)/r, so the value is
// exactly the reduced pairing of oracle/bn254_pairing.py (no exponent multiple).
//
// One thread per pairing (pairings are few: two per KZG check, batched across proofs —
// SURVEY.md §8e "replicas only"). Fq elements in Montgomery form inside kernels; the
// ABI carries canonical little-endian limbs (GT: 12 Fq in tower order).
#include <vector>
#include "../../include/pbf.h"
#include "ec_bn254.hpp"
#include "internal.hpp"

namespace pbf {

// ---------------------------------------------------------------- constants
// Generated from q alone by scripts/gen_pairing_constants.py (canonical, little-endian):
//   GAMMA_X = xi^((q-1)/3), GAMMA_Y = xi^((q-1)/2) (Fq2: twist Frobenius)
//   FROB2[k] = xi^(k(q^2-1)/6) (in Fq), k = 1..5 (Fq12 q^2-power Frobenius on w^k)
//   HARD = (q^4 - q^2 + 1)/r (761 bits), ATE = 6u+2
struct PairingConsts {
  U256 gx0, gx1, gy0, gy1;  // Montgomery
  U256 frob2[6];            // Montgomery
  U256 one, xi_unused;
  uint64_t hard[12];
  uint64_t ate;             // low 64 bits of 6u+2 (bit 64 is set too)
  uint64_t qm2[4];          // q - 2 (Fermat inverse)
};

static const uint64_t K_GX[2][4] = {
    {0x99e39557176f553dull, 0xb78cc310c2c3330cull, 0x4c0bec3cf559b143ull, 0x2fb347984f7911f7ull},
    {0x1665d51c640fcba2ull, 0x32ae2a1d0b7c9dceull, 0x4ba4cc8bd75a0794ull, 0x16c9e55061ebae20ull}};
static const uint64_t K_GY[2][4] = {
    {0xdc54014671a0135aull, 0xdbaae0eda9c95998ull, 0xdc5ec698b6e2f9b9ull, 0x063cf305489af5dcull},
    {0x82d37f632623b0e3ull, 0x21807dc98fa25bd2ull, 0x0704b5a7ec796f2bull, 0x07c03cbcac41049aull}};
static const uint64_t K_FROB2[6][4] = {
    {0x0000000000000001ull, 0, 0, 0},
    {0xe4bd44e5607cfd49ull, 0xc28f069fbb966e3dull, 0x5e6dd9e7e0acccb0ull, 0x30644e72e131a029ull},
    {0xe4bd44e5607cfd48ull, 0xc28f069fbb966e3dull, 0x5e6dd9e7e0acccb0ull, 0x30644e72e131a029ull},
    {0x3c208c16d87cfd46ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
    {0x5763473177fffffeull, 0xd4f263f1acdb5c4full, 0x59e26bcea0d48bacull, 0x0000000000000000ull},
    {0x5763473177ffffffull, 0xd4f263f1acdb5c4full, 0x59e26bcea0d48bacull, 0x0000000000000000ull}};
static const uint64_t K_HARD[12] = {0xe81bb482ccdf42b1ull, 0x5abf5cc4f49c36d4ull, 0xf1154e7e1da014fdull,
                                    0xdcc7b44c87cdbacfull, 0xaaa441e3954bcf8aull, 0x6b887d56d5095f23ull,
                                    0x79581e16f3fd90c6ull, 0x3b1b1355d189227dull, 0x4e529a5861876f6bull,
                                    0x6c0eb522d5b12278ull, 0x331ec15183177fafull, 0x01baaa710b0759adull};
static const uint64_t K_ATE_LO = 0x9d797039be763ba8ull;  // 6u+2 = 2^64 + K_ATE_LO

// ---------------------------------------------------------------- tower arithmetic
struct Fq2 {
  U256 c0, c1;
};
struct Fq6 {
  Fq2 a0, a1, a2;
};
struct Fq12 {
  Fq6 c0, c1;
};

__device__ inline Fq2 f2_add(const Fq2& a, const Fq2& b) { return {Fq::add(a.c0, b.c0), Fq::add(a.c1, b.c1)}; }
__device__ inline Fq2 f2_sub(const Fq2& a, const Fq2& b) { return {Fq::sub(a.c0, b.c0), Fq::sub(a.c1, b.c1)}; }
__device__ inline Fq2 f2_neg(const Fq2& a) { return {Fq::sub(u256_zero(), a.c0), Fq::sub(u256_zero(), a.c1)}; }
__device__ inline Fq2 f2_dbl(const Fq2& a) { return f2_add(a, a); }
__device__ inline Fq2 f2_conj(const Fq2& a) { return {a.c0, Fq::sub(u256_zero(), a.c1)}; }
__device__ inline Fq2 f2_muls(const Fq2& a, const U256& s) { return {Fq::mul(a.c0, s), Fq::mul(a.c1, s)}; }
__device__ __noinline__ Fq2 f2_mul(const Fq2& a, const Fq2& b) {
  // Karatsuba: (a0 b0 - a1 b1) + ((a0 + a1)(b0 + b1) - a0 b0 - a1 b1) u
  const U256 t0 = Fq::mul(a.c0, b.c0), t1 = Fq::mul(a.c1, b.c1);
  const U256 t2 = Fq::mul(Fq::add(a.c0, a.c1), Fq::add(b.c0, b.c1));
  return {Fq::sub(t0, t1), Fq::sub(Fq::sub(t2, t0), t1)};
}
__device__ inline Fq2 f2_sqr(const Fq2& a) { return f2_mul(a, a); }
// (9 + u)(a0 + a1 u) = (9 a0 - a1) + (a0 + 9 a1) u
__device__ inline Fq2 f2_mul_xi(const Fq2& a) {
  auto nine = [](const U256& x) {
    const U256 x2 = Fq::add(x, x), x4 = Fq::add(x2, x2), x8 = Fq::add(x4, x4);
    return Fq::add(x8, x);
  };
  return {Fq::sub(nine(a.c0), a.c1), Fq::add(a.c0, nine(a.c1))};
}
__device__ bool f2_is_zero(const Fq2& a) { return Fq::is_zero(a.c0) && Fq::is_zero(a.c1); }
__device__ bool f2_eq(const Fq2& a, const Fq2& b) { return Fq::eq(a.c0, b.c0) && Fq::eq(a.c1, b.c1); }

__device__ __noinline__ U256 fq_pow(U256 a, const uint64_t* e, int words) {
  U256 r = G1::one_m();
  for (int i = words * 64 - 1; i >= 0; --i) {
    r = Fq::mul(r, r);
    if ((e[i >> 6] >> (i & 63)) & 1) r = Fq::mul(r, a);
  }
  return r;
}
__device__ __noinline__ U256 fq_inv(const U256& a, const PairingConsts& k) { return fq_pow(a, k.qm2, 4); }
__device__ __noinline__ Fq2 f2_inv(const Fq2& a, const PairingConsts& k) {
  const U256 n = Fq::add(Fq::mul(a.c0, a.c0), Fq::mul(a.c1, a.c1));
  const U256 ni = fq_inv(n, k);
  return {Fq::mul(a.c0, ni), Fq::sub(u256_zero(), Fq::mul(a.c1, ni))};
}

__device__ inline Fq6 f6_add(const Fq6& a, const Fq6& b) {
  return {f2_add(a.a0, b.a0), f2_add(a.a1, b.a1), f2_add(a.a2, b.a2)};
}
__device__ inline Fq6 f6_sub(const Fq6& a, const Fq6& b) {
  return {f2_sub(a.a0, b.a0), f2_sub(a.a1, b.a1), f2_sub(a.a2, b.a2)};
}
__device__ inline Fq6 f6_neg(const Fq6& a) { return {f2_neg(a.a0), f2_neg(a.a1), f2_neg(a.a2)}; }
__device__ inline Fq6 f6_mul_v(const Fq6& a) { return {f2_mul_xi(a.a2), a.a0, a.a1}; }
__device__ __noinline__ Fq6 f6_mul(const Fq6& a, const Fq6& b) {
  // Karatsuba over Fq2 (v^3 = xi)
  const Fq2 t0 = f2_mul(a.a0, b.a0), t1 = f2_mul(a.a1, b.a1), t2 = f2_mul(a.a2, b.a2);
  const Fq2 m12 = f2_sub(f2_sub(f2_mul(f2_add(a.a1, a.a2), f2_add(b.a1, b.a2)), t1), t2);
  const Fq2 m01 = f2_sub(f2_sub(f2_mul(f2_add(a.a0, a.a1), f2_add(b.a0, b.a1)), t0), t1);
  const Fq2 m02 = f2_sub(f2_sub(f2_mul(f2_add(a.a0, a.a2), f2_add(b.a0, b.a2)), t0), t2);
  return {f2_add(t0, f2_mul_xi(m12)), f2_add(m01, f2_mul_xi(t2)), f2_add(m02, t1)};
}
__device__ __noinline__ Fq6 f6_inv(const Fq6& a, const PairingConsts& k) {
  const Fq2 t0 = f2_sub(f2_sqr(a.a0), f2_mul_xi(f2_mul(a.a1, a.a2)));
  const Fq2 t1 = f2_sub(f2_mul_xi(f2_sqr(a.a2)), f2_mul(a.a0, a.a1));
  const Fq2 t2 = f2_sub(f2_sqr(a.a1), f2_mul(a.a0, a.a2));
  const Fq2 n = f2_add(f2_mul(a.a0, t0), f2_mul_xi(f2_add(f2_mul(a.a2, t1), f2_mul(a.a1, t2))));
  const Fq2 ni = f2_inv(n, k);
  return {f2_mul(t0, ni), f2_mul(t1, ni), f2_mul(t2, ni)};
}

__device__ __noinline__ Fq12 f12_mul(const Fq12& a, const Fq12& b) {
  const Fq6 t0 = f6_mul(a.c0, b.c0), t1 = f6_mul(a.c1, b.c1);
  const Fq6 m = f6_sub(f6_sub(f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1)), t0), t1);
  return {f6_add(t0, f6_mul_v(t1)), m};
}
__device__ inline Fq12 f12_sqr(const Fq12& a) { return f12_mul(a, a); }
__device__ inline Fq12 f12_conj(const Fq12& a) { return {a.c0, f6_neg(a.c1)}; }
__device__ __noinline__ Fq12 f12_inv(const Fq12& a, const PairingConsts& k) {
  const Fq6 n = f6_sub(f6_mul(a.c0, a.c0), f6_mul_v(f6_mul(a.c1, a.c1)));
  const Fq6 ni = f6_inv(n, k);
  return {f6_mul(a.c0, ni), f6_neg(f6_mul(a.c1, ni))};
}
// x^(q^2): coefficient of w^k (c0: k = 0, 2, 4; c1: k = 1, 3, 5) times xi^(k(q^2-1)/6)
__device__ Fq12 f12_frob2(const Fq12& a, const PairingConsts& k) {
  Fq12 r;
  r.c0.a0 = a.c0.a0;
  r.c0.a1 = f2_muls(a.c0.a1, k.frob2[2]);
  r.c0.a2 = f2_muls(a.c0.a2, k.frob2[4]);
  r.c1.a0 = f2_muls(a.c1.a0, k.frob2[1]);
  r.c1.a1 = f2_muls(a.c1.a1, k.frob2[3]);
  r.c1.a2 = f2_muls(a.c1.a2, k.frob2[5]);
  return r;
}
__device__ Fq12 f12_one(const PairingConsts& k) {
  Fq12 r;
  const U256 z = u256_zero();
  r.c0.a0 = {k.one, z};
  r.c0.a1 = r.c0.a2 = r.c1.a0 = r.c1.a1 = r.c1.a2 = Fq2{z, z};
  return r;
}

__device__ __noinline__ Fq12 final_exp(const Fq12& f, const PairingConsts& k) {
  Fq12 f1 = f12_mul(f12_conj(f), f12_inv(f, k));   // f^(q^6 - 1)
  Fq12 f2 = f12_mul(f12_frob2(f1, k), f1);          // ^(q^2 + 1)
  Fq12 r = f12_one(k);                              // ^((q^4 - q^2 + 1)/r)
  for (int i = 12 * 64 - 1; i >= 0; --i) {
    if (i >= 761) continue;
    r = f12_sqr(r);
    if ((k.hard[i >> 6] >> (i & 63)) & 1) r = f12_mul(r, f2);
  }
  return r;
}

// ---------------------------------------------------------------- Miller loop
struct G2A {
  Fq2 x, y;
};

// f *= (yP) + (-lam xP) w + (lam xT - yT) v w
__device__ __noinline__ Fq12 mul_line(const Fq12& f, const Fq2& lam, const G2A& t, const U256& xp, const U256& yp) {
  Fq12 l;
  const U256 z = u256_zero();
  l.c0.a0 = {yp, z};
  l.c0.a1 = l.c0.a2 = Fq2{z, z};
  l.c1.a0 = f2_neg(f2_muls(lam, xp));
  l.c1.a1 = f2_sub(f2_mul(lam, t.x), t.y);
  l.c1.a2 = Fq2{z, z};
  return f12_mul(f, l);
}

__device__ __noinline__ Fq12 miller_loop(const U256& xp, const U256& yp, const G2A& q, const PairingConsts& k) {
  Fq12 f = f12_one(k);
  G2A t = q;
  const U256 three = Fq::add(Fq::add(k.one, k.one), k.one);
  // bits of 6u+2 = 2^64 + ATE_LO below the leading one (bit 64)
  for (int i = 63; i >= 0; --i) {
    // doubling step: lam = 3 xT^2 / (2 yT)
    Fq2 lam = f2_mul(f2_muls(f2_sqr(t.x), three), f2_inv(f2_dbl(t.y), k));
    f = mul_line(f12_sqr(f), lam, t, xp, yp);
    Fq2 x3 = f2_sub(f2_sqr(lam), f2_dbl(t.x));
    t.y = f2_sub(f2_mul(lam, f2_sub(t.x, x3)), t.y);
    t.x = x3;
    if ((k.ate >> i) & 1) {
      lam = f2_mul(f2_sub(q.y, t.y), f2_inv(f2_sub(q.x, t.x), k));
      f = mul_line(f, lam, t, xp, yp);
      x3 = f2_sub(f2_sub(f2_sqr(lam), t.x), q.x);
      t.y = f2_sub(f2_mul(lam, f2_sub(t.x, x3)), t.y);
      t.x = x3;
    }
  }
  // Q1 = pi(Q), Q2 = -pi^2(Q)
  const Fq2 gx{k.gx0, k.gx1}, gy{k.gy0, k.gy1};
  G2A q1{f2_mul(f2_conj(q.x), gx), f2_mul(f2_conj(q.y), gy)};
  G2A q2{f2_mul(f2_conj(q1.x), gx), f2_neg(f2_mul(f2_conj(q1.y), gy))};
  for (int s = 0; s < 2; ++s) {
    const G2A& qq = s ? q2 : q1;
    const Fq2 lam = f2_mul(f2_sub(qq.y, t.y), f2_inv(f2_sub(qq.x, t.x), k));
    f = mul_line(f, lam, t, xp, yp);
    const Fq2 x3 = f2_sub(f2_sub(f2_sqr(lam), t.x), qq.x);
    t.y = f2_sub(f2_mul(lam, f2_sub(t.x, x3)), t.y);
    t.x = x3;
  }
  return f;
}

// ---------------------------------------------------------------- ABI <-> device layouts
__device__ inline U256 ld_mont(const uint64_t* p) { return Fq::to_mont(u256_from_u64(p)); }
__device__ inline void st_canon(uint64_t* p, const U256& a) { u256_to_u64(Fq::from_mont(a), p); }
__device__ inline bool all_zero(const uint64_t* p, int n) {
  uint64_t o = 0;
  for (int i = 0; i < n; ++i) o |= p[i];
  return o == 0;
}
__device__ void store_f12(uint64_t* out, const Fq12& f) {
  const Fq2* c[6] = {&f.c0.a0, &f.c0.a1, &f.c0.a2, &f.c1.a0, &f.c1.a1, &f.c1.a2};
  for (int i = 0; i < 6; ++i) {
    st_canon(out + 8 * i, c[i]->c0);
    st_canon(out + 8 * i + 4, c[i]->c1);
  }
}
__device__ Fq12 load_f12_mont(const uint64_t* in) {  // raw Montgomery limbs (scratch)
  Fq12 f;
  Fq2* c[6] = {&f.c0.a0, &f.c0.a1, &f.c0.a2, &f.c1.a0, &f.c1.a1, &f.c1.a2};
  for (int i = 0; i < 6; ++i) {
    c[i]->c0 = u256_from_u64(in + 8 * i);
    c[i]->c1 = u256_from_u64(in + 8 * i + 4);
  }
  return f;
}
__device__ void store_f12_mont(uint64_t* out, const Fq12& f) {
  const Fq2* c[6] = {&f.c0.a0, &f.c0.a1, &f.c0.a2, &f.c1.a0, &f.c1.a1, &f.c1.a2};
  for (int i = 0; i < 6; ++i) {
    u256_to_u64(c[i]->c0, out + 8 * i);
    u256_to_u64(c[i]->c1, out + 8 * i + 4);
  }
}

// Miller value of pair i (Montgomery Fq12, 48 u64), identity inputs -> 1
__device__ Fq12 miller_of(const uint64_t* g1, const uint64_t* g2, size_t i, const PairingConsts& k) {
  const uint64_t* p = g1 + 8 * i;
  const uint64_t* q = g2 + 16 * i;
  if (all_zero(p, 8) || all_zero(q, 16)) return f12_one(k);
  G2A qa{{ld_mont(q), ld_mont(q + 4)}, {ld_mont(q + 8), ld_mont(q + 12)}};
  return miller_loop(ld_mont(p), ld_mont(p + 4), qa, k);
}

__global__ void __launch_bounds__(64) pairing_kernel(const uint64_t* g1, const uint64_t* g2, size_t n, uint64_t* out,
                                                     PairingConsts k) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  store_f12(out + 48 * i, final_exp(miller_of(g1, g2, i, k), k));
}

__global__ void __launch_bounds__(64) miller_kernel(const uint64_t* g1, const uint64_t* g2, size_t n, uint64_t* acc,
                                                    PairingConsts k) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  store_f12_mont(acc + 48 * i, miller_of(g1, g2, i, k));
}

// product of the n Miller values, final exponentiation, compare with 1
__global__ void pairing_check_final(const uint64_t* acc, size_t n, int* ok, PairingConsts k) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Fq12 f = load_f12_mont(acc);
  for (size_t i = 1; i < n; ++i) f = f12_mul(f, load_f12_mont(acc + 48 * i));
  const Fq12 e = final_exp(f, k);
  const Fq12 one = f12_one(k);
  const Fq2* a[6] = {&e.c0.a0, &e.c0.a1, &e.c0.a2, &e.c1.a0, &e.c1.a1, &e.c1.a2};
  const Fq2* b[6] = {&one.c0.a0, &one.c0.a1, &one.c0.a2, &one.c1.a0, &one.c1.a1, &one.c1.a2};
  bool eq = true;
  for (int i = 0; i < 6; ++i) eq = eq && f2_eq(*a[i], *b[i]);
  *ok = eq ? 1 : 0;
}

// ---------------------------------------------------------------- G2 scalar multiplication
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
  k.gx0 = Fq::to_mont(u256_from_u64(K_GX[0]));
  k.gx1 = Fq::to_mont(u256_from_u64(K_GX[1]));
  k.gy0 = Fq::to_mont(u256_from_u64(K_GY[0]));
  k.gy1 = Fq::to_mont(u256_from_u64(K_GY[1]));
  for (int i = 0; i < 6; ++i) k.frob2[i] = Fq::to_mont(u256_from_u64(K_FROB2[i]));
  k.one = Fq::to_mont(Fq::one_plain());
  k.xi_unused = u256_zero();
  for (int i = 0; i < 12; ++i) k.hard[i] = K_HARD[i];
  k.ate = K_ATE_LO;
  U256 p;
  for (int i = 0; i < 8; ++i) p.w[i] = Bn254FqParams::P[i];
  uint64_t pl[4];
  u256_to_u64(p, pl);
  pl[0] -= 2;  // q is odd and its low limb is > 2: no borrow
  for (int i = 0; i < 4; ++i) k.qm2[i] = pl[i];
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
  int rc = check_coords(g1, 2 * n);
  if (!rc) rc = check_coords(g2, 4 * n);
  if (rc) return rc;
  hipStream_t s = ctx->host_stream();
  if ((rc = ctx->io0.ensure(n * 64)) || (rc = ctx->io1.ensure(n * 128)) || (rc = ctx->io2.ensure(n * 384))) return rc;
  PBF_HIP(hipMemcpyAsync(ctx->io0.p, g1, n * 64, hipMemcpyHostToDevice, s));
  PBF_HIP(hipMemcpyAsync(ctx->io1.p, g2, n * 128, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(pairing_kernel, dim3((n + 63) / 64), dim3(64), 0, s, (const uint64_t*)ctx->io0.p,
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
  hipLaunchKernelGGL(pairing_kernel, dim3((n + 63) / 64), dim3(64), 0, pbf_ctx::pick(stream), d_g1, d_g2, n, d_out,
                     make_consts());
  PBF_HIP(hipGetLastError());
  return 0;
}

extern "C" int pbf_pairing_check_bn254(pbf_ctx* ctx, const uint64_t* g1, const uint64_t* g2, size_t n, int* ok) {
  if (!ctx || !ok || (n && (!g1 || !g2))) return fail(1, "null argument");
  *ok = 0;
  if (n == 0) {
    *ok = 1;  // empty product
    return 0;
  }
  int rc = check_coords(g1, 2 * n);
  if (!rc) rc = check_coords(g2, 4 * n);
  if (rc) return rc;
  hipStream_t s = ctx->host_stream();
  if ((rc = ctx->io0.ensure(n * 64)) || (rc = ctx->io1.ensure(n * 128)) || (rc = ctx->io2.ensure(n * 384 + 64)))
    return rc;
  PBF_HIP(hipMemcpyAsync(ctx->io0.p, g1, n * 64, hipMemcpyHostToDevice, s));
  PBF_HIP(hipMemcpyAsync(ctx->io1.p, g2, n * 128, hipMemcpyHostToDevice, s));
  const PairingConsts k = make_consts();
  uint64_t* acc = (uint64_t*)ctx->io2.p;
  int* d_ok = (int*)(acc + 48 * n);
  hipLaunchKernelGGL(miller_kernel, dim3((n + 63) / 64), dim3(64), 0, s, (const uint64_t*)ctx->io0.p,
                     (const uint64_t*)ctx->io1.p, n, acc, k);
  PBF_HIP(hipGetLastError());
  hipLaunchKernelGGL(pairing_check_final, dim3(1), dim3(64), 0, s, (const uint64_t*)acc, n, d_ok, k);
  PBF_HIP(hipGetLastError());
  PBF_HIP(hipMemcpyAsync(ok, d_ok, sizeof(int), hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  return 0;
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
