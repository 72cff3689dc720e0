// BN254 G1 (y^2 = x^3 + 3 over Fq, generator (1, 2) — the curve equation and
// generator of the reference's toy G1, src/pbh/g1.rs:34-36, over the real field).
//
// Coordinates inside kernels: XYZZ (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2), Fq elements in
// Montgomery form; ZZ = 0 is the identity. Formulas: EFD "xyzz" madd-2008-s,
// add-2008-s, dbl-2008-s-1, mdbl-2008-s-1 (a = 0). Every exceptional case (identity
// operand, P + P, P + (-P)) is handled, so results are exact group elements and the
// canonical affine output is bit-identical to any correct implementation.
// At the ABI an affine point is 8 x uint64_t (x, y canonical, little-endian limbs);
// (0, 0) encodes the identity (it is not on the curve).
#pragma once
#include "fp256.hpp"

namespace pbf {

struct Affine {
  U256 x, y;  // Montgomery inside kernels
};

struct Xyzz {
  U256 X, Y, ZZ, ZZZ;
};

__host__ __device__ __forceinline__ U256 u256_zero() {
  U256 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z.w[i] = 0;
  return z;
}

struct G1 {
  typedef Fq F;
  __host__ __device__ __forceinline__ static U256 one_m() { return F::to_mont(F::one_plain()); }
  __host__ __device__ __forceinline__ static Xyzz identity() {
    Xyzz r;
    r.X = one_m(); r.Y = one_m(); r.ZZ = u256_zero(); r.ZZZ = u256_zero();
    return r;
  }
  __host__ __device__ __forceinline__ static bool is_identity(const Xyzz& p) { return F::is_zero(p.ZZ); }
  __host__ __device__ __forceinline__ static Xyzz from_affine(const Affine& a) {
    Xyzz r;
    r.X = a.x; r.Y = a.y; r.ZZ = one_m(); r.ZZZ = one_m();
    return r;
  }
  __host__ __device__ __forceinline__ static U256 dbl_f(const U256& a) { return F::add(a, a); }

  // mdbl-2008-s-1: 2*(x, y) for an affine point (y != 0 on BN254 G1: no 2-torsion)
  __host__ __device__ __forceinline__ static Xyzz mdbl(const Affine& a) {
    const U256 U = dbl_f(a.y);
    const U256 V = F::mul(U, U);
    const U256 W = F::mul(U, V);
    const U256 S = F::mul(a.x, V);
    const U256 xx = F::mul(a.x, a.x);
    const U256 M = F::add(dbl_f(xx), xx);
    Xyzz r;
    r.X = F::sub(F::mul(M, M), dbl_f(S));
    r.Y = F::sub(F::mul(M, F::sub(S, r.X)), F::mul(W, a.y));
    r.ZZ = V;
    r.ZZZ = W;
    return r;
  }
  // dbl-2008-s-1
  __host__ __device__ __forceinline__ static Xyzz dbl(const Xyzz& p) {
    if (is_identity(p)) return p;
    const U256 U = dbl_f(p.Y);
    const U256 V = F::mul(U, U);
    const U256 W = F::mul(U, V);
    const U256 S = F::mul(p.X, V);
    const U256 xx = F::mul(p.X, p.X);
    const U256 M = F::add(dbl_f(xx), xx);
    Xyzz r;
    r.X = F::sub(F::mul(M, M), dbl_f(S));
    r.Y = F::sub(F::mul(M, F::sub(S, r.X)), F::mul(W, p.Y));
    r.ZZ = F::mul(V, p.ZZ);
    r.ZZZ = F::mul(W, p.ZZZ);
    return r;
  }
  // madd-2008-s: p + a (a affine, not the identity)
  __host__ __device__ __forceinline__ static Xyzz madd(const Xyzz& p, const Affine& a) {
    if (is_identity(p)) return from_affine(a);
    const U256 U2 = F::mul(a.x, p.ZZ);
    const U256 S2 = F::mul(a.y, p.ZZZ);
    const U256 P = F::sub(U2, p.X);
    const U256 R = F::sub(S2, p.Y);
    if (F::is_zero(P)) {
      if (F::is_zero(R)) return mdbl(a);
      return identity();
    }
    const U256 PP = F::mul(P, P);
    const U256 PPP = F::mul(P, PP);
    const U256 Q = F::mul(p.X, PP);
    Xyzz r;
    r.X = F::sub(F::sub(F::mul(R, R), PPP), dbl_f(Q));
    r.Y = F::sub(F::mul(R, F::sub(Q, r.X)), F::mul(p.Y, PPP));
    r.ZZ = F::mul(p.ZZ, PP);
    r.ZZZ = F::mul(p.ZZZ, PPP);
    return r;
  }
  // madd-2008-s with the single-chain product (Fq::mul_tp, identical results): the MSM
  // accumulation, which is VALU-issue-bound at four waves per SIMD
  __host__ __device__ __forceinline__ static U256 mul_tp(const U256& a, const U256& b) { return F::mul_tp(a, b); }
  __host__ __device__ __forceinline__ static Xyzz madd_tp(const Xyzz& p, const Affine& a) {
    if (is_identity(p)) return from_affine(a);
    const U256 U2 = mul_tp(a.x, p.ZZ);
    const U256 S2 = mul_tp(a.y, p.ZZZ);
    const U256 P = F::sub(U2, p.X);
    const U256 R = F::sub(S2, p.Y);
    if (F::is_zero(P)) {
      if (F::is_zero(R)) return mdbl(a);
      return identity();
    }
    const U256 PP = mul_tp(P, P);
    const U256 PPP = mul_tp(P, PP);
    const U256 Q = mul_tp(p.X, PP);
    Xyzz r;
    r.X = F::sub(F::sub(mul_tp(R, R), PPP), dbl_f(Q));
    r.Y = F::sub(mul_tp(R, F::sub(Q, r.X)), mul_tp(p.Y, PPP));
    r.ZZ = mul_tp(p.ZZ, PP);
    r.ZZZ = mul_tp(p.ZZZ, PPP);
    return r;
  }
  // add-2008-s: p + q
  __host__ __device__ __forceinline__ static Xyzz add(const Xyzz& p, const Xyzz& q) {
    if (is_identity(p)) return q;
    if (is_identity(q)) return p;
    const U256 U1 = F::mul(p.X, q.ZZ);
    const U256 U2 = F::mul(q.X, p.ZZ);
    const U256 S1 = F::mul(p.Y, q.ZZZ);
    const U256 S2 = F::mul(q.Y, p.ZZZ);
    const U256 P = F::sub(U2, U1);
    const U256 R = F::sub(S2, S1);
    if (F::is_zero(P)) {
      if (F::is_zero(R)) return dbl(p);
      return identity();
    }
    const U256 PP = F::mul(P, P);
    const U256 PPP = F::mul(P, PP);
    const U256 Q = F::mul(U1, PP);
    Xyzz r;
    r.X = F::sub(F::sub(F::mul(R, R), PPP), dbl_f(Q));
    r.Y = F::sub(F::mul(R, F::sub(Q, r.X)), F::mul(S1, PPP));
    r.ZZ = F::mul(F::mul(p.ZZ, q.ZZ), PP);
    r.ZZZ = F::mul(F::mul(p.ZZZ, q.ZZZ), PPP);
    return r;
  }
  // add / dbl for single-lane latency chains (the MSM's joins and reduction trees), with the
  // independent products of each step interleaved in one column scan (F::mulN / F::mul2,
  // bit-identical results): add-2008-s in 4 dependent product steps (4 + 4 + 3 + 3 products)
  // instead of 7 pairs, dbl-2008-s-1 in 4 (2 + 3 + 3 + 1). A lane's time on these chains is
  // its dependency latency, not its issue count (one wave per SIMD), so wider steps are
  // shorter chains. PBF_EC_PAIRS restores the round-2 pairing for A/B. The throughput
  // kernels keep add / dbl.
#if defined(PBF_EC_PAIRS)
  __host__ __device__ __forceinline__ static Xyzz dbl2(const Xyzz& p) {
    if (is_identity(p)) return p;
    const U256 U = dbl_f(p.Y);
    U256 V, xx, W, S, MM, ZZ3, WY, ZZZ3;
    F::mul2(U, U, p.X, p.X, &V, &xx);
    F::mul2(U, V, p.X, V, &W, &S);
    const U256 M = F::add(dbl_f(xx), xx);
    F::mul2(M, M, V, p.ZZ, &MM, &ZZ3);
    F::mul2(W, p.Y, W, p.ZZZ, &WY, &ZZZ3);
    Xyzz r;
    r.X = F::sub(MM, dbl_f(S));
    r.Y = F::sub(F::mul(M, F::sub(S, r.X)), WY);
    r.ZZ = ZZ3;
    r.ZZZ = ZZZ3;
    return r;
  }
  __host__ __device__ __forceinline__ static Xyzz add2(const Xyzz& p, const Xyzz& q) {
    if (is_identity(p)) return q;
    if (is_identity(q)) return p;
    U256 U1, U2, S1, S2;
    F::mul2(p.X, q.ZZ, q.X, p.ZZ, &U1, &U2);
    F::mul2(p.Y, q.ZZZ, q.Y, p.ZZZ, &S1, &S2);
    const U256 P = F::sub(U2, U1);
    const U256 R = F::sub(S2, S1);
    if (F::is_zero(P)) {
      if (F::is_zero(R)) return dbl2(p);
      return identity();
    }
    U256 PP, RR, PPP, Q, ZZ12, ZZZ12, S1P, Y3a;
    F::mul2(P, P, R, R, &PP, &RR);
    F::mul2(p.ZZ, q.ZZ, p.ZZZ, q.ZZZ, &ZZ12, &ZZZ12);
    F::mul2(P, PP, U1, PP, &PPP, &Q);
    Xyzz r;
    r.X = F::sub(F::sub(RR, PPP), dbl_f(Q));
    F::mul2(R, F::sub(Q, r.X), S1, PPP, &Y3a, &S1P);
    r.Y = F::sub(Y3a, S1P);
    F::mul2(ZZ12, PP, ZZZ12, PPP, &r.ZZ, &r.ZZZ);
    return r;
  }
#else
  __host__ __device__ __forceinline__ static Xyzz dbl2(const Xyzz& p) {
    if (is_identity(p)) return p;
    const U256 U = dbl_f(p.Y);
    U256 V, xx, W, S, ZZ3, MM, WY, ZZZ3;
    F::mul2(U, U, p.X, p.X, &V, &xx);
    {
      const U256* x[3] = {&U, &p.X, &V};
      const U256* y[3] = {&V, &V, &p.ZZ};
      U256* o[3] = {&W, &S, &ZZ3};
      F::template mulN<3>(x, y, o);
    }
    const U256 M = F::add(dbl_f(xx), xx);
    {
      const U256* x[3] = {&M, &W, &W};
      const U256* y[3] = {&M, &p.Y, &p.ZZZ};
      U256* o[3] = {&MM, &WY, &ZZZ3};
      F::template mulN<3>(x, y, o);
    }
    Xyzz r;
    r.X = F::sub(MM, dbl_f(S));
    r.Y = F::sub(F::mul(M, F::sub(S, r.X)), WY);
    r.ZZ = ZZ3;
    r.ZZZ = ZZZ3;
    return r;
  }
  __host__ __device__ __forceinline__ static Xyzz add2(const Xyzz& p, const Xyzz& q) {
    if (is_identity(p)) return q;
    if (is_identity(q)) return p;
    U256 U1, U2, S1, S2;
    {
      const U256* x[4] = {&p.X, &q.X, &p.Y, &q.Y};
      const U256* y[4] = {&q.ZZ, &p.ZZ, &q.ZZZ, &p.ZZZ};
      U256* o[4] = {&U1, &U2, &S1, &S2};
      F::template mulN<4>(x, y, o);
    }
    const U256 P = F::sub(U2, U1);
    const U256 R = F::sub(S2, S1);
    if (F::is_zero(P)) {
      if (F::is_zero(R)) return dbl2(p);
      return identity();
    }
    U256 PP, RR, ZZ12, ZZZ12, PPP, Q, ZZ3, Y3a, S1P, ZZZ3;
    {
      const U256* x[4] = {&P, &R, &p.ZZ, &p.ZZZ};
      const U256* y[4] = {&P, &R, &q.ZZ, &q.ZZZ};
      U256* o[4] = {&PP, &RR, &ZZ12, &ZZZ12};
      F::template mulN<4>(x, y, o);
    }
    {
      const U256* x[3] = {&P, &U1, &ZZ12};
      const U256* y[3] = {&PP, &PP, &PP};
      U256* o[3] = {&PPP, &Q, &ZZ3};
      F::template mulN<3>(x, y, o);
    }
    Xyzz r;
    r.X = F::sub(F::sub(RR, PPP), dbl_f(Q));
    const U256 QX = F::sub(Q, r.X);
    {
      const U256* x[3] = {&R, &S1, &ZZZ12};
      const U256* y[3] = {&QX, &PPP, &PPP};
      U256* o[3] = {&Y3a, &S1P, &ZZZ3};
      F::template mulN<3>(x, y, o);
    }
    r.Y = F::sub(Y3a, S1P);
    r.ZZ = ZZ3;
    r.ZZZ = ZZZ3;
    return r;
  }
#endif
  // k * p for a small non-negative k (double-and-add, MSB first)
  __host__ __device__ __forceinline__ static Xyzz mul_small(const Xyzz& p, uint32_t k) {
    Xyzz r = identity();
    int top = 31;
    while (top >= 0 && !((k >> top) & 1)) --top;  // from the leading one
    for (int b = top; b >= 0; --b) {
      r = dbl(r);
      if ((k >> b) & 1) r = add(r, p);
    }
    return r;
  }
  // a^(q-2) (Fermat), Montgomery in/out
  __host__ __device__ static U256 inv(const U256& a) {
    uint32_t e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = Bn254FqParams::P[i];
    e[0] -= 2;
    U256 r = one_m();
    for (int i = 255; i >= 0; --i) {
      r = F::mul(r, r);
      if ((e[i >> 5] >> (i & 31)) & 1) r = F::mul(r, a);
    }
    return r;
  }
  // canonical affine (plain form); identity -> (0, 0)
  __host__ __device__ static void to_affine_plain(const Xyzz& p, U256* x, U256* y) {
    if (is_identity(p)) { *x = u256_zero(); *y = u256_zero(); return; }
    // ZZ^3 = ZZZ^2, so 1/ZZ = ZZ^2 * (1/ZZZ)^2: one inversion
    const U256 izzz = inv(p.ZZZ);
    const U256 t = F::mul(p.ZZ, izzz);
    const U256 izz = F::mul(t, t);
    *x = F::from_mont(F::mul(p.X, izz));
    *y = F::from_mont(F::mul(p.Y, izzz));
  }
};

// ---- quad-lane point arithmetic for latency chains (the MSM's bucket-reduction tails) -----
// The four lanes of a quad (lanes 4i .. 4i+3) hold the same operands. Each dependent product
// step of add-2008-s / dbl-2008-s-1 (the 4 + 4 + 3 + 3 and 2 + 3 + 3 + 1 steps of add2 /
// dbl2) computes product i on lane i and broadcasts the results across the quad with DPP
// quad_perm moves (8 dwords per product), so a step costs one product of latency instead of
// three or four interleaved ones. The additions and subtractions run redundantly on all four
// lanes, and every branch depends only on quad-uniform values, so a quad never diverges. The
// results are bit-identical to add2 / dbl2 (same formulas, same products). Callers keep all
// four lanes of a quad active together.
struct G1Quad {
  typedef Fq F;
  template <int SRC>
  __device__ __forceinline__ static U256 bcast(const U256& v) {
    constexpr int ctrl = SRC | (SRC << 2) | (SRC << 4) | (SRC << 6);  // quad_perm [SRC x 4]
    U256 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.w[i], ctrl, 0xF, 0xF, false);
    return r;
  }
  // lane l's operand, branch-free: hipcc compiled the nested ternary into divergent branches
  // per limb (~2 k cycles per product round on one wave, as much as the product itself;
  // masks: 2.36 k cycles for select + product against 4.37 k, scripts/ubench/quad_lat.hip)
  __device__ __forceinline__ static U256 sel(uint32_t l, const U256& a, const U256& b, const U256& c, const U256& d) {
    const uint32_t m0 = 0u - (uint32_t)(l == 0), m1 = 0u - (uint32_t)(l == 1), m2 = 0u - (uint32_t)(l == 2),
                   m3 = 0u - (uint32_t)(l == 3);
    U256 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = (a.w[i] & m0) | (b.w[i] & m1) | (c.w[i] & m2) | (d.w[i] & m3);
    return r;
  }
  // out_i = x_i * y_i for i < N (N = 2, 3 or 4), product i on lane i of the quad
  template <int N>
  __device__ __forceinline__ static void mulN(const U256* const* x, const U256* const* y, U256* const* out) {
    const uint32_t l = threadIdx.x & 3;
    const U256 xs = sel(l, *x[0], *x[1], *x[N > 2 ? 2 : 1], *x[N > 3 ? 3 : N - 1]);
    const U256 ys = sel(l, *y[0], *y[1], *y[N > 2 ? 2 : 1], *y[N > 3 ? 3 : N - 1]);
    const U256 r = F::mul(xs, ys);
    *out[0] = bcast<0>(r);
    *out[1] = bcast<1>(r);
    if constexpr (N > 2) *out[2] = bcast<2>(r);
    if constexpr (N > 3) *out[3] = bcast<3>(r);
  }
  // dbl-2008-s-1 in three product rounds (round 5; four before, with M (S - X3) on one lane
  // after the third): M^2 joins the second round, M (S - X3) the third. Measured level on one
  // wave (13.3 k against 13.0 k cycles, profiles/r05/pairing_lat_g1*.log): the selects, DPP
  // broadcasts and reduced add / sub chains around the products, not the product rounds, set
  // a quad operation's latency
  __device__ __forceinline__ static Xyzz dbl(const Xyzz& p) {
    if (G1::is_identity(p)) return p;
    const U256 U = G1::dbl_f(p.Y);
    U256 V, xx, W, S, ZZ3, MM, MSX, WY, ZZZ3;
    {
      const U256* x[2] = {&U, &p.X};
      const U256* y[2] = {&U, &p.X};
      U256* o[2] = {&V, &xx};
      mulN<2>(x, y, o);
    }
    const U256 M = F::add(G1::dbl_f(xx), xx);
    {
      const U256* x[4] = {&U, &p.X, &V, &M};
      const U256* y[4] = {&V, &V, &p.ZZ, &M};
      U256* o[4] = {&W, &S, &ZZ3, &MM};
      mulN<4>(x, y, o);
    }
    Xyzz r;
    r.X = F::sub(MM, G1::dbl_f(S));
    const U256 SX = F::sub(S, r.X);
    {
      const U256* x[3] = {&M, &W, &W};
      const U256* y[3] = {&SX, &p.Y, &p.ZZZ};
      U256* o[3] = {&MSX, &WY, &ZZZ3};
      mulN<3>(x, y, o);
    }
    r.Y = F::sub(MSX, WY);
    r.ZZ = ZZ3;
    r.ZZZ = ZZZ3;
    return r;
  }
  __device__ __forceinline__ static Xyzz add(const Xyzz& p, const Xyzz& q) {
    if (G1::is_identity(p)) return q;
    if (G1::is_identity(q)) return p;
    U256 U1, U2, S1, S2;
    {
      const U256* x[4] = {&p.X, &q.X, &p.Y, &q.Y};
      const U256* y[4] = {&q.ZZ, &p.ZZ, &q.ZZZ, &p.ZZZ};
      U256* o[4] = {&U1, &U2, &S1, &S2};
      mulN<4>(x, y, o);
    }
    const U256 P = F::sub(U2, U1);
    const U256 R = F::sub(S2, S1);
    if (F::is_zero(P)) {
      if (F::is_zero(R)) return dbl(p);
      return G1::identity();
    }
    U256 PP, RR, ZZ12, ZZZ12, PPP, Q, ZZ3, Y3a, S1P, ZZZ3;
    {
      const U256* x[4] = {&P, &R, &p.ZZ, &p.ZZZ};
      const U256* y[4] = {&P, &R, &q.ZZ, &q.ZZZ};
      U256* o[4] = {&PP, &RR, &ZZ12, &ZZZ12};
      mulN<4>(x, y, o);
    }
    {
      const U256* x[3] = {&P, &U1, &ZZ12};
      const U256* y[3] = {&PP, &PP, &PP};
      U256* o[3] = {&PPP, &Q, &ZZ3};
      mulN<3>(x, y, o);
    }
    Xyzz r;
    r.X = F::sub(F::sub(RR, PPP), G1::dbl_f(Q));
    const U256 QX = F::sub(Q, r.X);
    {
      const U256* x[3] = {&R, &S1, &ZZZ12};
      const U256* y[3] = {&QX, &PPP, &PPP};
      U256* o[3] = {&Y3a, &S1P, &ZZZ3};
      mulN<3>(x, y, o);
    }
    r.Y = F::sub(Y3a, S1P);
    r.ZZ = ZZ3;
    r.ZZZ = ZZZ3;
    return r;
  }
};

}  // namespace pbf
