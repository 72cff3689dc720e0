// ORACLE — TEST INFRASTRUCTURE ONLY (see field.hpp header).
// Restates src/matrix.rs (interpolation), src/pbh/{g1,g2,gt,pairing,mod}.rs,
// src/constraints.rs and src/plonk.rs of the reference.
#pragma once
#include <array>
#include <stdexcept>
#include <vector>
#include "fft.hpp"

namespace oracle {

typedef Fe<StaticMod<101>> F101;
typedef Fe<StaticMod<17>> F17;
inline F101 f101(uint64_t x) { return F101::from_u64(x); }
inline F17 f17(uint64_t x) { return F17::from_u64(x); }

// ---------------------------------------------------------------- matrix.rs
// Row-major dense matrix; only what interpolate_at_h needs (matrix.rs:40-104, 130-155).
template <class F>
struct Matrix {
  size_t m, n;
  std::vector<F> v;
  Matrix(size_t m_, size_t n_) : m(m_), n(n_), v(m_ * n_, F::zero()) {}
  F& at(size_t r, size_t c) { return v[c + r * n]; }
  const F& at(size_t r, size_t c) const { return v[c + r * n]; }
  // matrix.rs:61-104 gauss_jordan_general (reduced row echelon form)
  void gauss_jordan() {
    size_t lead = 0;
    for (size_t r = 0; r < m; ++r) {
      if (n <= lead) break;
      size_t i = r;
      bool stop = false;
      while (at(i, lead) == F::zero()) {
        ++i;
        if (i == m) {
          i = r;
          ++lead;
          if (lead == n) { stop = true; break; }
        }
      }
      if (stop) break;
      for (size_t col = 0; col < n; ++col) std::swap(v[n * i + col], v[n * r + col]);
      if (at(r, lead) != F::zero()) {
        F d = at(r, lead);
        for (size_t j = 0; j < n; ++j) at(r, j) = at(r, j).div_unwrap(d);
      }
      for (size_t k = 0; k < m; ++k) {
        if (k != r) {
          F mult = at(k, lead);
          for (size_t j = 0; j < n; ++j) at(k, j) = at(k, j) - at(r, j) * mult;
        }
      }
      ++lead;
    }
  }
  // matrix.rs:40-59 inv via augmented [A | I]
  Matrix inv() const {
    size_t len = n;
    Matrix aug(len, len * 2);
    for (size_t i = 0; i < len; ++i) {
      for (size_t j = 0; j < len; ++j) aug.at(i, j) = at(i, j);
      aug.at(i, i + len) = F::one();
    }
    aug.gauss_jordan();
    Matrix u(len, len);
    for (size_t i = 0; i < len; ++i)
      for (size_t j = 0; j < len; ++j) u.at(i, j) = aug.at(i, j + len);
    return u;
  }
  // matrix.rs:147-155 Mul<Poly>: pad coeffs to m, M * column, then Poly::new.
  Poly<F> mul_poly(const Poly<F>& p) const {
    std::vector<F> col = p.c;
    col.resize(m, F::zero());
    std::vector<F> out(m, F::zero());
    for (size_t i = 0; i < m; ++i) {
      F acc = F::zero();
      for (size_t k = 0; k < n; ++k) acc = acc + at(i, k) * col[k];
      out[i] = acc;
    }
    return Poly<F>(out);
  }
};

// ---------------------------------------------------------------- pbh/g1.rs
// Affine point on y^2 = x^3 + 3 over F101 with an infinity flag (g1.rs:18-26).
struct G1P {
  F101 x, y;
  bool inf;
  static G1P make(F101 x, F101 y) { return G1P{x, y, false}; }
  static G1P generator() { return make(f101(1), f101(2)); }          // g1.rs:71-77
  static G1P identity() { return G1P{F101::zero(), F101::zero(), true}; }  // g1.rs:83-89
  static uint64_t subgroup_size() { return 17; }                     // g1.rs:79-81
  bool in_curve() const { return y.pow(2) == x.pow(3) + f101(3); }   // g1.rs:63-65
  bool operator==(const G1P& o) const { return x == o.x && y == o.y && inf == o.inf; }
  bool operator!=(const G1P& o) const { return !(*this == o); }
  G1P operator-() const { return inf ? *this : make(x, -y); }        // g1.rs:108-117
  // g1.rs:119-144 chord / tangent addition (a = 0 doubling formula).
  G1P operator+(const G1P& r) const {
    if (inf) return r;
    if (r.inf) return *this;
    if (*this == -r) return identity();
    if (*this == r) {
      F101 two = f101(2), three = f101(3);
      F101 m = (three * x.pow(2)).div_unwrap(two * y);
      return make(m * m - two * x, m * (three * x - m.pow(2)) - y);
    }
    F101 lambda = (r.y - y).div_unwrap(r.x - x);
    F101 nx = lambda.pow(2) - x - r.x;
    return make(nx, lambda * (x - nx) - y);
  }
  // g1.rs:146-168 LSB-first double-and-add over scalar.as_u64()
  G1P operator*(F101 s) const {
    uint64_t e = s.as_u64();
    if (e == 0 || inf) return identity();
    bool have = false;
    G1P res = identity(), base = *this;
    while (e > 0) {
      if (e & 1) { res = have ? res + base : base; have = true; }
      e >>= 1;
      base = base + base;
    }
    return res;
  }
};

// ---------------------------------------------------------------- pbh/g2.rs
// (a, b*u) with u^2 = -2 over F101 (g2.rs:14-36). No identity handling, as in the reference.
struct G2P {
  F101 a, b;
  static G2P generator() { return G2P{f101(36), f101(31)}; }
  bool operator==(const G2P& o) const { return a == o.a && b == o.b; }
  G2P operator-() const { return G2P{a, -b}; }
  // g2.rs:58-80
  G2P operator+(const G2P& r) const {
    if (*this == r) {
      F101 two = f101(2), three = f101(3);
      F101 m_u = (three * a.pow(2)).div_unwrap(two * b);
      F101 u2inv = (-f101(2)).inv_unwrap();
      F101 m2 = m_u.pow(2) * u2inv;
      return G2P{m2 - two * a, u2inv * m_u * (three * a - m2) - b};
    }
    F101 lu = (r.b - b).div_unwrap(r.a - a);
    F101 l2 = lu.pow(2) * (-f101(2));
    F101 na = l2 - a - r.a;
    return G2P{na, lu * (a - na) - b};
  }
  // g2.rs:82-101 (panics on 0 in the reference)
  G2P operator*(F101 s) const {
    uint64_t e = s.as_u64();
    if (e == 0) throw std::string("G2P * 0 (reference panics on unwrap)");
    bool have = false;
    G2P res = *this, base = *this;
    while (e > 0) {
      if (e & 1) { res = have ? res + base : base; have = true; }
      e >>= 1;
      base = base + base;
    }
    return res;
  }
};

// ---------------------------------------------------------------- pbh/gt.rs
// F101[u]/(u^2+2) (gt.rs:8-69).
struct GTP {
  F101 a, b;
  bool operator==(const GTP& o) const { return a == o.a && b == o.b; }
  GTP operator-() const { return GTP{a, -b}; }  // gt.rs:21-29 (conjugate = Frobenius)
  GTP operator*(const GTP& r) const {           // gt.rs:61-69
    return GTP{a * r.a - f101(2) * b * r.b, a * r.b + b * r.a};
  }
  // gt.rs:31-60: n >= 101 uses x^101 = conj(x), then square-and-multiply.
  GTP pow(uint64_t n) const {
    GTP p{F101::one(), F101::zero()}, base = *this;
    if (n >= 101) {
      p = -pow(n / 101);
      n %= 101;
    }
    while (n > 0) {
      if (n & 1) p = p * base;
      n >>= 1;
      base = base * base;
    }
    return p;
  }
};

// ---------------------------------------------------------------- pbh/pairing.rs
// pairing.rs:23-47 recursive Miller loop (no vertical-line denominators).
inline GTP pairing_f(uint64_t r, const G1P& p, const G2P& q) {
  auto line = [](const G1P& a, const G1P& b, F101& x, F101& y, F101& c) {
    F101 m = b.x - a.x, n = b.y - a.y;
    x = n; y = -m; c = m * a.y - n * a.x;
  };
  if (r == 1) return GTP{f101(1), f101(0)};
  F101 x, y, c;
  if (r % 2 == 1) {
    uint64_t r1 = r - 1;
    line(p * f101(r1), p, x, y, c);
    return pairing_f(r1, p, q) * GTP{q.a * x + c, q.b * y};
  }
  uint64_t r2 = r / 2;
  line(p * f101(r2), (-p) * f101(r2) * f101(2), x, y, c);
  return pairing_f(r2, p, q).pow(2) * GTP{q.a * x + c, q.b * y};
}

// pairing.rs:12-20 reduced Tate pairing, exponent (p^k - 1)/r = 600.
inline GTP pairing(const G1P& p, const G2P& q) {
  uint64_t pp = 101, r = G1P::subgroup_size(), k = 2;
  uint64_t e = (pp * pp - 1) / r;
  (void)k;
  return pairing_f(r, p, q).pow(e);
}

// ---------------------------------------------------------------- constraints.rs
enum CopyKind { COPY_A = 0, COPY_B = 1, COPY_C = 2 };
struct CopyOf { int kind; size_t idx; };  // constraints.rs:66-71 (1-based idx)

template <class F>
struct Constrains {  // constraints.rs:108-118
  std::vector<F> q_l, q_r, q_o, q_m, q_c;
  std::vector<CopyOf> c_a, c_b, c_c;
  // constraints.rs:198-230. Quirk kept: q_l * b instead of q_r * b (constraints.rs:203).
  bool satisfies(const std::vector<F>& a, const std::vector<F>& b, const std::vector<F>& c) const {
    for (size_t i = 0; i < a.size(); ++i) {
      F r = q_l[i] * a[i] + q_l[i] * b[i] + q_o[i] * c[i] + q_m[i] * a[i] * b[i] + q_c[i];
      if (r != F::zero()) return false;
    }
    auto val = [&](const CopyOf& co) -> F {
      return co.kind == COPY_A ? a[co.idx - 1] : co.kind == COPY_B ? b[co.idx - 1] : c[co.idx - 1];
    };
    for (size_t i = 0; i < c_a.size(); ++i)
      if (a[i] != val(c_a[i]) || b[i] != val(c_b[i]) || c[i] != val(c_c[i])) return false;
    return true;
  }
};

// ---------------------------------------------------------------- plonk.rs
// PlonkByHandTypes (pbh/mod.rs:18-33): HF=F17, GF=F101, K1=2, K2=3, OMEGA=4.
struct PBH {
  typedef F17 HF;
  typedef F101 GF;
  static HF K1() { return f17(2); }
  static HF K2() { return f17(3); }
  static HF OMEGA() { return f17(4); }
  static GF gf(HF v) { return F101::from_u64(v.as_u64()); }
};

struct Proof {  // plonk.rs:61-95
  G1P a_s, b_s, c_s, z_s, t_lo_s, t_mid_s, t_hi_s, w_z_s, w_z_omega_s;
  F17 a_z, b_z, c_z, s_sigma_1_z, s_sigma_2_z, r_z, z_omega_z;
};

struct Challange { F17 alpha, beta, gamma, z, v; };  // plonk.rs:97-108

struct SRS {  // plonk.rs:28-59
  std::vector<G1P> g1s;
  G2P g2_1, g2_s;
  static SRS create(F101 s, size_t n) {
    SRS r;
    F101 s_pow = s;
    r.g1s.push_back(G1P::generator());
    for (size_t i = 0; i < n; ++i) {
      r.g1s.push_back(G1P::generator() * s_pow);
      s_pow = s_pow * s;
    }
    r.g2_1 = G2P::generator();
    r.g2_s = G2P::generator() * s;
    return r;
  }
  // plonk.rs:51-58 naive MSM: left fold from identity of g1s[i] * gf(c_i)
  G1P eval_at_s(const Poly<F17>& p) const {
    G1P acc = G1P::identity();
    // g1s[n] panics in the reference when the polynomial is longer than the SRS
    for (size_t i = 0; i < p.c.size(); ++i) acc = acc + g1s.at(i) * PBH::gf(p.c[i]);
    return acc;
  }
};

struct Plonk {  // plonk.rs:110-175
  SRS srs;
  std::vector<F17> h, k1_h, k2_h;
  Matrix<F17> h_pows_inv{1, 1};
  Poly<F17> z_h_x;

  Plonk(const SRS& s, F17 omega_pows) : srs(s) {
    for (uint64_t i = 0; i < omega_pows.as_u64(); ++i) h.push_back(PBH::OMEGA().pow(i));
    for (auto& r : h) k1_h.push_back(r * PBH::K1());
    for (auto& r : h) k2_h.push_back(r * PBH::K2());
    Matrix<F17> hp(h.size(), h.size());
    for (size_t c = 0; c < h.size(); ++c)
      for (size_t r = 0; r < h.size(); ++r) hp.at(r, c) = h[r].pow(c);
    h_pows_inv = hp.inv();
    z_h_x = poly_z(h);
  }
  // plonk.rs:177-179 (== natural-order INTT)
  Poly<F17> interpolate_at_h(const std::vector<F17>& v) const { return h_pows_inv.mul_poly(Poly<F17>(v)); }
  std::vector<F17> copy_to_roots(const std::vector<CopyOf>& c) const {  // plonk.rs:181-189
    std::vector<F17> o;
    for (auto& x : c) o.push_back(x.kind == COPY_A ? h[x.idx - 1] : x.kind == COPY_B ? k1_h[x.idx - 1] : k2_h[x.idx - 1]);
    return o;
  }

  // plonk.rs:191-466
  Proof prove(const Constrains<F17>& cs, const std::vector<F17>& A, const std::vector<F17>& B,
              const std::vector<F17>& C, const Challange& ch, const std::array<F17, 9>& rnd) const {
    typedef F17 HF;
    typedef Poly<HF> P;
    if (!cs.satisfies(A, B, C)) throw std::string("constraints not satisfied");
    HF alpha = ch.alpha, beta = ch.beta, gamma = ch.gamma, z = ch.z, v = ch.v;
    HF omega = PBH::OMEGA(), k1 = PBH::K1(), k2 = PBH::K2();
    uint64_t n = cs.c_a.size();
    auto sigma_1 = copy_to_roots(cs.c_a), sigma_2 = copy_to_roots(cs.c_b), sigma_3 = copy_to_roots(cs.c_c);
    P f_a_x = interpolate_at_h(A), f_b_x = interpolate_at_h(B), f_c_x = interpolate_at_h(C);
    P q_o_x = interpolate_at_h(cs.q_o), q_m_x = interpolate_at_h(cs.q_m), q_l_x = interpolate_at_h(cs.q_l);
    P q_r_x = interpolate_at_h(cs.q_r), q_c_x = interpolate_at_h(cs.q_c);
    P s_sigma_1 = interpolate_at_h(sigma_1), s_sigma_2 = interpolate_at_h(sigma_2), s_sigma_3 = interpolate_at_h(sigma_3);

    // round 1 (plonk.rs:248-257)
    P a_x = P({rnd[1], rnd[0]}) * z_h_x + f_a_x;
    P b_x = P({rnd[3], rnd[2]}) * z_h_x + f_b_x;
    P c_x = P({rnd[5], rnd[4]}) * z_h_x + f_c_x;
    Proof pf;
    pf.a_s = srs.eval_at_s(a_x);
    pf.b_s = srs.eval_at_s(b_x);
    pf.c_s = srs.eval_at_s(c_x);

    // round 2 (plonk.rs:267-313)
    std::vector<HF> acc{HF::one()};
    for (size_t i = 1; i < n; ++i) {
      HF a = A[i - 1], b = B[i - 1], c = C[i - 1];
      HF wp = omega.pow(i - 1);
      HF dend = (a + beta * wp + gamma) * (b + beta * k1 * wp + gamma) * (c + beta * k2 * wp + gamma);
      HF dsor = (a + beta * s_sigma_1.eval(wp) + gamma) * (b + beta * s_sigma_2.eval(wp) + gamma) *
                (c + beta * s_sigma_3.eval(wp) + gamma);
      acc.push_back(acc[i - 1] * dend.div_unwrap(dsor));
    }
    P acc_x = interpolate_at_h(acc);
    if (acc_x.eval(omega.pow(n)) != HF::one()) throw std::string("accumulator check failed");  // plonk.rs:307
    P z_x = P({rnd[8], rnd[7], rnd[6]}) * z_h_x + acc_x;
    pf.z_s = srs.eval_at_s(z_x);

    // round 3 (plonk.rs:328-385)
    std::vector<HF> lv(h.size(), HF::zero());
    lv[0] = HF::one();
    P l_1_x = interpolate_at_h(lv);
    P p_i_x = P::zero();
    P a_x_b_x_q_m_x = (a_x * b_x) * q_m_x;
    P a_x_q_l_x = a_x * q_l_x;
    P b_x_q_r_x = b_x * q_r_x;
    P c_x_q_o_x = c_x * q_o_x;
    P alpha_a_x_beta_x_gamma = (a_x + P({gamma, beta})) * alpha;
    P b_x_beta_k1_x_gamma = b_x + P({gamma, beta * k1});
    P c_x_beta_k2_x_gamma = c_x + P({gamma, beta * k2});
    std::vector<HF> zo;
    for (size_t i = 0; i < z_x.c.size(); ++i) zo.push_back(z_x.c[i] * omega.pow(i));
    P z_omega_x(zo);
    P alpha_a_x_beta_s_sigma1_x_gamma = ((a_x + s_sigma_1 * beta) + gamma) * alpha;
    P b_x_beta_s_sigma2_x_gamma = (b_x + s_sigma_2 * beta) + gamma;
    P c_x_beta_s_sigma3_x_gamma = (c_x + s_sigma_3 * beta) + gamma;
    P alpha_2_z_x_1_l_1_x = ((z_x + P({-HF::one()})) * alpha.pow(2)) * l_1_x;

    P t_1 = a_x_b_x_q_m_x + a_x_q_l_x + b_x_q_r_x + c_x_q_o_x + p_i_x + q_c_x;
    P t_2 = alpha_a_x_beta_x_gamma * b_x_beta_k1_x_gamma * c_x_beta_k2_x_gamma * z_x;
    P t_3 = alpha_a_x_beta_s_sigma1_x_gamma * b_x_beta_s_sigma2_x_gamma * c_x_beta_s_sigma3_x_gamma * z_omega_x;
    P t_4 = alpha_2_z_x_1_l_1_x;
    P t_x, rem;
    poly_div(((t_1 + t_2) - t_3) + t_4, z_h_x, t_x, rem);
    if (!(rem == P::zero())) throw std::string("t(x) remainder != 0");  // plonk.rs:370
    // plonk.rs:376-378 split at fixed n+2 = 6 offsets (reference hard-codes n = 4)
    size_t s = n + 2;
    auto chunk = [&](size_t lo) {
      std::vector<HF> v;
      for (size_t i = lo; i < lo + s; ++i) v.push_back(i < t_x.c.size() ? t_x.c[i] : HF::zero());
      return P(v);
    };
    P t_hi_x = chunk(2 * s), t_mid_x = chunk(s), t_lo_x = chunk(0);
    pf.t_hi_s = srs.eval_at_s(t_hi_x);
    pf.t_mid_s = srs.eval_at_s(t_mid_x);
    pf.t_lo_s = srs.eval_at_s(t_lo_x);

    // round 4 (plonk.rs:393-422)
    HF a_z = a_x.eval(z), b_z = b_x.eval(z), c_z = c_x.eval(z);
    HF s_sigma_1_z = s_sigma_1.eval(z), s_sigma_2_z = s_sigma_2.eval(z);
    HF t_z = t_x.eval(z), z_omega_z = z_omega_x.eval(z);
    P r_1 = (q_m_x * a_z) * b_z + q_l_x * a_z + q_r_x * b_z + q_o_x * c_z + q_c_x;
    P r_2 = z_x * ((a_z + beta * z + gamma) * (b_z + beta * k1 * z + gamma) * (c_z + beta * k2 * z + gamma) * alpha);
    // plonk.rs:414-416: z(x) * (s_sigma_3 * beta * z_omega_z) * (...) with a + sign (quirk kept)
    P r_3 = (z_x * ((s_sigma_3 * beta) * z_omega_z)) *
            ((a_z + beta * s_sigma_1_z + gamma) * (b_z + beta * s_sigma_2_z + gamma) * alpha);
    P r_4 = (z_x * l_1_x.eval(z)) * alpha.pow(2);
    P r_x = r_1 + r_2 + r_3 + r_4;
    HF r_z = r_x.eval(z);

    // round 5 (plonk.rs:430-446)
    P w = (((t_lo_x + t_mid_x * z.pow(n + 2)) + t_hi_x * z.pow(2 * n + 4)) - t_z) + (r_x - r_z) * v +
          (a_x - a_z) * v.pow(2) + (b_x - b_z) * v.pow(3) + (c_x - c_z) * v.pow(4) +
          (s_sigma_1 - s_sigma_1_z) * v.pow(5) + (s_sigma_2 - s_sigma_2_z) * v.pow(6);
    P w_z_x, w_z_omega_x;
    poly_div(w, P({-z, HF::one()}), w_z_x, rem);
    if (!(rem == P::zero())) throw std::string("w_z remainder != 0");  // plonk.rs:438
    poly_div(z_x - z_omega_z, P({-z * omega, HF::one()}), w_z_omega_x, rem);
    if (!(rem == P::zero())) throw std::string("w_zw remainder != 0");  // plonk.rs:442
    pf.w_z_s = srs.eval_at_s(w_z_x);
    pf.w_z_omega_s = srs.eval_at_s(w_z_omega_x);
    pf.a_z = a_z; pf.b_z = b_z; pf.c_z = c_z;
    pf.s_sigma_1_z = s_sigma_1_z; pf.s_sigma_2_z = s_sigma_2_z;
    pf.r_z = r_z; pf.z_omega_z = z_omega_z;
    return pf;
  }

  // plonk.rs:468-650
  bool verify(const Constrains<F17>& cs, const Proof& pf, const Challange& ch, F17 u) const {
    typedef F17 HF;
    typedef Poly<HF> P;
    HF alpha = ch.alpha, beta = ch.beta, gamma = ch.gamma, z = ch.z, v = ch.v;
    HF omega = PBH::OMEGA(), k1 = PBH::K1(), k2 = PBH::K2();
    auto sigma_1 = copy_to_roots(cs.c_a), sigma_2 = copy_to_roots(cs.c_b), sigma_3 = copy_to_roots(cs.c_c);
    auto cm = [&](const std::vector<HF>& vv) { return srs.eval_at_s(interpolate_at_h(vv)); };
    G1P q_m_s = cm(cs.q_m), q_l_s = cm(cs.q_l), q_r_s = cm(cs.q_r), q_o_s = cm(cs.q_o), q_c_s = cm(cs.q_c);
    G1P sigma_1_s = cm(sigma_1), sigma_2_s = cm(sigma_2), sigma_3_s = cm(sigma_3);
    const G1P* pts[9] = {&pf.a_s, &pf.b_s, &pf.c_s, &pf.z_s, &pf.t_lo_s, &pf.t_mid_s, &pf.t_hi_s, &pf.w_z_s, &pf.w_z_omega_s};
    for (auto p : pts) if (!p->in_curve()) return false;
    const HF* fs[7] = {&pf.a_z, &pf.b_z, &pf.c_z, &pf.s_sigma_1_z, &pf.s_sigma_2_z, &pf.r_z, &pf.z_omega_z};
    for (auto f : fs) if (!f->in_field()) return false;
    HF z_h_z = z_h_x.eval(z);
    std::vector<HF> lv(h.size(), HF::zero());
    lv[0] = HF::one();
    HF l_1_z = interpolate_at_h(lv).eval(z);
    HF p_i_z = HF::zero();
    HF a1 = beta * pf.s_sigma_1_z + gamma + pf.a_z;
    HF b1 = beta * pf.s_sigma_2_z + gamma + pf.b_z;
    HF c1 = pf.c_z + gamma;
    HF l1a2 = l_1_z * alpha.pow(2);
    HF t_z = (pf.r_z + p_i_z - (a1 * b1 * c1 * pf.z_omega_z) - l1a2).div_unwrap(z_h_z);  // plonk.rs:575-580
    auto gf = PBH::gf;
    G1P d_1 = q_m_s * gf(pf.a_z * pf.b_z * v) + q_l_s * gf(pf.a_z * v) + q_r_s * gf(pf.b_z * v) +
              q_o_s * gf(pf.c_z * v) + q_c_s * gf(v);
    G1P d_2 = pf.z_s * gf((pf.a_z + beta * z + gamma) * (pf.b_z + beta * k1 * z + gamma) *
                              (pf.c_z + beta * k2 * z + gamma) * alpha * v +
                          l_1_z * alpha.pow(2) * v + u);
    G1P d_3 = sigma_3_s * gf((pf.a_z + beta * pf.s_sigma_1_z + gamma) * (pf.b_z + beta * pf.s_sigma_2_z + gamma) *
                             alpha * v * beta * pf.z_omega_z);
    G1P d_s = d_1 + d_2 + (-d_3);
    uint64_t n = cs.c_a.size();
    G1P f_s = pf.t_lo_s + pf.t_mid_s * gf(z.pow(n + 2)) + pf.t_hi_s * gf(z.pow(2 * n + 4)) + d_s +
              pf.a_s * gf(v.pow(2)) + pf.b_s * gf(v.pow(3)) + pf.c_s * gf(v.pow(4)) +
              sigma_1_s * gf(v.pow(5)) + sigma_2_s * gf(v.pow(6));
    G1P e_s = srs.eval_at_s(P::from_i64({1})) *
              gf(t_z + v * pf.r_z + v.pow(2) * pf.a_z + v.pow(3) * pf.b_z + v.pow(4) * pf.c_z +
                 v.pow(5) * pf.s_sigma_1_z + v.pow(6) * pf.s_sigma_2_z + u * pf.z_omega_z);
    G1P e_1_q1 = pf.w_z_s + pf.w_z_omega_s * gf(u);
    G1P e_2_q1 = pf.w_z_s * gf(z) + pf.w_z_omega_s * gf(u * z * omega) + f_s + (-e_s);
    GTP e_1 = pairing(e_1_q1, srs.g2_s);
    GTP e_2 = pairing(e_2_q1, srs.g2_1);
    return e_1 == e_2;
  }
};

}  // namespace oracle
