// ORACLE — TEST INFRASTRUCTURE ONLY (see field.hpp header).
// Flat C entry points over the restatement, loaded by tests/ and bench.py's
// cpu_baseline leg through ctypes. Never linked into libpbf.so.
#include <cstring>
#include <string>
#include "pbh.hpp"

using namespace oracle;

namespace {
struct ModGuard {
  explicit ModGuard(uint64_t m) { DynMod::ref() = m; }
};
std::vector<DF> to_vec(const uint64_t* p, size_t n) {
  std::vector<DF> v(n);
  for (size_t i = 0; i < n; ++i) v[i] = DF::raw(p[i]);
  return v;
}
void from_vec(const std::vector<DF>& v, uint64_t* out) {
  for (size_t i = 0; i < v.size(); ++i) out[i] = v[i].v;
}
bool canonical(const uint64_t* p, size_t n, uint64_t M) {
  for (size_t i = 0; i < n; ++i) if (p[i] >= M) return false;
  return true;
}
}  // namespace

extern "C" {

// -------- field (u64field.rs)
uint64_t oracle_f_add(uint64_t M, uint64_t a, uint64_t b) { ModGuard g(M); return (DF::raw(a) + DF::raw(b)).v; }
uint64_t oracle_f_sub(uint64_t M, uint64_t a, uint64_t b) { ModGuard g(M); return (DF::raw(a) - DF::raw(b)).v; }
uint64_t oracle_f_mul(uint64_t M, uint64_t a, uint64_t b) { ModGuard g(M); return (DF::raw(a) * DF::raw(b)).v; }
uint64_t oracle_f_neg(uint64_t M, uint64_t a) { ModGuard g(M); return (-DF::raw(a)).v; }
uint64_t oracle_f_pow(uint64_t M, uint64_t a, uint64_t e) { ModGuard g(M); return DF::raw(a).pow(e).v; }
uint64_t oracle_f_from_i64(uint64_t M, int64_t a) { ModGuard g(M); return DF::from_i64(a).v; }
int oracle_f_inv(uint64_t M, uint64_t a, uint64_t* out) {
  ModGuard g(M);
  bool ok;
  DF r = DF::raw(a).inv(ok);
  *out = r.v;
  return ok ? 1 : 0;
}

// -------- fft.rs. Return 0 ok, 1 bad args, 2 n^-1 does not exist.
// Recursion-faithful CooleyTurkey (fft.rs:55-106); inverse per fft.rs:71-78.
int oracle_ntt_ct(uint64_t M, uint64_t omega, const uint64_t* in, uint64_t* out, size_t n, int inverse) {
  if (n == 0 || (n & (n - 1)) || !canonical(in, n, M)) return 1;
  ModGuard g(M);
  std::vector<DF> pows = ct_domain(DF::raw(omega), n);
  std::vector<DF> v = to_vec(in, n);
  if (!inverse) { from_vec(ct_fft(pows, v), out); return 0; }
  bool ok;
  std::vector<DF> r = ct_fft_inv(pows, v, ok);
  if (!ok) return 2;
  from_vec(r, out);
  return 0;
}

// Vandermonde variant (fft.rs:27-49), O(n^2): small n only.
int oracle_ntt_vandermonde(uint64_t M, uint64_t omega, const uint64_t* in, uint64_t* out, size_t n, int inverse) {
  if (n == 0 || !canonical(in, n, M)) return 1;
  ModGuard g(M);
  std::vector<DF> v = vandermonde_fft(DF::raw(omega), to_vec(in, n));
  if (!inverse) { from_vec(v, out); return 0; }
  bool ok;
  DF ninv = DF::from_u64(n).inv(ok);
  if (!ok) return 2;
  out[0] = (ninv * v[0]).v;
  for (size_t i = 1; i < n; ++i) out[i] = (ninv * v[n - i]).v;
  return 0;
}

// Iterative radix-2 NTT: fast checker (not the reference algorithm).
int oracle_ntt_iter(uint64_t M, uint64_t omega, const uint64_t* in, uint64_t* out, size_t n, int inverse) {
  if (n == 0 || (n & (n - 1)) || !canonical(in, n, M)) return 1;
  ModGuard g(M);
  std::vector<DF> v = to_vec(in, n);
  DF w = DF::raw(omega);
  DF ninv = DF::one();
  if (inverse) {
    bool ok;
    w = w.inv(ok);
    if (!ok) return 1;
    ninv = DF::from_u64(n).inv(ok);
    if (!ok) return 2;
  }
  iter_ntt(v, w);
  if (inverse) for (auto& x : v) x = x * ninv;
  from_vec(v, out);
  return 0;
}

// fft.rs:109-132 mul_ntt; out has la+lb entries (un-normalised). Domain size = la+lb.
int oracle_mul_ntt(uint64_t M, uint64_t omega, const uint64_t* a, size_t la, const uint64_t* b, size_t lb,
                   uint64_t* out) {
  size_t n = la + lb;
  if (n == 0 || (n & (n - 1))) return 1;
  ModGuard g(M);
  bool ok;
  std::vector<DF> pows = ct_domain(DF::raw(omega), n);
  std::vector<DF> r = mul_ntt(pows, to_vec(a, la), to_vec(b, lb), ok);
  if (!ok) return 2;
  from_vec(r, out);
  return 0;
}

// -------- poly.rs. Lengths in/out are coefficient counts after normalisation.
size_t oracle_poly_mul(uint64_t M, const uint64_t* a, size_t la, const uint64_t* b, size_t lb, uint64_t* out) {
  ModGuard g(M);
  Poly<DF> p = Poly<DF>(to_vec(a, la)) * Poly<DF>(to_vec(b, lb));
  from_vec(p.c, out);
  return p.c.size();
}
uint64_t oracle_poly_eval(uint64_t M, const uint64_t* c, size_t n, uint64_t x) {
  ModGuard g(M);
  return Poly<DF>(to_vec(c, n)).eval(DF::raw(x)).v;
}
int oracle_poly_div(uint64_t M, const uint64_t* num, size_t ln, const uint64_t* den, size_t ld, uint64_t* q,
                    size_t* lq, uint64_t* r, size_t* lr) {
  ModGuard g(M);
  try {
    Poly<DF> Q, R;
    poly_div(Poly<DF>(to_vec(num, ln)), Poly<DF>(to_vec(den, ld)), Q, R);
    from_vec(Q.c, q); *lq = Q.c.size();
    from_vec(R.c, r); *lr = R.c.size();
  } catch (...) { return 1; }
  return 0;
}

// -------- toy curve (pbh/g1.rs, g2.rs, gt.rs, pairing.rs). Points as [x, y, inf].
static G1P g1_in(const uint64_t* p) { return G1P{f101(p[0]), f101(p[1]), p[2] != 0}; }
static void g1_out(const G1P& p, uint64_t* o) { o[0] = p.x.v; o[1] = p.y.v; o[2] = p.inf ? 1 : 0; }
int oracle_g1_add(const uint64_t* a, const uint64_t* b, uint64_t* out) {
  try { g1_out(g1_in(a) + g1_in(b), out); } catch (...) { return 1; }
  return 0;
}
int oracle_g1_mul(const uint64_t* a, uint64_t s, uint64_t* out) {
  try { g1_out(g1_in(a) * f101(s), out); } catch (...) { return 1; }
  return 0;
}
int oracle_g1_neg(const uint64_t* a, uint64_t* out) { g1_out(-g1_in(a), out); return 0; }
int oracle_g1_in_curve(const uint64_t* a) { return g1_in(a).in_curve() ? 1 : 0; }
int oracle_g2_add(const uint64_t* a, const uint64_t* b, uint64_t* out) {
  try {
    G2P r = G2P{f101(a[0]), f101(a[1])} + G2P{f101(b[0]), f101(b[1])};
    out[0] = r.a.v; out[1] = r.b.v;
  } catch (...) { return 1; }
  return 0;
}
int oracle_g2_mul(const uint64_t* a, uint64_t s, uint64_t* out) {
  try {
    G2P r = G2P{f101(a[0]), f101(a[1])} * f101(s);
    out[0] = r.a.v; out[1] = r.b.v;
  } catch (...) { return 1; }
  return 0;
}
void oracle_gt_mul(const uint64_t* a, const uint64_t* b, uint64_t* out) {
  GTP r = GTP{f101(a[0]), f101(a[1])} * GTP{f101(b[0]), f101(b[1])};
  out[0] = r.a.v; out[1] = r.b.v;
}
void oracle_gt_pow(const uint64_t* a, uint64_t e, uint64_t* out) {
  GTP r = GTP{f101(a[0]), f101(a[1])}.pow(e);
  out[0] = r.a.v; out[1] = r.b.v;
}
int oracle_pairing(const uint64_t* g1, const uint64_t* g2, uint64_t* out) {
  try {
    GTP r = pairing(g1_in(g1), G2P{f101(g2[0]), f101(g2[1])});
    out[0] = r.a.v; out[1] = r.b.v;
  } catch (...) { return 1; }
  return 0;
}

// -------- plonk.rs over PlonkByHandTypes.
// gates: n x [q_l, q_r, q_o, q_m, q_c] (already reduced mod 17)
// copies: 3 x n x [kind(0=A,1=B,2=C), idx(1-based)]
// abc: 3 x n witness; chal: [alpha, beta, gamma, z, v]; rnd: 9 blinders; s: toxic waste in F101.
// out_pts: 9 x [x, y, inf] ; out_f: 7 field values. Returns 0 ok, 1 error; *verified set when verify_u < 17.
int oracle_pbh_prove(size_t n, const uint64_t* gates, const uint64_t* copies, const uint64_t* abc,
                     const uint64_t* chal, const uint64_t* rnd, uint64_t s, uint64_t srs_n, uint64_t omega_pows,
                     uint64_t verify_u, uint64_t* out_pts, uint64_t* out_f, int* verified) {
  try {
    SRS srs = SRS::create(f101(s), srs_n);
    Plonk pk(srs, f17(omega_pows));
    Constrains<F17> cs;
    for (size_t i = 0; i < n; ++i) {
      cs.q_l.push_back(f17(gates[5 * i + 0]));
      cs.q_r.push_back(f17(gates[5 * i + 1]));
      cs.q_o.push_back(f17(gates[5 * i + 2]));
      cs.q_m.push_back(f17(gates[5 * i + 3]));
      cs.q_c.push_back(f17(gates[5 * i + 4]));
    }
    std::vector<CopyOf>* cols[3] = {&cs.c_a, &cs.c_b, &cs.c_c};
    for (int c = 0; c < 3; ++c)
      for (size_t i = 0; i < n; ++i)
        cols[c]->push_back(CopyOf{(int)copies[(c * n + i) * 2], (size_t)copies[(c * n + i) * 2 + 1]});
    std::vector<F17> A, B, C;
    for (size_t i = 0; i < n; ++i) {
      A.push_back(f17(abc[i]));
      B.push_back(f17(abc[n + i]));
      C.push_back(f17(abc[2 * n + i]));
    }
    Challange ch{f17(chal[0]), f17(chal[1]), f17(chal[2]), f17(chal[3]), f17(chal[4])};
    std::array<F17, 9> r;
    for (int i = 0; i < 9; ++i) r[i] = f17(rnd[i]);
    Proof pf = pk.prove(cs, A, B, C, ch, r);
    const G1P* pts[9] = {&pf.a_s, &pf.b_s, &pf.c_s, &pf.z_s, &pf.t_lo_s, &pf.t_mid_s, &pf.t_hi_s, &pf.w_z_s, &pf.w_z_omega_s};
    for (int i = 0; i < 9; ++i) g1_out(*pts[i], out_pts + 3 * i);
    const F17* fs[7] = {&pf.a_z, &pf.b_z, &pf.c_z, &pf.s_sigma_1_z, &pf.s_sigma_2_z, &pf.r_z, &pf.z_omega_z};
    for (int i = 0; i < 7; ++i) out_f[i] = fs[i]->v;
    if (verified) *verified = (verify_u < 17) ? (pk.verify(cs, pf, ch, f17(verify_u)) ? 1 : 0) : -1;
  } catch (...) { return 1; }
  return 0;
}

}  // extern "C"
