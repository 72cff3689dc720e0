// ORACLE / CPU BASELINE — TEST INFRASTRUCTURE ONLY (see field.hpp header). Never linked
// into libpbf.so; only tests/ and bench.py's cpu_baseline leg load it (liboracle.so).
//
// C++ restatements of the reference's config-3 and config-4 paths over BN254, the CPU
// baselines BASELINE.md rows 3-4 name (the reference has no 256-bit field; these are its
// algorithms instantiated for the field SURVEY.md §0.5 picks):
//   * mul_ntt (src/fft.rs:109-132) over Fr with the recursion-faithful CooleyTurkey of
//     fft.rs:55-106 (even/odd split into fresh vectors at every level, x + y w / x - y w
//     combine, fft_inv = fft then reverse and scale by n^-1, fft.rs:71-78), one core;
//   * SRS::eval_at_s (src/plonk.rs:51-58): the naive left fold acc + g1s[i] * c_i, every
//     product an affine double-and-add (the G1P arithmetic of src/pbh/g1.rs:108-168:
//     affine chord / tangent formulas, one field inversion per step), one core;
//   * the same sum by an all-core Pippenger (16-bit windows, one window per thread, XYZZ
//     buckets, running-sum reduction, Horner over windows): what a tuned CPU library does.
// Field elements: 4 x u64 little-endian, Montgomery form inside (R = 2^256), canonical at
// the C boundary. G1 points: affine (x, y), (0, 0) = identity, as on the GPU.
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <thread>
#include <vector>

namespace {
typedef unsigned __int128 u128;

struct F4 {
  uint64_t v[4];
};

struct Field {
  uint64_t p[4];
  uint64_t inv;  // -p^-1 mod 2^64
  F4 r2;         // R^2 mod p
  F4 one;        // R mod p
};

inline bool geq(const uint64_t* a, const uint64_t* b) {
  for (int i = 3; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return true;
}
inline void sub_raw(uint64_t* a, const uint64_t* b) {  // a -= b (no underflow expected)
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    const u128 d = (u128)a[i] - b[i] - br;
    a[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
}

inline F4 fadd(const Field& f, const F4& a, const F4& b) {
  F4 r;
  uint64_t c = 0;
  for (int i = 0; i < 4; ++i) {
    const u128 s = (u128)a.v[i] + b.v[i] + c;
    r.v[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (c || geq(r.v, f.p)) sub_raw(r.v, f.p);
  return r;
}
inline F4 fsub(const Field& f, const F4& a, const F4& b) {
  F4 r;
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    const u128 d = (u128)a.v[i] - b.v[i] - br;
    r.v[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 4; ++i) {
      const u128 s = (u128)r.v[i] + f.p[i] + c;
      r.v[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  return r;
}
// CIOS Montgomery product a b R^-1
inline F4 fmul(const Field& f, const F4& a, const F4& b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < 4; ++j) {
      const u128 x = (u128)a.v[j] * b.v[i] + t[j] + c;
      t[j] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    u128 s = (u128)t[4] + c;
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    const uint64_t m = t[0] * f.inv;
    u128 x = (u128)m * f.p[0] + t[0];
    c = (uint64_t)(x >> 64);
    for (int j = 1; j < 4; ++j) {
      x = (u128)m * f.p[j] + t[j] + c;
      t[j - 1] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    s = (u128)t[4] + c;
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  F4 r;
  memcpy(r.v, t, 32);
  if (t[4] || geq(r.v, f.p)) sub_raw(r.v, f.p);
  return r;
}
inline bool fzero(const F4& a) { return !(a.v[0] | a.v[1] | a.v[2] | a.v[3]); }
inline bool feq(const F4& a, const F4& b) { return !memcmp(a.v, b.v, 32); }

Field make_field(const uint64_t* p) {
  Field f;
  memcpy(f.p, p, 32);
  uint64_t inv = 1;  // Newton: inv = p^-1 mod 2^64
  for (int i = 0; i < 6; ++i) inv *= 2 - p[0] * inv;
  f.inv = 0 - inv;
  // R mod p and R^2 mod p by doubling 1 (mod p) 256 / 512 times
  F4 x{{1, 0, 0, 0}};
  for (int i = 0; i < 512; ++i) {
    x = fadd(f, x, x);  // canonical arithmetic: fadd reduces
    if (i == 255) f.one = x;
  }
  f.r2 = x;
  return f;
}
inline F4 to_m(const Field& f, const F4& a) { return fmul(f, a, f.r2); }
inline F4 from_m(const Field& f, const F4& a) {
  F4 one{{1, 0, 0, 0}};
  return fmul(f, a, one);
}
F4 fpow(const Field& f, F4 a, const uint64_t* e) {  // a in Montgomery form
  F4 r = f.one;
  for (int i = 3; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      r = fmul(f, r, r);
      if ((e[i] >> b) & 1) r = fmul(f, r, a);
    }
  return r;
}
F4 finv(const Field& f, const F4& a) {  // Fermat, a^(p-2)
  uint64_t e[4];
  memcpy(e, f.p, 32);
  e[0] -= 2;
  return fpow(f, a, e);
}

const uint64_t R_MOD[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull};
const uint64_t Q_MOD[4] = {0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull};

const Field& fr() {
  static const Field f = make_field(R_MOD);
  return f;
}
const Field& fq() {
  static const Field f = make_field(Q_MOD);
  return f;
}

// ---------------------------------------------------------------- fft.rs restatement
void ct_fft(const std::vector<const F4*>& vals, const std::vector<const F4*>& dom, std::vector<F4>& out) {
  const Field& f = fr();
  const size_t n = vals.size();
  if (n == 1) {
    out.assign(1, *vals[0]);
    return;
  }
  std::vector<const F4*> half, ev, od;  // split(domain, true), split(vals, true / false)
  half.reserve(n / 2);
  ev.reserve(n / 2);
  od.reserve(n / 2);
  for (size_t i = 0; i < n; i += 2) half.push_back(dom[i]);
  for (size_t i = 0; i < n; ++i) (i % 2 == 0 ? ev : od).push_back(vals[i]);
  std::vector<F4> l, r;
  ct_fft(ev, half, l);
  ct_fft(od, half, r);
  out.assign(n, F4{{0, 0, 0, 0}});
  for (size_t i = 0; i < n / 2; ++i) {
    const F4 y = fmul(f, r[i], *dom[i]);
    out[i] = fadd(f, l[i], y);
    out[i + n / 2] = fsub(f, l[i], y);
  }
}
std::vector<F4> fft(const std::vector<F4>& pows, const std::vector<F4>& v) {
  std::vector<const F4*> pv(v.size()), dv(pows.size());
  for (size_t i = 0; i < v.size(); ++i) pv[i] = &v[i];
  for (size_t i = 0; i < pows.size(); ++i) dv[i] = &pows[i];
  std::vector<F4> out;
  ct_fft(pv, dv, out);
  return out;
}
}  // namespace

extern "C" {

// mul_ntt (fft.rs:109-132) over BN254 Fr: a (la) and b (lb) canonical 4 x u64, omega of order
// la + lb (a power of two, canonical); out: la + lb canonical elements. Returns 0 / 1 (bad n).
int oracle_fr_mul_ntt(const uint64_t* a, size_t la, const uint64_t* b, size_t lb, const uint64_t* omega,
                      uint64_t* out) {
  const size_t n = la + lb;
  if (n == 0 || (n & (n - 1))) return 1;
  const Field& f = fr();
  std::vector<F4> av(n, F4{{0, 0, 0, 0}}), bv(n, F4{{0, 0, 0, 0}});
  for (size_t i = 0; i < la; ++i) av[i] = to_m(f, *(const F4*)(a + 4 * i));
  for (size_t i = 0; i < lb; ++i) bv[i] = to_m(f, *(const F4*)(b + 4 * i));
  // CooleyTurkey::new (fft.rs:55-65): pows = omega^i, i < n
  std::vector<F4> pows(n);
  const F4 w = to_m(f, *(const F4*)omega);
  pows[0] = f.one;
  for (size_t i = 1; i < n; ++i) pows[i] = fmul(f, pows[i - 1], w);
  const std::vector<F4> af = fft(pows, av), bf = fft(pows, bv);
  std::vector<F4> cf(n);
  for (size_t i = 0; i < n; ++i) cf[i] = fmul(f, af[i], bf[i]);
  // fft_inv (fft.rs:71-78): vals = fft(freq); [vals[0], vals[n-1], ..., vals[1]] * n^-1
  const std::vector<F4> vals = fft(pows, cf);
  F4 nn{{(uint64_t)n, 0, 0, 0}};
  const F4 ninv = finv(f, to_m(f, nn));
  for (size_t i = 0; i < n; ++i) {
    const F4 r = from_m(f, fmul(f, vals[i == 0 ? 0 : n - i], ninv));
    memcpy(out + 4 * i, r.v, 32);
  }
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------- G1 over Fq
namespace {
struct Aff {
  F4 x, y;
  bool inf;
};
// affine addition, chord / tangent (src/pbh/g1.rs:108-144 for y^2 = x^3 + 3)
Aff aff_add(const Aff& p, const Aff& q) {
  const Field& f = fq();
  if (p.inf) return q;
  if (q.inf) return p;
  F4 lam;
  if (feq(p.x, q.x)) {
    if (!feq(p.y, q.y) || fzero(p.y)) return Aff{{}, {}, true};  // p == -q
    const F4 x2 = fmul(f, p.x, p.x);
    const F4 num = fadd(f, fadd(f, x2, x2), x2);  // 3 x^2
    lam = fmul(f, num, finv(f, fadd(f, p.y, p.y)));
  } else {
    lam = fmul(f, fsub(f, q.y, p.y), finv(f, fsub(f, q.x, p.x)));
  }
  Aff r;
  r.inf = false;
  r.x = fsub(f, fsub(f, fmul(f, lam, lam), p.x), q.x);
  r.y = fsub(f, fmul(f, lam, fsub(f, p.x, r.x)), p.y);
  return r;
}
// double-and-add, most significant bit first (g1.rs:146-168)
Aff aff_mul(const Aff& p, const uint64_t* s) {
  Aff acc{{}, {}, true};
  for (int i = 3; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      acc = aff_add(acc, acc);
      if ((s[i] >> b) & 1) acc = aff_add(acc, p);
    }
  return acc;
}

struct Xyzz {
  F4 X, Y, ZZ, ZZZ;
};
inline bool xyzz_inf(const Xyzz& p) { return fzero(p.ZZ); }
// madd-2008-s (mixed XYZZ + affine)
Xyzz xyzz_madd(const Xyzz& p, const Aff& q) {
  const Field& f = fq();
  if (q.inf) return p;
  if (xyzz_inf(p)) return Xyzz{q.x, q.y, fq().one, fq().one};
  const F4 U2 = fmul(f, q.x, p.ZZ), S2 = fmul(f, q.y, p.ZZZ);
  const F4 P = fsub(f, U2, p.X), R = fsub(f, S2, p.Y);
  if (fzero(P)) {
    if (!fzero(R)) return Xyzz{{}, {}, {}, {}};
    // doubling of q (mdbl-2008-s-1)
    const F4 U = fadd(f, q.y, q.y), V = fmul(f, U, U), W = fmul(f, U, V), S = fmul(f, q.x, V);
    const F4 x2 = fmul(f, q.x, q.x), M = fadd(f, fadd(f, x2, x2), x2);
    Xyzz r;
    r.X = fsub(f, fsub(f, fmul(f, M, M), S), S);
    r.Y = fsub(f, fmul(f, M, fsub(f, S, r.X)), fmul(f, W, q.y));
    r.ZZ = V;
    r.ZZZ = W;
    return r;
  }
  const F4 PP = fmul(f, P, P), PPP = fmul(f, P, PP), Q = fmul(f, p.X, PP);
  Xyzz r;
  r.X = fsub(f, fsub(f, fsub(f, fmul(f, R, R), PPP), Q), Q);
  r.Y = fsub(f, fmul(f, R, fsub(f, Q, r.X)), fmul(f, p.Y, PPP));
  r.ZZ = fmul(f, p.ZZ, PP);
  r.ZZZ = fmul(f, p.ZZZ, PPP);
  return r;
}
// general XYZZ addition (add-2008-s)
Xyzz xyzz_add(const Xyzz& p, const Xyzz& q) {
  const Field& f = fq();
  if (xyzz_inf(p)) return q;
  if (xyzz_inf(q)) return p;
  const F4 U1 = fmul(f, p.X, q.ZZ), U2 = fmul(f, q.X, p.ZZ);
  const F4 S1 = fmul(f, p.Y, q.ZZZ), S2 = fmul(f, q.Y, p.ZZZ);
  const F4 P = fsub(f, U2, U1), R = fsub(f, S2, S1);
  if (fzero(P)) {
    if (!fzero(R)) return Xyzz{{}, {}, {}, {}};
    // doubling (dbl-2008-s-1)
    const F4 U = fadd(f, p.Y, p.Y), V = fmul(f, U, U), W = fmul(f, U, V), S = fmul(f, p.X, V);
    const F4 x2 = fmul(f, p.X, p.X), M = fadd(f, fadd(f, x2, x2), x2);  // a = 0
    Xyzz r;
    r.X = fsub(f, fsub(f, fmul(f, M, M), S), S);
    r.Y = fsub(f, fmul(f, M, fsub(f, S, r.X)), fmul(f, W, p.Y));
    r.ZZ = fmul(f, V, p.ZZ);
    r.ZZZ = fmul(f, W, p.ZZZ);
    return r;
  }
  const F4 PP = fmul(f, P, P), PPP = fmul(f, P, PP), Q = fmul(f, U1, PP);
  Xyzz r;
  r.X = fsub(f, fsub(f, fsub(f, fmul(f, R, R), PPP), Q), Q);
  r.Y = fsub(f, fmul(f, R, fsub(f, Q, r.X)), fmul(f, S1, PPP));
  r.ZZ = fmul(f, fmul(f, p.ZZ, q.ZZ), PP);
  r.ZZZ = fmul(f, fmul(f, p.ZZZ, q.ZZZ), PPP);
  return r;
}
Aff xyzz_to_aff(const Xyzz& p) {
  const Field& f = fq();
  if (xyzz_inf(p)) return Aff{{}, {}, true};
  const F4 izzz = finv(f, p.ZZZ);
  const F4 izz = fmul(f, fmul(f, p.ZZ, izzz), fmul(f, p.ZZ, izzz));  // (ZZ / ZZZ)^2 = 1 / ZZ
  return Aff{fmul(f, p.X, izz), fmul(f, p.Y, izzz), false};
}

Aff load_aff(const uint64_t* p) {
  const Field& f = fq();
  Aff a;
  const F4 x = *(const F4*)p, y = *(const F4*)(p + 4);
  a.inf = fzero(x) && fzero(y);
  a.x = to_m(f, x);
  a.y = to_m(f, y);
  return a;
}
void store_aff(const Aff& a, uint64_t* out) {
  const Field& f = fq();
  if (a.inf) {
    memset(out, 0, 64);
    return;
  }
  const F4 x = from_m(f, a.x), y = from_m(f, a.y);
  memcpy(out, x.v, 32);
  memcpy(out + 4, y.v, 32);
}
}  // namespace

extern "C" {

// SRS::eval_at_s (plonk.rs:51-58), literally: fold of affine double-and-add products.
// points: n x 8 u64 affine canonical; scalars: n x 4 u64 canonical Fr; out: 8 u64.
int oracle_g1_msm_naive(const uint64_t* points, const uint64_t* scalars, size_t n, uint64_t* out) {
  Aff acc{{}, {}, true};
  for (size_t i = 0; i < n; ++i) acc = aff_add(acc, aff_mul(load_aff(points + 8 * i), scalars + 4 * i));
  store_aff(acc, out);
  return 0;
}

// The same sum, Pippenger with 16-bit windows on `threads` threads (one window at a time per
// thread): bucket accumulation in XYZZ (mixed additions), running-sum reduction, Horner.
int oracle_g1_msm_pippenger(const uint64_t* points, const uint64_t* scalars, size_t n, int threads,
                            uint64_t* out) {
  constexpr int C = 16, NW = 16;
  std::vector<Aff> pts(n);
  for (size_t i = 0; i < n; ++i) pts[i] = load_aff(points + 8 * i);
  std::vector<Xyzz> win(NW);
  auto work = [&](int w) {
    std::vector<Xyzz> bk((size_t)1 << C, Xyzz{{}, {}, {}, {}});
    for (size_t i = 0; i < n; ++i) {
      const uint32_t d = (uint32_t)((scalars[4 * i + w / 4] >> (16 * (w % 4))) & 0xFFFF);
      if (d) bk[d] = xyzz_madd(bk[d], pts[i]);
    }
    Xyzz run{{}, {}, {}, {}}, sum{{}, {}, {}, {}};
    for (size_t d = ((size_t)1 << C) - 1; d >= 1; --d) {  // sum_d d B_d as running sums
      run = xyzz_add(run, bk[d]);
      sum = xyzz_add(sum, run);
    }
    win[w] = sum;
  };
  if (threads < 1) threads = 1;
  for (int w0 = 0; w0 < NW; w0 += threads) {
    std::vector<std::thread> ts;
    for (int w = w0; w < NW && w < w0 + threads; ++w) ts.emplace_back(work, w);
    for (auto& t : ts) t.join();
  }
  Xyzz acc = win[NW - 1];
  for (int w = NW - 2; w >= 0; --w) {
    for (int k = 0; k < C; ++k) acc = xyzz_add(acc, acc);
    acc = xyzz_add(acc, win[w]);
  }
  store_aff(xyzz_to_aff(acc), out);
  return 0;
}

// points k_i G for canonical Fr scalars k (setup of the MSM baselines; double-and-add in
// XYZZ, then one inversion per point)
int oracle_g1_mul_gen(const uint64_t* scalars, size_t n, uint64_t* out) {
  const Field& f = fq();
  const F4 one_plain{{1, 0, 0, 0}}, two_plain{{2, 0, 0, 0}};
  const Aff g{to_m(f, one_plain), to_m(f, two_plain), false};
  for (size_t i = 0; i < n; ++i) {
    Xyzz acc{{}, {}, {}, {}};
    const uint64_t* s = scalars + 4 * i;
    for (int l = 3; l >= 0; --l)
      for (int b = 63; b >= 0; --b) {
        acc = xyzz_add(acc, acc);
        if ((s[l] >> b) & 1) acc = xyzz_madd(acc, g);
      }
    store_aff(xyzz_to_aff(acc), out + 8 * i);
  }
  return 0;
}

// P_i = (k0 + i d) G for i < n, affine (setup of the Pippenger baseline at 2^20 points: one
// mixed addition per point, then a batch inversion of the ZZZ (Montgomery's trick))
int oracle_g1_progression(const uint64_t* k0, const uint64_t* d, size_t n, uint64_t* out) {
  const Field& f = fq();
  if (n == 0) return 0;
  std::vector<uint64_t> tmp(16);
  oracle_g1_mul_gen(k0, 1, tmp.data());
  oracle_g1_mul_gen(d, 1, tmp.data() + 8);
  const Aff D = load_aff(tmp.data() + 8);
  std::vector<Xyzz> xs(n);
  xs[0] = Xyzz{load_aff(tmp.data()).x, load_aff(tmp.data()).y, f.one, f.one};
  for (size_t i = 1; i < n; ++i) xs[i] = xyzz_madd(xs[i - 1], D);
  std::vector<F4> pre(n + 1);
  pre[0] = f.one;
  for (size_t i = 0; i < n; ++i) pre[i + 1] = fmul(f, pre[i], xyzz_inf(xs[i]) ? f.one : xs[i].ZZZ);
  F4 inv = finv(f, pre[n]);
  for (size_t i = n; i-- > 0;) {
    if (xyzz_inf(xs[i])) {
      memset(out + 8 * i, 0, 64);
      continue;
    }
    const F4 izzz = fmul(f, inv, pre[i]);
    inv = fmul(f, inv, xs[i].ZZZ);
    const F4 q = fmul(f, xs[i].ZZ, izzz);
    store_aff(Aff{fmul(f, xs[i].X, fmul(f, q, q)), fmul(f, xs[i].Y, izzz), false}, out + 8 * i);
  }
  return 0;
}

}  // extern "C"
