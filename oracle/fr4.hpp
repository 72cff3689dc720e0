// ORACLE / CPU BASELINE — TEST INFRASTRUCTURE ONLY (see field.hpp header). Never linked
// into libpbf.so; only tests/ and bench.py's cpu_baseline legs load it (liboracle.so).
//
// 4 x 64-bit Montgomery arithmetic for the BN254 fields (Fr, Fq; R = 2^256) and affine / XYZZ
// G1 arithmetic over Fq, shared by the CPU restatements in bn254_cpu.cpp (config 3-4
// baselines) and prover_cpu.cpp (config 5 baseline and the O(n) proof checker).
// Field elements canonical at the C boundary, Montgomery inside.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <thread>
#include <vector>

namespace bn4 {
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

inline Field make_field(const uint64_t* p) {
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
inline F4 fpow(const Field& f, F4 a, const uint64_t* e) {  // a in Montgomery form
  F4 r = f.one;
  for (int i = 3; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      r = fmul(f, r, r);
      if ((e[i] >> b) & 1) r = fmul(f, r, a);
    }
  return r;
}
inline F4 finv(const Field& f, const F4& a) {  // Fermat, a^(p-2)
  uint64_t e[4];
  memcpy(e, f.p, 32);
  e[0] -= 2;
  return fpow(f, a, e);
}

constexpr uint64_t R_MOD[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull};
constexpr uint64_t Q_MOD[4] = {0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull};

inline const Field& fr() {
  static const Field f = make_field(R_MOD);
  return f;
}
inline const Field& fq() {
  static const Field f = make_field(Q_MOD);
  return f;
}

// ---------------------------------------------------------------- G1 over Fq
struct Aff {
  F4 x, y;
  bool inf;
};
// affine addition, chord / tangent (src/pbh/g1.rs:108-144 for y^2 = x^3 + 3)
inline Aff aff_add(const Aff& p, const Aff& q) {
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
inline Aff aff_mul(const Aff& p, const uint64_t* s) {
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
inline Xyzz xyzz_madd(const Xyzz& p, const Aff& q) {
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
inline Xyzz xyzz_add(const Xyzz& p, const Xyzz& q) {
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
inline Aff xyzz_to_aff(const Xyzz& p) {
  const Field& f = fq();
  if (xyzz_inf(p)) return Aff{{}, {}, true};
  const F4 izzz = finv(f, p.ZZZ);
  const F4 izz = fmul(f, fmul(f, p.ZZ, izzz), fmul(f, p.ZZ, izzz));  // (ZZ / ZZZ)^2 = 1 / ZZ
  return Aff{fmul(f, p.X, izz), fmul(f, p.Y, izzz), false};
}

inline Aff load_aff(const uint64_t* p) {
  const Field& f = fq();
  Aff a;
  const F4 x = *(const F4*)p, y = *(const F4*)(p + 4);
  a.inf = fzero(x) && fzero(y);
  a.x = to_m(f, x);
  a.y = to_m(f, y);
  return a;
}
inline void store_aff(const Aff& a, uint64_t* out) {
  const Field& f = fq();
  if (a.inf) {
    memset(out, 0, 64);
    return;
  }
  const F4 x = from_m(f, a.x), y = from_m(f, a.y);
  memcpy(out, x.v, 32);
  memcpy(out + 4, y.v, 32);
}

// parallel for over [0, n) in contiguous slices on `threads` host threads
template <class F>
void par_for(size_t n, int threads, F&& f) {
  if (threads <= 1 || n < 4096) {
    f((size_t)0, n);
    return;
  }
  std::vector<std::thread> ts;
  const size_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const size_t lo = (size_t)t * per, hi = lo + per < n ? lo + per : n;
    if (lo >= hi) break;
    ts.emplace_back([&f, lo, hi] { f(lo, hi); });
  }
  for (auto& t : ts) t.join();
}
}  // namespace bn4
