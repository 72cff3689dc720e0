// ORACLE / CPU BASELINE — TEST INFRASTRUCTURE ONLY (see field.hpp header). Never linked
// into libpbf.so; only tests/ and bench.py's cpu_baseline legs load it (liboracle.so).
//
// BASELINE config 5 on the host, three pieces:
//  * oracle_synth_circuit: a restatement of the GPU's synthetic config-5 circuit
//    (plonk-by-fingers_amd/csrc/prover.hip k_synth_circuit: splitmix64-derived a, b, c = a b,
//    every 4th gate's c copied into the next gate's a), so fixtures of a seeded circuit can be
//    produced here without a GPU;
//  * oracle_commitment_scalars: the O(n) checker of oracle/plonk_bn254.py commitment_scalars
//    (barycentric evaluations of every polynomial of Plonk::prove, src/plonk.rs:245-446, at the
//    SRS secret s and the challenge z) in 4 x u64 Montgomery arithmetic on all host cores --
//    what pins the 2^24-gate proof (tests/golden/gen_prove_2p24.py);
//  * oracle_plonk_prove_cpu: the generalised prover as a CPU baseline (BASELINE.md row 5,
//    "generalised C++ prover, 1 and all cores"): Plonk::prove (src/plonk.rs:191-466) for any
//    power-of-two n with the O(n log n) algorithms the GPU prover uses -- interpolation and
//    the quotient by (coset) NTTs, the accumulator by prefix products and one batch inversion,
//    openings by synthetic division, commitments by a Pippenger MSM -- with every step
//    recomputed per proof as the reference does (no proving key). Output: the proof's 9 points
//    and 7 field elements, canonical (bit-identical to the GPU's: tests compare them).
#include "fr4.hpp"

#include <algorithm>
#include <cmath>

namespace {
using namespace bn4;

inline F4 fr_from_u64(uint64_t v) { return to_m(fr(), F4{{v, 0, 0, 0}}); }
inline F4 fr_load(const uint64_t* p) { return to_m(fr(), *(const F4*)p); }
inline void fr_store(const F4& m, uint64_t* p) {
  const F4 c = from_m(fr(), m);
  memcpy(p, c.v, 32);
}
inline F4 fr_neg(const F4& a) { return fsub(fr(), F4{{0, 0, 0, 0}}, a); }
F4 fr_pow64(F4 a, uint64_t e) {
  F4 r = fr().one;
  while (e) {
    if (e & 1) r = fmul(fr(), r, a);
    a = fmul(fr(), a, a);
    e >>= 1;
  }
  return r;
}
F4 fr_inv(const F4& a) { return finv(fr(), a); }
// primitive 2^k-th root of unity 5^((r-1)/2^k) (Montgomery)
F4 fr_root(uint32_t log_n) {
  uint64_t e[4];
  memcpy(e, R_MOD, 32);
  e[0] -= 1;
  for (uint32_t s = 0; s < log_n; ++s)
    for (int i = 0; i < 4; ++i) e[i] = (e[i] >> 1) | (i < 3 ? (e[i + 1] << 63) : 0);
  return fpow(fr(), fr_from_u64(5), e);
}

// ---- splitmix64 / rand_fr exactly as prover.hip's sm64 / rand_fr
inline uint64_t sm64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
F4 rand_fr_plain(uint64_t seed, uint64_t i) {
  const uint64_t G = 0x9E3779B97F4A7C15ull;
  uint64_t ctr = seed + (i + 1) * G * 4;
  for (;;) {
    F4 v;
    for (int k = 0; k < 4; ++k) v.v[k] = sm64(ctr += G);
    v.v[3] &= (1ull << 62) - 1;
    if (!geq(v.v, R_MOD)) return v;
  }
}

// ---- iterative radix-2 NTT (natural order in and out), parallel per stage
void bitrev(std::vector<F4>& a) {
  const size_t n = a.size();
  for (size_t i = 1, j = 0; i < n; ++i) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
}
// out[k] = sum_j a[j] w^(jk); inverse: w^-1 and n^-1
void ntt(std::vector<F4>& a, const F4& w, bool inverse, int threads) {
  const Field& f = fr();
  const size_t n = a.size();
  if (n <= 1) return;
  const F4 root = inverse ? fr_inv(w) : w;
  std::vector<F4> tw(n / 2);  // root^i
  tw[0] = f.one;
  for (size_t i = 1; i < n / 2; ++i) tw[i] = fmul(f, tw[i - 1], root);
  bitrev(a);
  for (size_t len = 2; len <= n; len <<= 1) {
    const size_t half = len / 2, step = n / len;
    par_for(n / 2, threads, [&](size_t lo, size_t hi) {
      for (size_t t = lo; t < hi; ++t) {
        const size_t blk = t / half, j = t % half;
        const size_t i0 = blk * len + j, i1 = i0 + half;
        const F4 y = fmul(f, a[i1], tw[j * step]);
        a[i1] = fsub(f, a[i0], y);
        a[i0] = fadd(f, a[i0], y);
      }
    });
  }
  if (inverse) {
    const F4 ninv = fr_inv(fr_from_u64(n));
    par_for(n, threads, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) a[i] = fmul(f, a[i], ninv);
    });
  }
}

// ---- G1 MSM: Pippenger, window c from n, one window per thread at a time
Xyzz msm(const std::vector<Aff>& pts, const std::vector<F4>& sc_m, size_t cnt, int threads) {
  const Field& f = fr();
  if (cnt == 0) return Xyzz{{}, {}, {}, {}};
  std::vector<F4> sc(cnt);  // canonical scalars
  for (size_t i = 0; i < cnt; ++i) sc[i] = from_m(f, sc_m[i]);
  const int c = std::max(4, std::min(16, (int)std::log2((double)cnt) - 3));
  const int nw = (254 + c - 1) / c;
  std::vector<Xyzz> win(nw);
  auto digit = [&](size_t i, int w) -> uint32_t {
    const int bit = w * c, limb = bit / 64, off = bit % 64;
    uint64_t v = sc[i].v[limb] >> off;
    if (off + c > 64 && limb < 3) v |= sc[i].v[limb + 1] << (64 - off);
    return (uint32_t)(v & ((1ull << c) - 1));
  };
  auto work = [&](int w) {
    std::vector<Xyzz> bk((size_t)1 << c, Xyzz{{}, {}, {}, {}});
    for (size_t i = 0; i < cnt; ++i) {
      const uint32_t d = digit(i, w);
      if (d) bk[d] = xyzz_madd(bk[d], pts[i]);
    }
    Xyzz run{{}, {}, {}, {}}, sum{{}, {}, {}, {}};
    for (size_t d = ((size_t)1 << c) - 1; d >= 1; --d) {
      run = xyzz_add(run, bk[d]);
      sum = xyzz_add(sum, run);
    }
    win[w] = sum;
  };
  const int T = std::max(1, threads);
  for (int w0 = 0; w0 < nw; w0 += T) {
    std::vector<std::thread> ts;
    for (int w = w0; w < nw && w < w0 + T; ++w) ts.emplace_back(work, w);
    for (auto& t : ts) t.join();
  }
  Xyzz acc = win[nw - 1];
  for (int w = nw - 2; w >= 0; --w) {
    for (int k = 0; k < c; ++k) acc = xyzz_add(acc, acc);
    acc = xyzz_add(acc, win[w]);
  }
  return acc;
}

// p(x) by Horner
F4 horner(const F4* p, size_t len, const F4& x) {
  const Field& f = fr();
  F4 acc{{0, 0, 0, 0}};
  for (size_t j = len; j-- > 0;) acc = fadd(f, fmul(f, acc, x), p[j]);
  return acc;
}
// (p - y) / (x - z): q of len-1 coefficients; returns the remainder p(z) - y
F4 synth_div(const F4* p, size_t len, const F4& z, const F4& y, std::vector<F4>& q) {
  const Field& f = fr();
  q.assign(len > 1 ? len - 1 : 0, F4{{0, 0, 0, 0}});
  F4 s{{0, 0, 0, 0}};
  for (size_t k = 0; k < len; ++k) {
    const size_t j = len - 1 - k;
    F4 u = p[j];
    if (j == 0) u = fsub(f, u, y);
    s = fadd(f, u, fmul(f, z, s));
    if (j > 0) q[j - 1] = s;
  }
  return s;
}

// ---- the O(n) barycentric evaluator of plonk_bn254.py: f(x) = (x^n - 1)/n sum_i f_i w^i/(x - w^i)
struct Bary {
  std::vector<F4> w;
  F4 scale;
};
Bary bary(size_t n, const std::vector<F4>& h, const F4& x, int threads) {
  const Field& f = fr();
  Bary b;
  b.w.resize(n);
  std::vector<F4> d(n);
  for (size_t i = 0; i < n; ++i) d[i] = fsub(f, x, h[i]);
  // batch inversion in `threads` chunks (prefix products per chunk, one Fermat inverse each)
  const int T = std::max(1, threads);
  const size_t per = (n + T - 1) / T;
  std::vector<std::thread> ts;
  for (int t = 0; t < T; ++t) {
    const size_t lo = (size_t)t * per, hi = std::min(n, lo + per);
    if (lo >= hi) break;
    ts.emplace_back([&, lo, hi] {
      std::vector<F4> pre(hi - lo + 1);
      pre[0] = f.one;
      for (size_t i = lo; i < hi; ++i) pre[i - lo + 1] = fmul(f, pre[i - lo], d[i]);
      F4 inv = fr_inv(pre[hi - lo]);
      for (size_t i = hi; i-- > lo;) {
        b.w[i] = fmul(f, fmul(f, inv, pre[i - lo]), h[i]);
        inv = fmul(f, inv, d[i]);
      }
    });
  }
  for (auto& t : ts) t.join();
  b.scale = fmul(f, fsub(f, fr_pow64(x, n), f.one), fr_inv(fr_from_u64(n)));
  return b;
}
F4 bary_eval(const Bary& b, const F4* vals, size_t n, int threads) {
  const Field& f = fr();
  const int T = std::max(1, threads);
  std::vector<F4> part(T, F4{{0, 0, 0, 0}});
  par_for(n, T, [&](size_t lo, size_t hi) {
    F4 acc{{0, 0, 0, 0}};
    for (size_t i = lo; i < hi; ++i) acc = fadd(f, acc, fmul(f, vals[i], b.w[i]));
    const size_t slot = lo / ((n + T - 1) / T);
    part[slot < (size_t)T ? slot : T - 1] = acc;
  });
  F4 s{{0, 0, 0, 0}};
  for (const F4& p : part) s = fadd(f, s, p);
  return fmul(f, s, b.scale);
}

struct Circuit {
  size_t n;
  std::vector<F4> q[5], abc[3], sig[3];  // Montgomery
  std::vector<F4> h;
};
void load_circuit(Circuit& C, size_t n, const uint64_t* q, const uint64_t* copies, const uint64_t* abc, const F4& k1,
                  const F4& k2, const F4& omega, int threads) {
  const Field& f = fr();
  C.n = n;
  C.h.resize(n);
  C.h[0] = f.one;
  for (size_t i = 1; i < n; ++i) C.h[i] = fmul(f, C.h[i - 1], omega);
  for (int k = 0; k < 5; ++k) {
    C.q[k].resize(n);
    par_for(n, threads, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) C.q[k][i] = fr_load(q + 4 * (k * n + i));
    });
  }
  for (int k = 0; k < 3; ++k) {
    C.abc[k].resize(n);
    C.sig[k].resize(n);
    par_for(n, threads, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        C.abc[k][i] = fr_load(abc + 4 * (k * n + i));
        const uint64_t kind = copies[2 * (k * n + i)], idx = copies[2 * (k * n + i) + 1];
        F4 v = C.h[idx - 1];
        if (kind == 1) v = fmul(f, v, k1);
        if (kind == 2) v = fmul(f, v, k2);
        C.sig[k][i] = v;
      }
    });
  }
}
// acc_i = prod_{j<i} num_j / den_j (plonk.rs:278-299), one batch inversion
std::vector<F4> accumulator(const Circuit& C, const F4& beta, const F4& gamma, const F4& k1, const F4& k2) {
  const Field& f = fr();
  const size_t n = C.n;
  std::vector<F4> nums(n, f.one), dens(n, f.one);
  F4 pn = f.one, pd = f.one;
  for (size_t i = 1; i < n; ++i) {
    const F4 wi = C.h[i - 1], bw = fmul(f, beta, wi);
    const F4& a = C.abc[0][i - 1];
    const F4& b = C.abc[1][i - 1];
    const F4& c = C.abc[2][i - 1];
    F4 t = fmul(f, fadd(f, fadd(f, a, bw), gamma), fadd(f, fadd(f, b, fmul(f, bw, k1)), gamma));
    pn = fmul(f, pn, fmul(f, t, fadd(f, fadd(f, c, fmul(f, bw, k2)), gamma)));
    F4 u = fmul(f, fadd(f, fadd(f, a, fmul(f, beta, C.sig[0][i - 1])), gamma),
                fadd(f, fadd(f, b, fmul(f, beta, C.sig[1][i - 1])), gamma));
    pd = fmul(f, pd, fmul(f, u, fadd(f, fadd(f, c, fmul(f, beta, C.sig[2][i - 1])), gamma)));
    nums[i] = pn;
    dens[i] = pd;
  }
  std::vector<F4> pre(n + 1);
  pre[0] = f.one;
  for (size_t i = 0; i < n; ++i) pre[i + 1] = fmul(f, pre[i], dens[i]);
  F4 inv = fr_inv(pre[n]);
  std::vector<F4> acc(n);
  for (size_t i = n; i-- > 0;) {
    acc[i] = fmul(f, nums[i], fmul(f, inv, pre[i]));
    inv = fmul(f, inv, dens[i]);
  }
  return acc;
}

}  // namespace

extern "C" {

// k_synth_circuit (prover.hip) on the host: q (5 x n x 4), copies (3 x n x 2), abc (3 x n x 4)
int oracle_synth_circuit(size_t n, uint64_t seed, uint64_t* q, uint64_t* copies, uint64_t* abc, int threads) {
  const Field& f = fr();
  F4 mone;
  memcpy(mone.v, R_MOD, 32);
  mone.v[0] -= 1;
  par_for(n, threads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      const F4 z{{0, 0, 0, 0}}, one{{1, 0, 0, 0}};
      memcpy(q + 4 * i, z.v, 32);
      memcpy(q + 4 * (n + i), z.v, 32);
      memcpy(q + 4 * (2 * n + i), mone.v, 32);
      memcpy(q + 4 * (3 * n + i), one.v, 32);
      memcpy(q + 4 * (4 * n + i), z.v, 32);
      const F4 b = rand_fr_plain(seed ^ 0xB0B0ull, i);
      F4 a;
      if (i % 4 == 1)
        a = from_m(f, fmul(f, to_m(f, rand_fr_plain(seed, i - 1)), to_m(f, rand_fr_plain(seed ^ 0xB0B0ull, i - 1))));
      else
        a = rand_fr_plain(seed, i);
      const F4 c = from_m(f, fmul(f, to_m(f, a), to_m(f, b)));
      memcpy(abc + 4 * i, a.v, 32);
      memcpy(abc + 4 * (n + i), b.v, 32);
      memcpy(abc + 4 * (2 * n + i), c.v, 32);
      uint64_t* ca = copies + 2 * i;
      uint64_t* cb = copies + 2 * (n + i);
      uint64_t* cc = copies + 2 * (2 * n + i);
      ca[0] = 0; ca[1] = i + 1;
      cb[0] = 1; cb[1] = i + 1;
      cc[0] = 2; cc[1] = i + 1;
      if (i % 4 == 1) { ca[0] = 2; ca[1] = i; }
      if (i % 4 == 0 && i + 1 < n) { cc[0] = 0; cc[1] = i + 2; }
    }
  });
  return 0;
}

// oracle/plonk_bn254.py commitment_scalars (O(n), barycentric). chal: alpha beta gamma z v;
// rnd: b1..b9; s: the SRS secret; k1k2: 2 x 4. out (canonical, 4 u64 each), per mode m in
// (0 reference, 1 paper) at out + 56 m: a b c z t wz wzw, then the 7 proof fields
// (a_z b_z c_z s1_z s2_z r_z zw_z). Returns 1 if s or z lies in H (the formula needs x not in H).
int oracle_commitment_scalars(size_t n, const uint64_t* q, const uint64_t* copies, const uint64_t* abc,
                              const uint64_t* chal, const uint64_t* rnd, const uint64_t* s_in, const uint64_t* k1k2,
                              int threads, uint64_t* out) {
  const Field& f = fr();
  uint32_t log_n = 0;
  while (((size_t)1 << log_n) < n) ++log_n;
  const F4 omega = fr_root(log_n);
  const F4 k1 = fr_load(k1k2), k2 = fr_load(k1k2 + 4);
  const F4 alpha = fr_load(chal), beta = fr_load(chal + 4), gamma = fr_load(chal + 8), z = fr_load(chal + 12),
           v = fr_load(chal + 16);
  F4 b[9];
  for (int i = 0; i < 9; ++i) b[i] = fr_load(rnd + 4 * i);
  const F4 s = fr_load(s_in);
  Circuit C;
  load_circuit(C, n, q, copies, abc, k1, k2, omega, threads);
  const std::vector<F4> acc = accumulator(C, beta, gamma, k1, k2);
  for (size_t i = 0; i < n; ++i)
    if (feq(C.h[i], s) || feq(C.h[i], z)) return 1;
  struct At {
    F4 x, zh, a, b, c, z, s1, s2, s3, ql, qr, qo, qm, qc, l1;
  };
  auto at = [&](const F4& x) {
    At d;
    const Bary w = bary(n, C.h, x, threads);
    auto ev = [&](const std::vector<F4>& vals) { return bary_eval(w, vals.data(), n, threads); };
    d.x = x;
    d.zh = fsub(f, fr_pow64(x, n), f.one);
    d.a = fadd(f, fmul(f, fadd(f, fmul(f, b[0], x), b[1]), d.zh), ev(C.abc[0]));
    d.b = fadd(f, fmul(f, fadd(f, fmul(f, b[2], x), b[3]), d.zh), ev(C.abc[1]));
    d.c = fadd(f, fmul(f, fadd(f, fmul(f, b[4], x), b[5]), d.zh), ev(C.abc[2]));
    const F4 bz = fadd(f, fadd(f, fmul(f, b[6], fmul(f, x, x)), fmul(f, b[7], x)), b[8]);
    d.z = fadd(f, fmul(f, bz, d.zh), ev(acc));
    d.s1 = ev(C.sig[0]);
    d.s2 = ev(C.sig[1]);
    d.s3 = ev(C.sig[2]);
    d.ql = ev(C.q[0]);
    d.qr = ev(C.q[1]);
    d.qo = ev(C.q[2]);
    d.qm = ev(C.q[3]);
    d.qc = ev(C.q[4]);
    d.l1 = fmul(f, d.zh, fr_inv(fmul(f, fr_from_u64(n), fsub(f, x, f.one))));
    return d;
  };
  auto z_at = [&](const F4& x) {
    const Bary w = bary(n, C.h, x, threads);
    const F4 zh = fsub(f, fr_pow64(x, n), f.one);
    const F4 bz = fadd(f, fadd(f, fmul(f, b[6], fmul(f, x, x)), fmul(f, b[7], x)), b[8]);
    return fadd(f, fmul(f, bz, zh), bary_eval(w, acc.data(), n, threads));
  };
  auto numerator = [&](const At& d, const F4& zw) {
    const F4& x = d.x;
    F4 t1 = fadd(f, fadd(f, fadd(f, fadd(f, fmul(f, fmul(f, d.a, d.b), d.qm), fmul(f, d.a, d.ql)), fmul(f, d.b, d.qr)),
                              fmul(f, d.c, d.qo)),
                 d.qc);
    const F4 bx = fmul(f, beta, x);
    F4 t2 = fmul(f, fmul(f, fadd(f, fadd(f, d.a, bx), gamma), fadd(f, fadd(f, d.b, fmul(f, bx, k1)), gamma)),
                 fadd(f, fadd(f, d.c, fmul(f, bx, k2)), gamma));
    t2 = fmul(f, fmul(f, alpha, t2), d.z);
    F4 t3 = fmul(f, fmul(f, fadd(f, fadd(f, d.a, fmul(f, beta, d.s1)), gamma),
                         fadd(f, fadd(f, d.b, fmul(f, beta, d.s2)), gamma)),
                 fadd(f, fadd(f, d.c, fmul(f, beta, d.s3)), gamma));
    t3 = fmul(f, fmul(f, alpha, t3), zw);
    const F4 t4 = fmul(f, fmul(f, fsub(f, d.z, f.one), fmul(f, alpha, alpha)), d.l1);
    return fadd(f, fsub(f, fadd(f, t1, t2), t3), t4);
  };
  const At S = at(s), Z = at(z);
  const F4 zw_s = z_at(fmul(f, omega, s)), zw_z = z_at(fmul(f, omega, z));
  const F4 t_s = fmul(f, numerator(S, zw_s), fr_inv(S.zh));
  const F4 t_z = fmul(f, numerator(Z, zw_z), fr_inv(Z.zh));
  const F4 k3 = fmul(f, fmul(f, fadd(f, fadd(f, Z.a, fmul(f, beta, Z.s1)), gamma),
                             fadd(f, fadd(f, Z.b, fmul(f, beta, Z.s2)), gamma)),
                     alpha);
  const F4 c2 = fmul(f, fmul(f, fmul(f, fadd(f, fadd(f, Z.a, fmul(f, beta, z)), gamma),
                                     fadd(f, fadd(f, Z.b, fmul(f, fmul(f, beta, k1), z)), gamma)),
                             fadd(f, fadd(f, Z.c, fmul(f, fmul(f, beta, k2), z)), gamma)),
                     alpha);
  for (int md = 0; md < 2; ++md) {
    auto r_at = [&](const At& d) {
      F4 r1 = fadd(f, fadd(f, fadd(f, fadd(f, fmul(f, d.qm, fmul(f, Z.a, Z.b)), fmul(f, d.ql, Z.a)), fmul(f, d.qr, Z.b)),
                           fmul(f, d.qo, Z.c)),
                   d.qc);
      const F4 r2 = fmul(f, d.z, c2);
      const F4 r3 = md == 0 ? fmul(f, fmul(f, fmul(f, d.z, d.s3), fmul(f, beta, zw_z)), k3)
                            : fr_neg(fmul(f, fmul(f, fmul(f, beta, zw_z), k3), d.s3));
      const F4 r4 = fmul(f, fmul(f, d.z, Z.l1), fmul(f, alpha, alpha));
      return fadd(f, fadd(f, fadd(f, r1, r2), r3), r4);
    };
    const F4 r_z = r_at(Z);
    F4 vp = v, wz = fr_neg(t_z);
    const F4 terms[6] = {fsub(f, r_at(S), r_z), fsub(f, S.a, Z.a), fsub(f, S.b, Z.b), fsub(f, S.c, Z.c),
                         fsub(f, S.s1, Z.s1), fsub(f, S.s2, Z.s2)};
    for (int k = 0; k < 6; ++k) {
      wz = fadd(f, wz, fmul(f, vp, terms[k]));
      vp = fmul(f, vp, v);
    }
    const F4 wzw = fmul(f, fsub(f, S.z, zw_z), fr_inv(fsub(f, s, fmul(f, omega, z))));
    const F4 vals[14] = {S.a, S.b, S.c, S.z, t_s, wz, wzw, Z.a, Z.b, Z.c, Z.s1, Z.s2, r_z, zw_z};
    for (int k = 0; k < 14; ++k) fr_store(vals[k], out + 56 * md + 4 * k);
  }
  return 0;
}

// The generalised prover on the host (see the file header). srs: srs_m affine points (8 u64,
// (0, 0) = identity); out_pts 9 x 8, out_f 7 x 4 (pbf.h pbf_plonk_prove_bn254 layout).
// Returns 0, or 1 for an unsatisfiable input (a nonzero quotient tail or remainder, a zero
// accumulator denominator), 2 for a short SRS.
int oracle_plonk_prove_cpu(size_t n, const uint64_t* q, const uint64_t* copies, const uint64_t* abc,
                           const uint64_t* chal, const uint64_t* rnd, const uint64_t* k1k2, const uint64_t* srs,
                           size_t srs_m, int mode, int threads, uint64_t* out_pts, uint64_t* out_f) {
  const Field& f = fr();
  uint32_t log_n = 0;
  while (((size_t)1 << log_n) < n) ++log_n;
  const size_t N = 4 * n, m = n + 2;
  const size_t rlen = mode == 0 ? 2 * n + 2 : n + 3;
  if (srs_m < (mode == 0 ? 2 * n + 2 : n + 3)) return 2;
  const F4 omega = fr_root(log_n), omegaN = fr_root(log_n + 2), g = fr_from_u64(5), g_inv = fr_inv(g);
  const F4 k1 = fr_load(k1k2), k2 = fr_load(k1k2 + 4);
  const F4 alpha = fr_load(chal), beta = fr_load(chal + 4), gamma = fr_load(chal + 8), zc = fr_load(chal + 12),
           v = fr_load(chal + 16);
  F4 bl[9];
  for (int i = 0; i < 9; ++i) bl[i] = fr_load(rnd + 4 * i);
  Circuit C;
  load_circuit(C, n, q, copies, abc, k1, k2, omega, threads);
  std::vector<Aff> pts(srs_m);
  par_for(srs_m, threads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) pts[i] = load_aff(srs + 8 * i);
  });
  Xyzz com[9];
  // ---- interpolation (plonk.rs:233-243): 11 INTTs of size n
  auto interp = [&](const std::vector<F4>& vals, size_t len) {
    std::vector<F4> c(vals);
    ntt(c, omega, true, threads);
    c.resize(len, F4{{0, 0, 0, 0}});
    return c;
  };
  std::vector<F4> A = interp(C.abc[0], n + 8), Bp = interp(C.abc[1], n + 8), Cp = interp(C.abc[2], n + 8);
  std::vector<F4> Q[5], Sg[3];
  for (int k = 0; k < 5; ++k) Q[k] = interp(C.q[k], n);
  for (int k = 0; k < 3; ++k) Sg[k] = interp(C.sig[k], n);
  // ---- round 1 (plonk.rs:250-257)
  std::vector<F4>* abcp[3] = {&A, &Bp, &Cp};
  for (int k = 0; k < 3; ++k) {
    std::vector<F4>& p = *abcp[k];
    const F4 lo = bl[2 * k + 1], hi = bl[2 * k];
    p[0] = fsub(f, p[0], lo);
    p[1] = fsub(f, p[1], hi);
    p[n] = fadd(f, p[n], lo);
    p[n + 1] = fadd(f, p[n + 1], hi);
    com[k] = msm(pts, p, n + 2, threads);
  }
  // ---- round 2 (plonk.rs:278-313)
  std::vector<F4> acc = accumulator(C, beta, gamma, k1, k2);
  std::vector<F4> Zx = interp(acc, n + 8);
  {
    const F4 c0 = bl[8], c1 = bl[7], c2 = bl[6];
    Zx[0] = fsub(f, Zx[0], c0);
    Zx[1] = fsub(f, Zx[1], c1);
    Zx[2] = fsub(f, Zx[2], c2);
    Zx[n] = fadd(f, Zx[n], c0);
    Zx[n + 1] = fadd(f, Zx[n + 1], c1);
    Zx[n + 2] = fadd(f, Zx[n + 2], c2);
  }
  com[3] = msm(pts, Zx, n + 3, threads);
  // ---- round 3: the quotient on the coset g H_4n (plonk.rs:326-382)
  auto coset = [&](const std::vector<F4>& c, size_t len, const F4& base) {
    std::vector<F4> e(N, F4{{0, 0, 0, 0}});
    F4 x = f.one;
    for (size_t j = 0; j < len; ++j) {
      e[j] = fmul(f, c[j], x);
      x = fmul(f, x, base);
    }
    ntt(e, omegaN, false, threads);
    return e;
  };
  std::vector<F4> L1(n, fr_inv(fr_from_u64(n)));
  const std::vector<F4> ea = coset(A, n + 2, g), eb = coset(Bp, n + 2, g), ec = coset(Cp, n + 2, g),
                        ez = coset(Zx, n + 3, g);
  std::vector<F4> eq[5], es[3];
  for (int k = 0; k < 5; ++k) eq[k] = coset(Q[k], n, g);
  for (int k = 0; k < 3; ++k) es[k] = coset(Sg[k], n, g);
  const std::vector<F4> el1 = coset(L1, n, g);
  F4 zh_inv[4];
  {
    const F4 gn = fr_pow64(g, n), w4 = fr_pow64(omegaN, n);
    F4 x = gn;
    for (int j = 0; j < 4; ++j) {
      zh_inv[j] = fr_inv(fsub(f, x, f.one));
      x = fmul(f, x, w4);
    }
  }
  std::vector<F4> T(N);
  const F4 alpha2 = fmul(f, alpha, alpha);
  par_for(N, threads, [&](size_t lo, size_t hi) {
    F4 x = fmul(f, g, fr_pow64(omegaN, lo));
    for (size_t i = lo; i < hi; ++i, x = fmul(f, x, omegaN)) {
      const F4 &a = ea[i], &b = eb[i], &c = ec[i], &z = ez[i], &zw = ez[(i + 4) % N];
      F4 t1 = fadd(f, fadd(f, fadd(f, fadd(f, fmul(f, fmul(f, a, b), eq[3][i]), fmul(f, a, eq[0][i])),
                                   fmul(f, b, eq[1][i])),
                           fmul(f, c, eq[2][i])),
                   eq[4][i]);
      const F4 bx = fmul(f, beta, x);
      F4 t2 = fmul(f, fmul(f, fadd(f, fadd(f, a, bx), gamma), fadd(f, fadd(f, b, fmul(f, bx, k1)), gamma)),
                   fadd(f, fadd(f, c, fmul(f, bx, k2)), gamma));
      t2 = fmul(f, t2, z);
      F4 t3 = fmul(f, fmul(f, fadd(f, fadd(f, a, fmul(f, beta, es[0][i])), gamma),
                           fadd(f, fadd(f, b, fmul(f, beta, es[1][i])), gamma)),
                   fadd(f, fadd(f, c, fmul(f, beta, es[2][i])), gamma));
      t3 = fmul(f, t3, zw);
      const F4 t23 = fmul(f, fsub(f, t2, t3), alpha);
      const F4 t4 = fmul(f, fmul(f, fsub(f, z, f.one), el1[i]), alpha2);
      T[i] = fmul(f, fadd(f, fadd(f, t1, t23), t4), zh_inv[i & 3]);
    }
  });
  ntt(T, omegaN, true, threads);
  {
    F4 x = f.one;
    for (size_t j = 0; j < N; ++j) {
      T[j] = fmul(f, T[j], x);
      x = fmul(f, x, g_inv);
    }
  }
  for (size_t j = 3 * m; j < N; ++j)
    if (!fzero(T[j])) return 1;
  for (int k = 0; k < 3; ++k) {
    std::vector<F4> part(T.begin() + k * m, T.begin() + (k + 1) * m);
    com[4 + k] = msm(pts, part, m, threads);
  }
  // ---- round 4 (plonk.rs:393-422)
  const F4 zw = fmul(f, zc, omega);
  const F4 a_z = horner(A.data(), n + 2, zc), b_z = horner(Bp.data(), n + 2, zc), c_z = horner(Cp.data(), n + 2, zc);
  const F4 s1_z = horner(Sg[0].data(), n, zc), s2_z = horner(Sg[1].data(), n, zc), t_z = horner(T.data(), 3 * m, zc);
  const F4 zw_z = horner(Zx.data(), n + 3, zw), l1_z = horner(L1.data(), n, zc);
  const F4 K2 = fmul(f, fmul(f, fmul(f, fadd(f, fadd(f, a_z, fmul(f, beta, zc)), gamma),
                                     fadd(f, fadd(f, b_z, fmul(f, fmul(f, beta, k1), zc)), gamma)),
                             fadd(f, fadd(f, c_z, fmul(f, fmul(f, beta, k2), zc)), gamma)),
                     alpha);
  const F4 K3 = fmul(f, fmul(f, fadd(f, fadd(f, a_z, fmul(f, beta, s1_z)), gamma),
                             fadd(f, fadd(f, b_z, fmul(f, beta, s2_z)), gamma)),
                     alpha);
  const F4 K4 = fmul(f, l1_z, alpha2);
  std::vector<F4> Rx(std::max(rlen, N), F4{{0, 0, 0, 0}});
  {
    const F4 cz = fadd(f, K2, K4), cab = fmul(f, a_z, b_z);
    for (size_t j = 0; j < n + 3; ++j) {
      F4 acc2 = fmul(f, cz, Zx[j]);
      if (j < n) {
        acc2 = fadd(f, acc2, fmul(f, cab, Q[3][j]));
        acc2 = fadd(f, acc2, fmul(f, a_z, Q[0][j]));
        acc2 = fadd(f, acc2, fmul(f, b_z, Q[1][j]));
        acc2 = fadd(f, acc2, fmul(f, c_z, Q[2][j]));
        acc2 = fadd(f, acc2, Q[4][j]);
        if (mode == 1) acc2 = fadd(f, acc2, fmul(f, fr_neg(fmul(f, fmul(f, beta, zw_z), K3)), Sg[2][j]));
      }
      Rx[j] = acc2;
    }
    if (mode == 0) {  // + (beta z_w(z) K3) z(x) s_sigma_3(x) (plonk.rs:414-416), via the coset
      std::vector<F4> P(N);
      for (size_t i = 0; i < N; ++i) P[i] = fmul(f, ez[i], es[2][i]);
      ntt(P, omegaN, true, threads);
      F4 x = f.one;
      const F4 kk = fmul(f, fmul(f, beta, zw_z), K3);
      for (size_t j = 0; j < N; ++j) {
        Rx[j] = fadd(f, Rx[j], fmul(f, kk, fmul(f, P[j], x)));
        x = fmul(f, x, g_inv);
      }
    }
  }
  const F4 r_z = horner(Rx.data(), rlen, zc);
  // ---- round 5 (plonk.rs:430-446)
  F4 vp[7];
  vp[0] = f.one;
  for (int i = 1; i < 7; ++i) vp[i] = fmul(f, vp[i - 1], v);
  const size_t lnum = std::max(rlen, m);
  std::vector<F4> num(lnum, F4{{0, 0, 0, 0}});
  {
    const F4 zn2 = fr_pow64(zc, n + 2), z2n4 = fr_pow64(zc, 2 * n + 4);
    for (size_t j = 0; j < lnum; ++j) {
      F4 x{{0, 0, 0, 0}};
      if (j < m) {
        x = fadd(f, x, T[j]);
        x = fadd(f, x, fmul(f, zn2, T[m + j]));
        x = fadd(f, x, fmul(f, z2n4, T[2 * m + j]));
      }
      if (j < rlen) x = fadd(f, x, fmul(f, vp[1], Rx[j]));
      if (j < n + 2) {
        x = fadd(f, x, fmul(f, vp[2], A[j]));
        x = fadd(f, x, fmul(f, vp[3], Bp[j]));
        x = fadd(f, x, fmul(f, vp[4], Cp[j]));
      }
      if (j < n) {
        x = fadd(f, x, fmul(f, vp[5], Sg[0][j]));
        x = fadd(f, x, fmul(f, vp[6], Sg[1][j]));
      }
      num[j] = x;
    }
    F4 cst = fadd(f, t_z, fmul(f, vp[1], r_z));
    cst = fadd(f, cst, fmul(f, vp[2], a_z));
    cst = fadd(f, cst, fmul(f, vp[3], b_z));
    cst = fadd(f, cst, fmul(f, vp[4], c_z));
    cst = fadd(f, cst, fmul(f, vp[5], s1_z));
    cst = fadd(f, cst, fmul(f, vp[6], s2_z));
    num[0] = fsub(f, num[0], cst);
  }
  std::vector<F4> Wz, Wzw;
  if (!fzero(synth_div(num.data(), lnum, zc, F4{{0, 0, 0, 0}}, Wz))) return 1;
  com[7] = msm(pts, Wz, lnum - 1, threads);
  if (!fzero(synth_div(Zx.data(), n + 3, zw, zw_z, Wzw))) return 1;
  com[8] = msm(pts, Wzw, n + 2, threads);
  for (int k = 0; k < 9; ++k) store_aff(xyzz_to_aff(com[k]), out_pts + 8 * k);
  const F4 fo[7] = {a_z, b_z, c_z, s1_z, s2_z, r_z, zw_z};
  for (int k = 0; k < 7; ++k) fr_store(fo[k], out_f + 4 * k);
  return 0;
}

// mul_ntt (fft.rs:109-132) over Fr with the iterative NTT on `threads` host threads (the
// all-core config-3 CPU baseline; oracle_fr_mul_ntt is the recursion-faithful one-core form)
int oracle_fr_mul_ntt_par(const uint64_t* a, size_t la, const uint64_t* b, size_t lb, const uint64_t* omega, int threads,
                          uint64_t* out) {
  const size_t n = la + lb;
  if (n == 0 || (n & (n - 1))) return 1;
  const Field& f = fr();
  std::vector<F4> av(n, F4{{0, 0, 0, 0}}), bv(n, F4{{0, 0, 0, 0}});
  par_for(la, threads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) av[i] = fr_load(a + 4 * i);
  });
  par_for(lb, threads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) bv[i] = fr_load(b + 4 * i);
  });
  const F4 w = fr_load(omega);
  ntt(av, w, false, threads);
  ntt(bv, w, false, threads);
  par_for(n, threads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) av[i] = fmul(f, av[i], bv[i]);
  });
  ntt(av, w, true, threads);
  par_for(n, threads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) fr_store(av[i], out + 4 * i);
  });
  return 0;
}

}  // extern "C"
