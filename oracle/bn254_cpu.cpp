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
#include "fr4.hpp"

namespace {
using namespace bn4;
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


using namespace bn4;

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
