// ORACLE — TEST INFRASTRUCTURE ONLY (see field.hpp header).
// Restates src/fft.rs and src/poly.rs of the reference.
#pragma once
#include <algorithm>
#include <vector>
#include "field.hpp"

namespace oracle {

// ---------------------------------------------------------------- fft.rs
// fft.rs:55-65 CooleyTurkey::new — pows[i] = omega^i by repeated multiplication.
template <class F>
std::vector<F> ct_domain(F omega, size_t size) {
  std::vector<F> pows;
  pows.reserve(size);
  F m = F::one();
  pows.push_back(m);
  for (size_t i = 1; i < size; ++i) { m = m * omega; pows.push_back(m); }
  return pows;
}

// fft.rs:81-87 split: keep every element whose index parity matches `even`.
// Kept allocation-faithful (a fresh vector of references per call) because the
// recursion is also the CPU timing baseline.
template <class F>
std::vector<const F*> ct_split(const std::vector<const F*>& v, bool even) {
  std::vector<const F*> out;
  for (size_t i = 0; i < v.size(); ++i)
    if (((i % 2) == 0) == even) out.push_back(v[i]);
  return out;
}

// fft.rs:90-106 cooley_tukey_fft — recursive radix-2 DIT, natural order in/out.
template <class F>
std::vector<F> ct_fft_rec(const std::vector<const F*>& vals, const std::vector<const F*>& domain) {
  if (vals.size() == 1) return std::vector<F>{*vals[0]};
  std::vector<const F*> half_domain = ct_split(domain, true);
  std::vector<F> l = ct_fft_rec(ct_split(vals, true), half_domain);
  std::vector<F> r = ct_fft_rec(ct_split(vals, false), half_domain);
  std::vector<F> o(vals.size(), F::zero());
  size_t h = vals.size() / 2;
  for (size_t i = 0; i < l.size(); ++i) {
    F y_times_root = r[i] * *domain[i];  // fft.rs:100
    o[i] = l[i] + y_times_root;          // fft.rs:101
    o[i + h] = l[i] - y_times_root;      // fft.rs:102
  }
  return o;
}

// fft.rs:66-70 CooleyTurkey::fft
template <class F>
std::vector<F> ct_fft(const std::vector<F>& pows, const std::vector<F>& values) {
  std::vector<const F*> v, d;
  v.reserve(values.size()); d.reserve(pows.size());
  for (auto& x : values) v.push_back(&x);
  for (auto& x : pows) d.push_back(&x);
  return ct_fft_rec(v, d);
}

// fft.rs:71-78 CooleyTurkey::fft_inv = fft(freq), then [v0, v_{n-1}, ..., v1] * n^-1.
// n^-1 failing mirrors the `unwrap()` panic at fft.rs:73 (reported by `ok`).
template <class F>
std::vector<F> ct_fft_inv(const std::vector<F>& pows, const std::vector<F>& freq, bool& ok) {
  std::vector<F> vals = ct_fft(pows, freq);
  F ninv = F::from_u64((uint64_t)freq.size()).inv(ok);
  std::vector<F> out;
  if (!ok) return out;
  out.reserve(vals.size());
  out.push_back(ninv * vals[0]);
  for (size_t i = vals.size() - 1; i >= 1; --i) out.push_back(ninv * vals[i]);
  return out;
}

// fft.rs:27-49 VandermondeMatrix FFT: row n of the matrix is omega^(n*m).
template <class F>
std::vector<F> vandermonde_fft(F omega, const std::vector<F>& values) {
  size_t n = values.size();
  std::vector<F> out(n, F::zero());
  for (size_t r = 0; r < n; ++r) {
    F acc = F::zero();
    for (size_t c = 0; c < n; ++c) acc = acc + omega.pow((uint64_t)(r * c)) * values[c];
    out[r] = acc;
  }
  return out;
}

// fft.rs:109-132 mul_ntt: zero-pad both to la+lb, fft, pointwise, fft_inv.
// Output has la+lb entries and is NOT normalised (the caller wraps it in Poly::new).
template <class F>
std::vector<F> mul_ntt(const std::vector<F>& pows, std::vector<F> a, std::vector<F> b, bool& ok) {
  size_t sum = a.size() + b.size();
  a.resize(sum, F::zero());
  b.resize(sum, F::zero());
  std::vector<F> af = ct_fft(pows, a), bf = ct_fft(pows, b), cf;
  cf.reserve(af.size());
  for (size_t i = 0; i < af.size(); ++i) cf.push_back(af[i] * bf[i]);
  return ct_fft_inv(pows, cf, ok);
}

// Iterative in-place radix-2 NTT (bit reversal + butterflies). NOT the reference's
// algorithm: a fast checker for large n. Parity-checked against ct_fft in tests.
template <class F>
void iter_ntt(std::vector<F>& a, F omega) {
  size_t n = a.size();
  for (size_t i = 1, j = 0; i < n; ++i) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
  for (size_t len = 2; len <= n; len <<= 1) {
    F wl = omega.pow((uint64_t)(n / len));
    std::vector<F> tw(len / 2);
    F w = F::one();
    for (size_t k = 0; k < len / 2; ++k) { tw[k] = w; w = w * wl; }
    for (size_t i = 0; i < n; i += len)
      for (size_t k = 0; k < len / 2; ++k) {
        F u = a[i + k], v = a[i + k + len / 2] * tw[k];
        a[i + k] = u + v;
        a[i + k + len / 2] = u - v;
      }
  }
}

// ---------------------------------------------------------------- poly.rs
// Dense coefficient vector, c0 first (poly.rs:11-21).
template <class F>
struct Poly {
  std::vector<F> c;
  Poly() : c{F::zero()} {}
  explicit Poly(std::vector<F> v) : c(std::move(v)) { normalize(); }
  static Poly zero() { return Poly(std::vector<F>{F::zero()}); }  // poly.rs:34-36
  static Poly one() { return Poly(std::vector<F>{F::one()}); }    // poly.rs:39-41
  static Poly from_i64(const std::vector<int64_t>& v) {            // poly.rs:24-26
    std::vector<F> c;
    for (auto x : v) c.push_back(F::from_i64(x));
    return Poly(c);
  }
  // poly.rs:96-105 normalize: strip trailing zeros, keep at least one coefficient.
  void normalize() {
    if (c.empty()) { c.push_back(F::zero()); return; }
    if (c.size() > 1 && c.back().is_zero()) {
      size_t k = c.size();
      while (k > 0 && c[k - 1].is_zero()) --k;
      c.resize(k == 0 ? 1 : k, F::zero());
    }
  }
  size_t degree() const { return c.size() - 1; }                      // poly.rs:91-93
  bool is_zero() const { return c.size() == 1 && c[0].is_zero(); }   // poly.rs:108-110
  // poly.rs:113-119 set
  void set(size_t i, F p) {
    if (c.size() < i + 1) c.resize(i + 1, F::zero());
    c[i] = p;
    normalize();
  }
  // poly.rs:71-79 eval: y = c0; x_pow accumulates x^i (not Horner).
  F eval(F x) const {
    F x_pow = F::one();
    F y = c[0];
    for (size_t i = 1; i < c.size(); ++i) { x_pow = x_pow * x; y = y + x_pow * c[i]; }
    return y;
  }
  // poly.rs:165-176 AddAssign<&Poly>
  Poly& operator+=(const Poly& r) {
    size_t m = std::max(c.size(), r.c.size());
    for (size_t i = 0; i < m; ++i) {
      if (i >= c.size()) c.push_back(r.c[i]);
      else if (i < r.c.size()) c[i] = c[i] + r.c[i];
    }
    normalize();
    return *this;
  }
  // poly.rs:192-203 SubAssign<&Poly>. Quirk kept: when rhs is longer the extra
  // coefficients are pushed with a + sign (poly.rs:196), exactly as the reference.
  Poly& operator-=(const Poly& r) {
    size_t m = std::max(c.size(), r.c.size());
    for (size_t i = 0; i < m; ++i) {
      if (i >= c.size()) c.push_back(r.c[i]);
      else if (i < r.c.size()) c[i] = c[i] - r.c[i];
    }
    normalize();
    return *this;
  }
  Poly& operator+=(F r) { c[0] = c[0] + r; normalize(); return *this; }  // poly.rs:178-183
  Poly& operator-=(F r) { c[0] = c[0] - r; normalize(); return *this; }  // poly.rs:185-190
  // poly.rs:220-228 MulAssign<&F>: zero scalar -> Poly::zero(), no normalisation otherwise.
  Poly& operator*=(F r) {
    if (r.is_zero()) *this = zero();
    else for (auto& x : c) x = x * r;
    return *this;
  }
  bool operator==(const Poly& o) const {
    if (c.size() != o.c.size()) return false;
    for (size_t i = 0; i < c.size(); ++i) if (c[i] != o.c[i]) return false;
    return true;
  }
};

template <class F> Poly<F> operator+(Poly<F> a, const Poly<F>& b) { a += b; return a; }
template <class F> Poly<F> operator-(Poly<F> a, const Poly<F>& b) { a -= b; return a; }
template <class F> Poly<F> operator+(Poly<F> a, F b) { a += b; return a; }
template <class F> Poly<F> operator-(Poly<F> a, F b) { a -= b; return a; }
template <class F> Poly<F> operator*(Poly<F> a, F b) { a *= b; return a; }

// poly.rs:205-218 schoolbook product, result length l+r then normalised.
template <class F>
Poly<F> operator*(const Poly<F>& a, const Poly<F>& b) {
  std::vector<F> m(a.c.size() + b.c.size(), F::zero());
  for (size_t i = 0; i < a.c.size(); ++i)
    for (size_t j = 0; j < b.c.size(); ++j) m[i + j] = m[i + j] + a.c[i] * b.c[j];
  Poly<F> p;
  p.c = std::move(m);
  p.normalize();
  return p;
}

// poly.rs:230-247 long division -> (q, r).
template <class F>
void poly_div(const Poly<F>& num, const Poly<F>& den, Poly<F>& q, Poly<F>& r) {
  q = Poly<F>::zero();
  r = num;
  while (!r.is_zero() && r.degree() >= den.degree()) {
    F lead_r = r.c.back();
    F lead_d = den.c.back();
    Poly<F> t = Poly<F>::zero();
    t.set(r.c.size() - den.c.size(), lead_r * lead_d.inv_unwrap());
    q += t;
    r -= den * t;
  }
  q.normalize();
  r.normalize();
}

// poly.rs:64-68 z(points) = prod (x - p_i)
template <class F>
Poly<F> poly_z(const std::vector<F>& pts) {
  Poly<F> acc = Poly<F>::one();
  for (auto& x : pts) acc = acc * Poly<F>(std::vector<F>{-x, F::one()});
  return acc;
}

}  // namespace oracle
