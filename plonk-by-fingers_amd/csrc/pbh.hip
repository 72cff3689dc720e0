// Plonk-by-hand types on the GPU (BASELINE config 1) and the prover that drives the
// hot path. The toy curve of the reference — G1 y^2 = x^3 + 3 over F101 with an order-17
// subgroup (src/pbh/g1.rs), G2 over F101[u]/(u^2+2) (g2.rs), GT (gt.rs) and the reduced
// Tate pairing (pairing.rs) — as batched kernels; and Plonk::prove / Plonk::verify
// (src/plonk.rs:191-650) as host code whose hot steps run on the GPU:
//   interpolate_at_h  -> libpbf INTT   (plonk.rs:177-179 == natural-order INTT)
//   SRS::create       -> pbh_g1_mul_kernel (plonk.rs:35-48)
//   SRS::eval_at_s    -> pbh_msm_kernel    (plonk.rs:51-58)
//   Poly::eval        -> libpbf poly eval  (poly.rs:71-79), batched per round
//   Pairing::pairing  -> pbh_pairing_kernel (pairing.rs:12-47)
// The small polynomial products/divisions stay on the host (<= 20 coefficients).
#include <array>
#include <string>
#include <vector>
#include "../../include/pbf.h"
#include "internal.hpp"

namespace pbh {

constexpr uint32_t P = 101;  // GF (G1 base field)
constexpr uint32_t H = 17;   // HF (scalar field)

__host__ __device__ inline uint32_t md(int64_t x, uint32_t m) {
  int64_t r = x % (int64_t)m;
  return (uint32_t)(r < 0 ? r + m : r);
}
__host__ __device__ inline uint32_t pw(uint32_t a, uint32_t e, uint32_t m) {
  uint32_t r = 1 % m;
  a %= m;
  while (e) {
    if (e & 1) r = r * a % m;
    a = a * a % m;
    e >>= 1;
  }
  return r;
}
// x^-1 in F101 (x != 0 asserted by the callers' branch structure)
__host__ __device__ inline uint32_t inv101(uint32_t x) { return pw(x, P - 2, P); }

struct G1 {
  uint32_t x, y, inf;
};
struct G2 {
  uint32_t a, b;
};
struct GT {
  uint32_t a, b;
};

__host__ __device__ inline bool g1_eq(const G1& p, const G1& q) { return p.x == q.x && p.y == q.y && p.inf == q.inf; }
__host__ __device__ inline G1 g1_neg(const G1& p) { return p.inf ? p : G1{p.x, md(-(int64_t)p.y, P), 0}; }
// g1.rs:119-144
__host__ __device__ inline G1 g1_add(const G1& p, const G1& q) {
  if (p.inf) return q;
  if (q.inf) return p;
  if (g1_eq(p, g1_neg(q))) return G1{0, 0, 1};
  uint32_t m;
  if (g1_eq(p, q)) {
    m = (3 * p.x % P * p.x % P) * inv101(2 * p.y % P) % P;
    const uint32_t x = md((int64_t)m * m - 2 * p.x, P);
    return G1{x, md((int64_t)m * md(3 * (int64_t)p.x - (int64_t)m * m, P) - p.y, P), 0};
  }
  m = md((int64_t)q.y - p.y, P) * inv101(md((int64_t)q.x - p.x, P)) % P;
  const uint32_t x = md((int64_t)m * m - p.x - q.x, P);
  return G1{x, md((int64_t)m * md((int64_t)p.x - x, P) - p.y, P), 0};
}
// g1.rs:146-168 LSB-first double-and-add
__host__ __device__ inline G1 g1_mul(const G1& p, uint32_t s) {
  if (s == 0 || p.inf) return G1{0, 0, 1};
  bool have = false;
  G1 r{0, 0, 1}, b = p;
  while (s) {
    if (s & 1) { r = have ? g1_add(r, b) : b; have = true; }
    s >>= 1;
    b = g1_add(b, b);
  }
  return r;
}
// g2.rs:58-80 (no identity handling; `bad` set where the reference would panic)
__host__ __device__ inline G2 g2_add(const G2& p, const G2& q, bool* bad) {
  if (p.a == q.a && p.b == q.b) {
    if (p.b == 0) { *bad = true; return p; }
    const uint32_t mu = 3 * p.a % P * p.a % P * inv101(2 * p.b % P) % P;
    const uint32_t u2inv = inv101(P - 2);
    const uint32_t m2 = mu * mu % P * u2inv % P;
    return G2{md((int64_t)m2 - 2 * p.a, P), md((int64_t)u2inv * mu % P * md(3 * (int64_t)p.a - m2, P) - p.b, P)};
  }
  const uint32_t da = md((int64_t)q.a - p.a, P);
  if (da == 0) { *bad = true; return p; }
  const uint32_t lu = md((int64_t)q.b - p.b, P) * inv101(da) % P;
  const uint32_t l2 = lu * lu % P * (P - 2) % P;
  const uint32_t a = md((int64_t)l2 - p.a - q.a, P);
  return G2{a, md((int64_t)lu * md((int64_t)p.a - a, P) - p.b, P)};
}
// g2.rs:82-101 (panics on 0 in the reference)
__host__ __device__ inline G2 g2_mul(const G2& p, uint32_t s, bool* bad) {
  if (s == 0) { *bad = true; return p; }
  bool have = false;
  G2 r = p, b = p;
  while (s) {
    if (s & 1) { r = have ? g2_add(r, b, bad) : b; have = true; }
    s >>= 1;
    b = g2_add(b, b, bad);
  }
  return r;
}
// gt.rs:61-69
__host__ __device__ inline GT gt_mul(const GT& x, const GT& y) {
  return GT{md((int64_t)x.a * y.a - 2 * (int64_t)(x.b * y.b % P), P), (x.a * y.b + x.b * y.a) % P};
}
// gt.rs:31-60 equals x^n exactly: conjugation is the Frobenius of F101[u]/(u^2+2)
// (u^101 = (-2)^50 u = -u), so square-and-multiply gives the same element.
__host__ __device__ inline GT gt_pow(GT x, uint32_t n) {
  GT r{1, 0};
  while (n) {
    if (n & 1) r = gt_mul(r, x);
    x = gt_mul(x, x);
    n >>= 1;
  }
  return r;
}
// pairing.rs:23-47 recursion unrolled from the bottom: r = 17 -> 16 -> 8 -> 4 -> 2 -> 1
__host__ __device__ inline GT line_at(const G1& a, const G1& b, const G2& q) {
  const uint32_t m = md((int64_t)b.x - a.x, P), n = md((int64_t)b.y - a.y, P);
  const uint32_t x = n, y = md(-(int64_t)m, P);
  const uint32_t c = md((int64_t)m * a.y - (int64_t)n * a.x, P);
  return GT{(q.a * x + c) % P, q.b * y % P};
}
__host__ __device__ inline GT pairing(const G1& p, const G2& q) {
  // chain of r values of pairing_f(17, ...): odd r -> r-1, even r -> r/2
  uint32_t chain[8];
  int len = 0;
  for (uint32_t r = 17; r > 1; r = (r % 2) ? r - 1 : r / 2) chain[len++] = r;
  GT f{1, 0};
  for (int i = len - 1; i >= 0; --i) {
    const uint32_t r = chain[i];
    if (r % 2) {
      f = gt_mul(f, line_at(g1_mul(p, r - 1), p, q));
    } else {
      const uint32_t h = r / 2;
      const G1 ph = g1_mul(p, h);
      f = gt_mul(gt_mul(f, f), line_at(ph, g1_mul(g1_mul(g1_neg(p), h), 2), q));
    }
  }
  return gt_pow(f, (P * P - 1) / 17);  // pairing.rs:12-20: (p^k - 1) / r = 600
}

__global__ void pbh_g1_mul_kernel(const uint32_t* pts, const uint32_t* s, uint32_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G1 r = g1_mul(G1{pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]}, s[i] % P);
  out[3 * i] = r.x; out[3 * i + 1] = r.y; out[3 * i + 2] = r.inf;
}

// SRS::eval_at_s: sum_i pts[i] * s[i] (s already mapped by gf, plonk.rs:51-58); one workgroup
__global__ void __launch_bounds__(256) pbh_msm_kernel(const uint32_t* pts, const uint32_t* s, uint32_t n, uint32_t* out) {
  __shared__ G1 red[256];
  G1 acc{0, 0, 1};
  for (uint32_t i = threadIdx.x; i < n; i += 256)
    acc = g1_add(acc, g1_mul(G1{pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]}, s[i] % P));
  red[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] = g1_add(red[threadIdx.x], red[threadIdx.x + st]);
    __syncthreads();
  }
  if (threadIdx.x == 0) { out[0] = red[0].x; out[1] = red[0].y; out[2] = red[0].inf; }
}

__global__ void pbh_pairing_kernel(const uint32_t* g1, const uint32_t* g2, uint32_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const GT r = pairing(G1{g1[3 * i], g1[3 * i + 1], g1[3 * i + 2]}, G2{g2[2 * i], g2[2 * i + 1]});
  out[2 * i] = r.a; out[2 * i + 1] = r.b;
}

__global__ void pbh_g2_mul_kernel(const uint32_t* pts, const uint32_t* s, uint32_t* out, uint32_t* bad, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool b = false;
  const G2 r = g2_mul(G2{pts[2 * i], pts[2 * i + 1]}, s[i] % P, &b);
  out[2 * i] = r.a; out[2 * i + 1] = r.b;
  if (b) atomicOr(bad, 1u);
}

__global__ void pbh_gt_pow_kernel(const uint32_t* x, const uint32_t* e, uint32_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const GT r = gt_pow(GT{x[2 * i], x[2 * i + 1]}, e[i]);
  out[2 * i] = r.a; out[2 * i + 1] = r.b;
}

}  // namespace pbh

// ------------------------------------------------------------------ host side
using pbf::fail;

namespace {

bool g1_valid(const uint32_t* p) {
  if (p[2]) return true;
  return p[0] < pbh::P && p[1] < pbh::P && pbh::pw(p[1], 2, pbh::P) == (pbh::pw(p[0], 3, pbh::P) + 3) % pbh::P;
}

// Device round trip helper: copy n*w words in, launch, copy back. The buffers are the
// context's own named buffers (freed by pbf_ctx_destroy), so contexts share nothing.
struct Dev {
  pbf::DevBuf &a, &b, &c, &d;
};
Dev dev_for(pbf_ctx* ctx) {
  return Dev{ctx->buf("pbh.a"), ctx->buf("pbh.b"), ctx->buf("pbh.c"), ctx->buf("pbh.d")};
}

int gpu_g1_mul(pbf_ctx* ctx, const std::vector<uint32_t>& pts, const std::vector<uint32_t>& s, std::vector<uint32_t>& out) {
  const uint32_t n = (uint32_t)s.size();
  if (n == 0) { out.clear(); return 0; }
  Dev d = dev_for(ctx);
  int rc;
  if ((rc = d.a.ensure(pts.size() * 4)) || (rc = d.b.ensure(s.size() * 4)) || (rc = d.c.ensure(pts.size() * 4))) return rc;
  hipStream_t st = ctx->host_stream();
  PBF_HIP(hipMemcpyAsync(d.a.p, pts.data(), pts.size() * 4, hipMemcpyHostToDevice, st));
  PBF_HIP(hipMemcpyAsync(d.b.p, s.data(), s.size() * 4, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(pbh::pbh_g1_mul_kernel, dim3((n + 255) / 256), dim3(256), 0, st, (const uint32_t*)d.a.p,
                     (const uint32_t*)d.b.p, (uint32_t*)d.c.p, n);
  PBF_HIP(hipGetLastError());
  out.resize(pts.size());
  PBF_HIP(hipMemcpyAsync(out.data(), d.c.p, pts.size() * 4, hipMemcpyDeviceToHost, st));
  PBF_HIP(hipStreamSynchronize(st));
  return 0;
}

int gpu_msm(pbf_ctx* ctx, const std::vector<uint32_t>& pts, const std::vector<uint32_t>& s, uint32_t out[3]) {
  const uint32_t n = (uint32_t)s.size();
  Dev d = dev_for(ctx);
  int rc;
  if ((rc = d.a.ensure(pts.size() * 4 + 4)) || (rc = d.b.ensure(s.size() * 4 + 4)) || (rc = d.c.ensure(16))) return rc;
  hipStream_t st = ctx->host_stream();
  if (n) {
    PBF_HIP(hipMemcpyAsync(d.a.p, pts.data(), 3 * n * 4, hipMemcpyHostToDevice, st));
    PBF_HIP(hipMemcpyAsync(d.b.p, s.data(), n * 4, hipMemcpyHostToDevice, st));
  }
  hipLaunchKernelGGL(pbh::pbh_msm_kernel, dim3(1), dim3(256), 0, st, (const uint32_t*)d.a.p, (const uint32_t*)d.b.p, n,
                     (uint32_t*)d.c.p);
  PBF_HIP(hipGetLastError());
  PBF_HIP(hipMemcpyAsync(out, d.c.p, 12, hipMemcpyDeviceToHost, st));
  PBF_HIP(hipStreamSynchronize(st));
  return 0;
}

int gpu_pairing(pbf_ctx* ctx, const std::vector<uint32_t>& g1, const std::vector<uint32_t>& g2, std::vector<uint32_t>& out) {
  const uint32_t n = (uint32_t)(g2.size() / 2);
  Dev d = dev_for(ctx);
  int rc;
  if ((rc = d.a.ensure(g1.size() * 4 + 4)) || (rc = d.b.ensure(g2.size() * 4 + 4)) || (rc = d.c.ensure(g2.size() * 4 + 4)))
    return rc;
  hipStream_t st = ctx->host_stream();
  PBF_HIP(hipMemcpyAsync(d.a.p, g1.data(), g1.size() * 4, hipMemcpyHostToDevice, st));
  PBF_HIP(hipMemcpyAsync(d.b.p, g2.data(), g2.size() * 4, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(pbh::pbh_pairing_kernel, dim3((n + 255) / 256), dim3(256), 0, st, (const uint32_t*)d.a.p,
                     (const uint32_t*)d.b.p, (uint32_t*)d.c.p, n);
  PBF_HIP(hipGetLastError());
  out.resize(2 * n);
  PBF_HIP(hipMemcpyAsync(out.data(), d.c.p, 2 * n * 4, hipMemcpyDeviceToHost, st));
  PBF_HIP(hipStreamSynchronize(st));
  return 0;
}

// ---- host polynomials over F17 with the reference's semantics (poly.rs)
typedef std::vector<uint32_t> Pl;
constexpr uint32_t M = pbh::H;
uint32_t fa(uint32_t a, uint32_t b) { return (a + b) % M; }
uint32_t fs(uint32_t a, uint32_t b) { return (a + M - b) % M; }
uint32_t fm(uint32_t a, uint32_t b) { return a * b % M; }
uint32_t finv(uint32_t a) { return pbh::pw(a, M - 2, M); }
void norm(Pl& p) {  // poly.rs:96-105
  if (p.empty()) p.push_back(0);
  while (p.size() > 1 && p.back() == 0) p.pop_back();
}
Pl mk(Pl v) { norm(v); return v; }
Pl padd(Pl a, const Pl& b) {  // poly.rs:165-176
  for (size_t i = 0; i < std::max(a.size(), b.size()); ++i) {
    if (i >= a.size()) a.push_back(b[i]);
    else if (i < b.size()) a[i] = fa(a[i], b[i]);
  }
  norm(a);
  return a;
}
Pl psub(Pl a, const Pl& b) {  // poly.rs:192-203 (quirk: extra rhs terms pushed with + sign)
  for (size_t i = 0; i < std::max(a.size(), b.size()); ++i) {
    if (i >= a.size()) a.push_back(b[i]);
    else if (i < b.size()) a[i] = fs(a[i], b[i]);
  }
  norm(a);
  return a;
}
Pl pmul(const Pl& a, const Pl& b) {  // poly.rs:205-218
  Pl m(a.size() + b.size(), 0);
  for (size_t i = 0; i < a.size(); ++i)
    for (size_t j = 0; j < b.size(); ++j) m[i + j] = fa(m[i + j], fm(a[i], b[j]));
  norm(m);
  return m;
}
Pl pscale(Pl a, uint32_t s) {  // poly.rs:220-228
  if (s == 0) return Pl{0};
  for (auto& x : a) x = fm(x, s);
  return a;
}
Pl paddc(Pl a, uint32_t c) { a[0] = fa(a[0], c); norm(a); return a; }  // poly.rs:178-183
Pl psubc(Pl a, uint32_t c) { a[0] = fs(a[0], c); norm(a); return a; }  // poly.rs:185-190
bool pdiv(const Pl& num, const Pl& den, Pl& q, Pl& r) {  // poly.rs:230-247
  q = Pl{0};
  r = num;
  auto is_zero = [](const Pl& p) { return p.size() == 1 && p[0] == 0; };
  while (!is_zero(r) && r.size() - 1 >= den.size() - 1) {
    const uint32_t lead_d = den.back();
    if (lead_d == 0) return false;
    Pl t(r.size() - den.size() + 1, 0);
    t.back() = fm(r.back(), finv(lead_d));
    norm(t);
    q = padd(q, t);
    r = psub(r, pmul(den, t));
  }
  norm(q);
  norm(r);
  return true;
}

struct Ctx {
  pbf_ctx* ctx;
  uint32_t omega;
  std::vector<uint32_t> h, k1h, k2h;
  std::vector<uint32_t> g1s;  // SRS, 3 words per point
  uint32_t g2_1[2], g2_s[2];
  Pl zh;
};

// interpolate_at_h (plonk.rs:177-179) on the GPU: the natural-order INTT over H
int interp(const Ctx& c, const std::vector<uint32_t>& v, Pl& out) {
  const size_t n = v.size();
  std::vector<uint64_t> in(v.begin(), v.end()), res(n);
  int rc = pbf_ntt_u64(c.ctx, M, c.omega, in.data(), res.data(), n, 1);
  if (rc) return rc;
  out.assign(res.begin(), res.end());
  norm(out);
  return 0;
}
// Poly::eval at many points on the GPU (poly.rs:71-79)
int evals(const Ctx& c, const Pl& p, const std::vector<uint32_t>& xs, std::vector<uint32_t>& ys) {
  std::vector<uint64_t> cp(p.begin(), p.end()), x(xs.begin(), xs.end()), y(xs.size());
  int rc = pbf_poly_eval_u64(c.ctx, M, cp.data(), cp.size(), x.data(), x.size(), y.data());
  ys.assign(y.begin(), y.end());
  return rc;
}
uint32_t gfmap(uint32_t v) { return v % pbh::P; }  // PlonkByHandTypes::gf (pbh/mod.rs:30-32)
int eval_at_s(const Ctx& c, const Pl& p, uint32_t out[3]) {
  if (p.size() * 3 > c.g1s.size()) return fail(PBF_EINVAL, "polynomial longer than the SRS (plonk.rs:54 index panic)");
  std::vector<uint32_t> pts(c.g1s.begin(), c.g1s.begin() + 3 * p.size()), s(p.size());
  for (size_t i = 0; i < p.size(); ++i) s[i] = gfmap(p[i]);
  return gpu_msm(c.ctx, pts, s, out);
}
uint32_t copy_root(const Ctx& c, uint64_t kind, uint64_t idx) {
  return kind == 0 ? c.h[idx - 1] : kind == 1 ? c.k1h[idx - 1] : c.k2h[idx - 1];
}

}  // namespace

extern "C" {

// Batched toy-curve ops (src/pbh/*.rs). Points as 32-bit words: G1 [x, y, inf], G2 [a, b], GT [a, b].
int pbf_pbh_g1_mul(pbf_ctx* ctx, const uint32_t* pts, const uint32_t* scalars, size_t n, uint32_t* out) {
  if (!ctx || (n && (!pts || !scalars || !out))) return fail(PBF_EINVAL, "null argument");
  for (size_t i = 0; i < n; ++i)
    if (!g1_valid(pts + 3 * i)) return fail(PBF_EINVAL, "point not on the curve");
  std::vector<uint32_t> p(pts, pts + 3 * n), s(scalars, scalars + n), o;
  int rc = gpu_g1_mul(ctx, p, s, o);
  if (rc) return rc;
  std::copy(o.begin(), o.end(), out);
  return PBF_OK;
}

int pbf_pbh_pairing(pbf_ctx* ctx, const uint32_t* g1, const uint32_t* g2, size_t n, uint32_t* out) {
  if (!ctx || (n && (!g1 || !g2 || !out))) return fail(PBF_EINVAL, "null argument");
  for (size_t i = 0; i < n; ++i)
    if (!g1_valid(g1 + 3 * i)) return fail(PBF_EINVAL, "G1 point not on the curve");
  std::vector<uint32_t> a(g1, g1 + 3 * n), b(g2, g2 + 2 * n), o;
  int rc = gpu_pairing(ctx, a, b, o);
  if (rc) return rc;
  std::copy(o.begin(), o.end(), out);
  return PBF_OK;
}

int pbf_pbh_g2_mul(pbf_ctx* ctx, const uint32_t* pts, const uint32_t* scalars, size_t n, uint32_t* out) {
  if (!ctx || (n && (!pts || !scalars || !out))) return fail(PBF_EINVAL, "null argument");
  Dev d = dev_for(ctx);
  int rc;
  if ((rc = d.a.ensure(n * 8 + 8)) || (rc = d.b.ensure(n * 4 + 4)) || (rc = d.c.ensure(n * 8 + 8)) || (rc = d.d.ensure(4)))
    return rc;
  hipStream_t st = ctx->host_stream();
  PBF_HIP(hipMemsetAsync(d.d.p, 0, 4, st));
  PBF_HIP(hipMemcpyAsync(d.a.p, pts, n * 8, hipMemcpyHostToDevice, st));
  PBF_HIP(hipMemcpyAsync(d.b.p, scalars, n * 4, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(pbh::pbh_g2_mul_kernel, dim3((n + 255) / 256), dim3(256), 0, st, (const uint32_t*)d.a.p,
                     (const uint32_t*)d.b.p, (uint32_t*)d.c.p, (uint32_t*)d.d.p, (uint32_t)n);
  PBF_HIP(hipGetLastError());
  uint32_t bad = 0;
  PBF_HIP(hipMemcpyAsync(out, d.c.p, n * 8, hipMemcpyDeviceToHost, st));
  PBF_HIP(hipMemcpyAsync(&bad, d.d.p, 4, hipMemcpyDeviceToHost, st));
  PBF_HIP(hipStreamSynchronize(st));
  if (bad) return fail(PBF_EINVAL, "G2P arithmetic hit a case the reference panics on (g2.rs:58-101)");
  return PBF_OK;
}

int pbf_pbh_gt_pow(pbf_ctx* ctx, const uint32_t* x, const uint32_t* e, size_t n, uint32_t* out) {
  if (!ctx || (n && (!x || !e || !out))) return fail(PBF_EINVAL, "null argument");
  Dev d = dev_for(ctx);
  int rc;
  if ((rc = d.a.ensure(n * 8 + 8)) || (rc = d.b.ensure(n * 4 + 4)) || (rc = d.c.ensure(n * 8 + 8))) return rc;
  hipStream_t st = ctx->host_stream();
  PBF_HIP(hipMemcpyAsync(d.a.p, x, n * 8, hipMemcpyHostToDevice, st));
  PBF_HIP(hipMemcpyAsync(d.b.p, e, n * 4, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(pbh::pbh_gt_pow_kernel, dim3((n + 255) / 256), dim3(256), 0, st, (const uint32_t*)d.a.p,
                     (const uint32_t*)d.b.p, (uint32_t*)d.c.p, (uint32_t)n);
  PBF_HIP(hipGetLastError());
  PBF_HIP(hipMemcpyAsync(out, d.c.p, n * 8, hipMemcpyDeviceToHost, st));
  PBF_HIP(hipStreamSynchronize(st));
  return PBF_OK;
}

// Plonk::prove (+ optional Plonk::verify) over PlonkByHandTypes (pbh/mod.rs:18-33).
// Argument layout is that of oracle/capi.cpp:oracle_pbh_prove (tests compare the two).
int pbf_pbh_prove(pbf_ctx* pctx, size_t n, const uint64_t* gates, const uint64_t* copies, const uint64_t* abc,
                  const uint64_t* chal, const uint64_t* rnd, uint64_t s_in, uint64_t srs_n, uint64_t omega_pows,
                  uint64_t verify_u, uint64_t* out_pts, uint64_t* out_f, int* verified) {
  if (!pctx || !gates || !copies || !abc || !chal || !rnd || !out_pts || !out_f) return fail(PBF_EINVAL, "null argument");
  Ctx c;
  c.ctx = pctx;
  const uint32_t OMEGA = 4, K1 = 2, K2 = 3;
  c.omega = OMEGA;
  // ---- Plonk::new (plonk.rs:120-175)
  for (uint64_t i = 0; i < omega_pows % M; ++i) c.h.push_back(pbh::pw(OMEGA, (uint32_t)i, M));
  for (auto r : c.h) { c.k1h.push_back(fm(r, K1)); c.k2h.push_back(fm(r, K2)); }
  if (c.h.size() != n) return fail(PBF_EINVAL, "the domain H must have n elements (plonk.rs:233 interpolation size)");
  c.zh = Pl{1};
  for (auto x : c.h) c.zh = pmul(c.zh, mk(Pl{fs(0, x), 1}));
  // ---- SRS::create (plonk.rs:35-48) on the GPU
  {
    std::vector<uint32_t> pts, sc;
    uint32_t sp = (uint32_t)(s_in % pbh::P);
    pts.insert(pts.end(), {1, 2, 0});
    sc.push_back(1);
    for (uint64_t i = 0; i < srs_n; ++i) {
      pts.insert(pts.end(), {1, 2, 0});
      sc.push_back(sp);
      sp = sp * (uint32_t)(s_in % pbh::P) % pbh::P;
    }
    int rc = gpu_g1_mul(pctx, pts, sc, c.g1s);
    if (rc) return rc;
    bool bad = false;
    const pbh::G2 g2{36, 31};
    c.g2_1[0] = 36; c.g2_1[1] = 31;
    const pbh::G2 gs = pbh::g2_mul(g2, (uint32_t)(s_in % pbh::P), &bad);
    if (bad) return fail(PBF_EINVAL, "G2P * 0 (g2.rs:99 panic)");
    c.g2_s[0] = gs.a; c.g2_s[1] = gs.b;
  }
  // ---- circuit data
  std::vector<uint32_t> ql, qr, qo, qm, qc, A(n), B(n), C(n);
  for (size_t i = 0; i < n; ++i) {
    ql.push_back((uint32_t)(gates[5 * i] % M)); qr.push_back((uint32_t)(gates[5 * i + 1] % M));
    qo.push_back((uint32_t)(gates[5 * i + 2] % M)); qm.push_back((uint32_t)(gates[5 * i + 3] % M));
    qc.push_back((uint32_t)(gates[5 * i + 4] % M));
    A[i] = (uint32_t)(abc[i] % M); B[i] = (uint32_t)(abc[n + i] % M); C[i] = (uint32_t)(abc[2 * n + i] % M);
  }
  auto cp = [&](int col, size_t i, int f) { return copies[((size_t)col * n + i) * 2 + f]; };
  auto val = [&](uint64_t kind, uint64_t idx) { return kind == 0 ? A[idx - 1] : kind == 1 ? B[idx - 1] : C[idx - 1]; };
  // constraints.rs:198-230 (quirk kept: q_l * b)
  for (size_t i = 0; i < n; ++i) {
    uint32_t r = fa(fa(fa(fa(fm(ql[i], A[i]), fm(ql[i], B[i])), fm(qo[i], C[i])), fm(fm(qm[i], A[i]), B[i])), qc[i]);
    if (r) return fail(PBF_EINVAL, "constraints not satisfied (plonk.rs:199 assert)");
  }
  for (size_t i = 0; i < n; ++i)
    if (A[i] != val(cp(0, i, 0), cp(0, i, 1)) || B[i] != val(cp(1, i, 0), cp(1, i, 1)) ||
        C[i] != val(cp(2, i, 0), cp(2, i, 1)))
      return fail(PBF_EINVAL, "copy constraints not satisfied (plonk.rs:199 assert)");
  const uint32_t alpha = (uint32_t)(chal[0] % M), beta = (uint32_t)(chal[1] % M), gamma = (uint32_t)(chal[2] % M),
                 z = (uint32_t)(chal[3] % M), v = (uint32_t)(chal[4] % M);
  uint32_t rd[9];
  for (int i = 0; i < 9; ++i) rd[i] = (uint32_t)(rnd[i] % M);
  std::vector<uint32_t> sig[3];
  for (int col = 0; col < 3; ++col)
    for (size_t i = 0; i < n; ++i) sig[col].push_back(copy_root(c, cp(col, i, 0), cp(col, i, 1)));
  int rc;
  Pl f_a, f_b, f_c, q_o, q_m, q_l, q_r, q_c, ss1, ss2, ss3;
  if ((rc = interp(c, A, f_a)) || (rc = interp(c, B, f_b)) || (rc = interp(c, C, f_c)) || (rc = interp(c, qo, q_o)) ||
      (rc = interp(c, qm, q_m)) || (rc = interp(c, ql, q_l)) || (rc = interp(c, qr, q_r)) || (rc = interp(c, qc, q_c)) ||
      (rc = interp(c, sig[0], ss1)) || (rc = interp(c, sig[1], ss2)) || (rc = interp(c, sig[2], ss3)))
    return rc;
  uint32_t pts[9][3];
  // ---- round 1 (plonk.rs:248-257)
  Pl a_x = padd(pmul(mk(Pl{rd[1], rd[0]}), c.zh), f_a);
  Pl b_x = padd(pmul(mk(Pl{rd[3], rd[2]}), c.zh), f_b);
  Pl c_x = padd(pmul(mk(Pl{rd[5], rd[4]}), c.zh), f_c);
  if ((rc = eval_at_s(c, a_x, pts[0])) || (rc = eval_at_s(c, b_x, pts[1])) || (rc = eval_at_s(c, c_x, pts[2]))) return rc;
  // ---- round 2 (plonk.rs:267-313): sigma evaluations at w^(i-1) batched on the GPU
  std::vector<uint32_t> wpows;
  for (size_t i = 1; i < n; ++i) wpows.push_back(pbh::pw(OMEGA, (uint32_t)(i - 1), M));
  std::vector<uint32_t> e1, e2, e3;
  if (!wpows.empty() && ((rc = evals(c, ss1, wpows, e1)) || (rc = evals(c, ss2, wpows, e2)) || (rc = evals(c, ss3, wpows, e3))))
    return rc;
  std::vector<uint32_t> acc{1};
  for (size_t i = 1; i < n; ++i) {
    const uint32_t a = A[i - 1], b = B[i - 1], cc = C[i - 1], wp = wpows[i - 1];
    const uint32_t dend = fm(fm(fa(fa(a, fm(beta, wp)), gamma), fa(fa(b, fm(fm(beta, K1), wp)), gamma)),
                             fa(fa(cc, fm(fm(beta, K2), wp)), gamma));
    const uint32_t dsor = fm(fm(fa(fa(a, fm(beta, e1[i - 1])), gamma), fa(fa(b, fm(beta, e2[i - 1])), gamma)),
                             fa(fa(cc, fm(beta, e3[i - 1])), gamma));
    if (dsor == 0) return fail(PBF_EINVAL, "division by zero in the accumulator (plonk.rs:297 unwrap)");
    acc.push_back(fm(acc[i - 1], fm(dend, finv(dsor))));
  }
  Pl acc_x;
  if ((rc = interp(c, acc, acc_x))) return rc;
  Pl z_x = padd(pmul(mk(Pl{rd[8], rd[7], rd[6]}), c.zh), acc_x);
  if ((rc = eval_at_s(c, z_x, pts[3]))) return rc;
  // ---- round 3 (plonk.rs:328-385)
  std::vector<uint32_t> lv(c.h.size(), 0);
  lv[0] = 1;
  Pl l_1_x;
  if ((rc = interp(c, lv, l_1_x))) return rc;
  Pl zo(z_x.size());
  for (size_t i = 0; i < z_x.size(); ++i) zo[i] = fm(z_x[i], pbh::pw(OMEGA, (uint32_t)i, M));
  Pl z_omega_x = mk(zo);
  Pl t1 = padd(padd(padd(padd(padd(pmul(pmul(a_x, b_x), q_m), pmul(a_x, q_l)), pmul(b_x, q_r)), pmul(c_x, q_o)), Pl{0}), q_c);
  Pl t2 = pmul(pmul(pmul(pscale(padd(a_x, mk(Pl{gamma, beta})), alpha), padd(b_x, mk(Pl{gamma, fm(beta, K1)}))),
                    padd(c_x, mk(Pl{gamma, fm(beta, K2)}))), z_x);
  Pl t3 = pmul(pmul(pmul(pscale(paddc(padd(a_x, pscale(ss1, beta)), gamma), alpha), paddc(padd(b_x, pscale(ss2, beta)), gamma)),
                    paddc(padd(c_x, pscale(ss3, beta)), gamma)), z_omega_x);
  Pl t4 = pmul(pscale(padd(z_x, mk(Pl{fs(0, 1)})), fm(alpha, alpha)), l_1_x);
  Pl t_x, rem;
  if (!pdiv(padd(psub(padd(t1, t2), t3), t4), c.zh, t_x, rem)) return fail(PBF_EINVAL, "division by Z_H failed");
  if (!(rem.size() == 1 && rem[0] == 0)) return fail(PBF_EINVAL, "t(x) remainder != 0 (plonk.rs:370 assert)");
  const size_t sp = n + 2;  // plonk.rs:376-378 (the reference hard-codes n = 4: offsets 0/6/12/18)
  auto chunk = [&](size_t lo) {
    Pl out;
    for (size_t i = lo; i < lo + sp; ++i) out.push_back(i < t_x.size() ? t_x[i] : 0);
    return mk(out);
  };
  Pl t_hi = chunk(2 * sp), t_mid = chunk(sp), t_lo = chunk(0);
  if ((rc = eval_at_s(c, t_lo, pts[4])) || (rc = eval_at_s(c, t_mid, pts[5])) || (rc = eval_at_s(c, t_hi, pts[6]))) return rc;
  // ---- round 4 (plonk.rs:393-422): the seven evaluations at z on the GPU
  std::vector<uint32_t> one_z{z}, ev;
  uint32_t a_z, b_z, c_z, s1z, s2z, t_z, zwz;
  {
    const Pl* ps[7] = {&a_x, &b_x, &c_x, &ss1, &ss2, &t_x, &z_omega_x};
    uint32_t* dst[7] = {&a_z, &b_z, &c_z, &s1z, &s2z, &t_z, &zwz};
    for (int i = 0; i < 7; ++i) {
      if ((rc = evals(c, *ps[i], one_z, ev))) return rc;
      *dst[i] = ev[0];
    }
  }
  Pl r1 = padd(padd(padd(padd(pscale(pscale(q_m, a_z), b_z), pscale(q_l, a_z)), pscale(q_r, b_z)), pscale(q_o, c_z)), q_c);
  Pl r2 = pscale(z_x, fm(fm(fm(fa(fa(a_z, fm(beta, z)), gamma), fa(fa(b_z, fm(fm(beta, K1), z)), gamma)),
                            fa(fa(c_z, fm(fm(beta, K2), z)), gamma)), alpha));
  Pl r3 = pscale(pmul(z_x, pscale(pscale(ss3, beta), zwz)),
                 fm(fm(fa(fa(a_z, fm(beta, s1z)), gamma), fa(fa(b_z, fm(beta, s2z)), gamma)), alpha));
  uint32_t l1z;
  if ((rc = evals(c, l_1_x, one_z, ev))) return rc;
  l1z = ev[0];
  Pl r4 = pscale(pscale(z_x, l1z), fm(alpha, alpha));
  Pl r_x = padd(padd(padd(r1, r2), r3), r4);
  if ((rc = evals(c, r_x, one_z, ev))) return rc;
  const uint32_t r_z = ev[0];
  // ---- round 5 (plonk.rs:430-446)
  auto vp = [&](uint32_t e) { return pbh::pw(v, e, M); };
  Pl w = psubc(padd(padd(t_lo, pscale(t_mid, pbh::pw(z, (uint32_t)(n + 2), M))), pscale(t_hi, pbh::pw(z, (uint32_t)(2 * n + 4), M))), t_z);
  w = padd(w, pscale(psubc(r_x, r_z), v));
  w = padd(w, pscale(psubc(a_x, a_z), vp(2)));
  w = padd(w, pscale(psubc(b_x, b_z), vp(3)));
  w = padd(w, pscale(psubc(c_x, c_z), vp(4)));
  w = padd(w, pscale(psubc(ss1, s1z), vp(5)));
  w = padd(w, pscale(psubc(ss2, s2z), vp(6)));
  Pl w_z_x, w_zw_x;
  if (!pdiv(w, mk(Pl{fs(0, z), 1}), w_z_x, rem) || !(rem.size() == 1 && rem[0] == 0))
    return fail(PBF_EINVAL, "w_z remainder != 0 (plonk.rs:438 assert)");
  if (!pdiv(psubc(z_x, zwz), mk(Pl{fs(0, fm(z, OMEGA)), 1}), w_zw_x, rem) || !(rem.size() == 1 && rem[0] == 0))
    return fail(PBF_EINVAL, "w_zw remainder != 0 (plonk.rs:442 assert)");
  if ((rc = eval_at_s(c, w_z_x, pts[7])) || (rc = eval_at_s(c, w_zw_x, pts[8]))) return rc;
  for (int i = 0; i < 9; ++i)
    for (int k = 0; k < 3; ++k) out_pts[3 * i + k] = pts[i][k];
  const uint32_t fsv[7] = {a_z, b_z, c_z, s1z, s2z, r_z, zwz};
  for (int i = 0; i < 7; ++i) out_f[i] = fsv[i];
  if (!verified) return PBF_OK;
  if (verify_u >= M) { *verified = -1; return PBF_OK; }
  // ---- Plonk::verify (plonk.rs:468-650); the two pairings on the GPU
  const uint32_t u = (uint32_t)verify_u;
  auto cm = [&](const std::vector<uint32_t>& vv, uint32_t out[3]) {
    Pl p;
    int r2c = interp(c, vv, p);
    return r2c ? r2c : eval_at_s(c, p, out);
  };
  uint32_t qms[3], qls[3], qrs[3], qos[3], qcs[3], s1s[3], s2s[3], s3s[3];
  if ((rc = cm(qm, qms)) || (rc = cm(ql, qls)) || (rc = cm(qr, qrs)) || (rc = cm(qo, qos)) || (rc = cm(qc, qcs)) ||
      (rc = cm(sig[0], s1s)) || (rc = cm(sig[1], s2s)) || (rc = cm(sig[2], s3s)))
    return rc;
  *verified = 0;
  for (int i = 0; i < 9; ++i)
    if (!g1_valid(pts[i]) || pts[i][2]) return PBF_OK;  // in_curve on affine coords (plonk.rs:523-535)
  uint32_t zhz, l1z2;
  if ((rc = evals(c, c.zh, one_z, ev))) return rc;
  zhz = ev[0];
  if ((rc = evals(c, l_1_x, one_z, ev))) return rc;
  l1z2 = ev[0];
  if (zhz == 0) return fail(PBF_EINVAL, "z_h(z) = 0 (plonk.rs:575 unwrap)");
  const uint32_t a1 = fa(fa(fm(beta, s1z), gamma), a_z), b1 = fa(fa(fm(beta, s2z), gamma), b_z), c1 = fa(c_z, gamma);
  const uint32_t tz = fm(fs(fs(fa(r_z, 0), fm(fm(fm(a1, b1), c1), zwz)), fm(l1z2, fm(alpha, alpha))), finv(zhz));
  auto G = [](const uint32_t* p) { return pbh::G1{p[0], p[1], p[2]}; };
  auto gm = [&](const uint32_t* p, uint32_t s) { return pbh::g1_mul(G(p), gfmap(s)); };
  using pbh::g1_add;
  pbh::G1 d1 = g1_add(g1_add(g1_add(g1_add(gm(qms, fm(fm(a_z, b_z), v)), gm(qls, fm(a_z, v))), gm(qrs, fm(b_z, v))),
                             gm(qos, fm(c_z, v))), gm(qcs, v));
  pbh::G1 d2 = gm(pts[3], fa(fa(fm(fm(fm(fm(fa(fa(a_z, fm(beta, z)), gamma), fa(fa(b_z, fm(fm(beta, K1), z)), gamma)),
                                         fa(fa(c_z, fm(fm(beta, K2), z)), gamma)), alpha), v),
                                fm(fm(l1z2, fm(alpha, alpha)), v)), u));
  pbh::G1 d3 = gm(s3s, fm(fm(fm(fm(fm(fa(fa(a_z, fm(beta, s1z)), gamma), fa(fa(b_z, fm(beta, s2z)), gamma)), alpha), v), beta), zwz));
  pbh::G1 d_s = g1_add(g1_add(d1, d2), pbh::g1_neg(d3));
  pbh::G1 f_s = g1_add(g1_add(g1_add(g1_add(g1_add(g1_add(g1_add(g1_add(G(pts[4]), gm(pts[5], pbh::pw(z, (uint32_t)(n + 2), M))),
                                                               gm(pts[6], pbh::pw(z, (uint32_t)(2 * n + 4), M))), d_s),
                                                 gm(pts[0], vp(2))), gm(pts[1], vp(3))), gm(pts[2], vp(4))), gm(s1s, vp(5))),
                       gm(s2s, vp(6)));
  const uint32_t ev_e = fa(fa(fa(fa(fa(fa(fa(tz, fm(v, r_z)), fm(vp(2), a_z)), fm(vp(3), b_z)), fm(vp(4), c_z)), fm(vp(5), s1z)),
                              fm(vp(6), s2z)), fm(u, zwz));
  pbh::G1 e_s = pbh::g1_mul(G(&c.g1s[0]), gfmap(ev_e));
  pbh::G1 e1q1 = g1_add(G(pts[7]), gm(pts[8], u));
  pbh::G1 e2q1 = g1_add(g1_add(g1_add(gm(pts[7], z), gm(pts[8], fm(fm(u, z), OMEGA))), f_s), pbh::g1_neg(e_s));
  std::vector<uint32_t> g1v{e1q1.x, e1q1.y, e1q1.inf, e2q1.x, e2q1.y, e2q1.inf}, g2v{c.g2_s[0], c.g2_s[1], c.g2_1[0], c.g2_1[1]}, e;
  if ((rc = gpu_pairing(pctx, g1v, g2v, e))) return rc;
  *verified = (e[0] == e[2] && e[1] == e[3]) ? 1 : 0;
  return PBF_OK;
}

}  // extern "C"
