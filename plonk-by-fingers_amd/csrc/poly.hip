// Poly arithmetic of src/poly.rs beyond mul/eval, for the 64-bit
// fields of the NTT path:
//   pbf_poly_div_u64   Div for Poly (poly.rs:230-247): (q, r) with num = q den + r,
//                      deg r < deg den, both normalised (poly.rs:96-105)
//   pbf_poly_add_u64   AddAssign<&Poly> (poly.rs:165-176)
//   pbf_poly_sub_u64   SubAssign<&Poly> (poly.rs:192-203), including the reference's quirk:
//                      coefficients of a longer rhs are appended with a + sign (:196)
//
// Division is not the reference's O(n^2) long division but its O(n log n) equivalent with
// the same unique result: with k = deg num - deg den + 1 and rev(p) = x^deg p p(1/x),
//   rev(q) = rev(num) * rev(den)^-1  mod x^k,   r = num - den q  (mod x^deg den),
// the power-series inverse by Newton's iteration I <- I (2 - rev(den) I) mod x^(2 len)
// from I = lead(den)^-1. Every product is an NTT product on the device (root of unity of
// order 2^root_log supplied by the caller: the NTT size of each product is a power of
// two <= 2^root_log), every elementwise step a device kernel; the host only sequences
// launches, inverts the one leading coefficient and strips trailing zeros of the result.
#include <cstring>
#include <vector>
#include "../../include/pbf.h"
#include "internal.hpp"

namespace pbf {

__global__ void k_copy_pad(const uint64_t* in, uint64_t n_in, uint64_t* out, uint64_t n_out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_out; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = i < n_in ? in[i] : 0;
}
// out[i] = in[n_in - 1 - i] for i < n_in, 0 up to n_out (the reversed coefficient list)
__global__ void k_rev_pad(const uint64_t* in, uint64_t n_in, uint64_t* out, uint64_t n_out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_out; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = i < n_in ? in[n_in - 1 - i] : 0;
}
// t = 2 - t (the Newton step's correction factor)
template <class F>
__global__ void k_two_minus(uint64_t* t, uint64_t n, FieldArgs fa) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    t[i] = F::sub(i == 0 ? 2 : 0, t[i], fa);  // every supported modulus is > 2
}
// out[i] = a[i] +/- b[i] over the first n (missing entries are zero); `quirk`: where only b
// has a coefficient the result is +b[i] even for subtraction (poly.rs:196)
template <class F>
__global__ void k_addsub(const uint64_t* a, uint64_t la, const uint64_t* b, uint64_t lb, uint64_t* out, uint64_t n,
                         int sub, FieldArgs fa) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = i < la ? a[i] : 0, y = i < lb ? b[i] : 0;
    if (i >= la) out[i] = y;  // pushed as is (both ops)
    else out[i] = sub ? F::sub(x, y, fa) : F::add(x, y, fa);
  }
}

static unsigned grid_for(uint64_t n) {
  uint64_t b = (n + 255) / 256;
  return (unsigned)(b > 8192 ? 8192 : (b ? b : 1));
}

static uint64_t mulmod(uint64_t a, uint64_t b, uint64_t m) { return (uint64_t)((unsigned __int128)a * b % m); }
static uint64_t powmod(uint64_t a, uint64_t e, uint64_t m) {
  uint64_t r = 1 % m;
  for (; e; e >>= 1, a = mulmod(a, a, m))
    if (e & 1) r = mulmod(r, a, m);
  return r;
}
// inverse by extended Euclid (the reference's Field::inv, u64field.rs:52-63); false if none
static bool invmod(uint64_t a, uint64_t m, uint64_t* out) {
  __int128 t = 0, nt = 1, r = m, nr = a % m;
  while (nr) {
    const __int128 q = r / nr;
    __int128 tmp = t - q * nt; t = nt; nt = tmp;
    tmp = r - q * nr; r = nr; nr = tmp;
  }
  if (r != 1) return false;
  if (t < 0) t += m;
  *out = (uint64_t)t;
  return true;
}

struct PolyCtx {
  pbf_ctx* ctx;
  uint64_t m, root;
  uint32_t root_log;
  FieldKind kind;
  FieldArgs fa;
  hipStream_t s;

  int two_minus(uint64_t* t, uint64_t n) {
    if (kind == FIELD_GOLDILOCKS) hipLaunchKernelGGL(k_two_minus<Goldilocks>, dim3(grid_for(n)), dim3(256), 0, s, t, n, fa);
    else hipLaunchKernelGGL(k_two_minus<Mod32>, dim3(grid_for(n)), dim3(256), 0, s, t, n, fa);
    PBF_HIP(hipGetLastError());
    return 0;
  }
  int addsub(const uint64_t* a, uint64_t la, const uint64_t* b, uint64_t lb, uint64_t* out, uint64_t n, int sub) {
    if (kind == FIELD_GOLDILOCKS)
      hipLaunchKernelGGL(k_addsub<Goldilocks>, dim3(grid_for(n)), dim3(256), 0, s, a, la, b, lb, out, n, sub, fa);
    else hipLaunchKernelGGL(k_addsub<Mod32>, dim3(grid_for(n)), dim3(256), 0, s, a, la, b, lb, out, n, sub, fa);
    PBF_HIP(hipGetLastError());
    return 0;
  }
  // out[0..nout) = (x * y)[0..nout) by an NTT product of size L = 2^ceil(log2(nx + ny - 1))
  int mul(const uint64_t* x, uint64_t nx, const uint64_t* y, uint64_t ny, uint64_t* out, uint64_t nout) {
    uint64_t L = 1;
    uint32_t lg = 0;
    while (L < nx + ny - 1) L <<= 1, ++lg;
    if (lg > root_log) return fail(PBF_EINVAL, "product longer than the root of unity's order");
    const uint64_t omega = powmod(root, 1ull << (root_log - lg), m);
    NttPlan *fw, *iv;
    int rc = ctx->plan(m, omega, L, 0, &fw);
    if (!rc) rc = ctx->plan(m, omega, L, 1, &iv);
    if (rc) return rc;
    DevBuf& w = ctx->buf("poly.mul");
    if ((rc = w.ensure(2 * L * 8))) return rc;
    uint64_t* d = (uint64_t*)w.p;
    hipLaunchKernelGGL(k_copy_pad, dim3(grid_for(L)), dim3(256), 0, s, x, nx, d, L);
    hipLaunchKernelGGL(k_copy_pad, dim3(grid_for(L)), dim3(256), 0, s, y, ny, d + L, L);
    PBF_HIP(hipGetLastError());
    if ((rc = run_plan(*fw, d, d, 2, ctx->scratch0, ctx->scratch1, s))) return rc;
    if ((rc = launch_pointwise_mul(kind, fa, d, d + L, d, L, s))) return rc;
    if ((rc = run_plan(*iv, d, d, 1, ctx->scratch0, ctx->scratch1, s))) return rc;
    hipLaunchKernelGGL(k_copy_pad, dim3(grid_for(nout)), dim3(256), 0, s, d, L < nout ? L : nout, out, nout);
    PBF_HIP(hipGetLastError());
    return 0;
  }
};

static size_t normalized_len(const uint64_t* v, size_t n) {  // poly.rs:96-105 (at least 1)
  while (n > 1 && v[n - 1] == 0) --n;
  return n;
}

static int poly_common(pbf_ctx* ctx, uint64_t m, const uint64_t* a, size_t la, const uint64_t* b, size_t lb,
                       FieldKind* k, FieldArgs* fa) {
  if (!ctx || (!a && la) || (!b && lb)) return fail(PBF_EINVAL, "null argument");
  if (la == 0 || lb == 0) return fail(PBF_EINVAL, "a Poly has at least one coefficient (poly.rs:17-21)");
  if (!field_for(m, k, fa)) return fail(PBF_EUNSUPPORTED, "unsupported modulus");
  for (size_t i = 0; i < la; ++i)
    if (a[i] >= m) return fail(PBF_EINVAL, "input not canonical");
  for (size_t i = 0; i < lb; ++i)
    if (b[i] >= m) return fail(PBF_EINVAL, "input not canonical");
  return PBF_OK;
}

static int poly_addsub(pbf_ctx* ctx, uint64_t m, const uint64_t* a, size_t la, const uint64_t* b, size_t lb,
                       uint64_t* out, size_t* lout, int sub) {
  FieldKind k;
  FieldArgs fa;
  int rc = poly_common(ctx, m, a, la, b, lb, &k, &fa);
  if (rc) return rc;
  if (!out || !lout) return fail(PBF_EINVAL, "null argument");
  PBF_HIP(hipSetDevice(ctx->device));
  PolyCtx P{ctx, m, 0, 0, k, fa, ctx->host_stream()};
  const size_t n = la > lb ? la : lb;
  DevBuf& d = ctx->buf("poly.io");
  if ((rc = d.ensure(3 * n * 8))) return rc;
  uint64_t* da = (uint64_t*)d.p;
  uint64_t* db = da + n;
  uint64_t* dc = db + n;
  PBF_HIP(hipMemcpyAsync(da, a, la * 8, hipMemcpyHostToDevice, P.s));
  PBF_HIP(hipMemcpyAsync(db, b, lb * 8, hipMemcpyHostToDevice, P.s));
  if ((rc = P.addsub(da, la, db, lb, dc, n, sub))) return rc;
  PBF_HIP(hipMemcpyAsync(out, dc, n * 8, hipMemcpyDeviceToHost, P.s));
  PBF_HIP(hipStreamSynchronize(P.s));
  *lout = normalized_len(out, n);
  return PBF_OK;
}

}  // namespace pbf

using namespace pbf;

extern "C" {

int pbf_poly_add_u64(pbf_ctx* ctx, uint64_t modulus, const uint64_t* a, size_t la, const uint64_t* b, size_t lb,
                     uint64_t* out, size_t* lout) {
  return poly_addsub(ctx, modulus, a, la, b, lb, out, lout, 0);
}

int pbf_poly_sub_u64(pbf_ctx* ctx, uint64_t modulus, const uint64_t* a, size_t la, const uint64_t* b, size_t lb,
                     uint64_t* out, size_t* lout) {
  return poly_addsub(ctx, modulus, a, la, b, lb, out, lout, 1);
}

int pbf_poly_div_u64(pbf_ctx* ctx, uint64_t modulus, uint64_t root, uint32_t root_log, const uint64_t* num,
                     size_t nn, const uint64_t* den, size_t nd, uint64_t* q, size_t* lq, uint64_t* r, size_t* lr) {
  FieldKind kind;
  FieldArgs fa;
  int rc = poly_common(ctx, modulus, num, nn, den, nd, &kind, &fa);
  if (rc) return rc;
  if (!q || !lq || !r || !lr) return fail(PBF_EINVAL, "null argument");
  if (root_log > 32 || root >= modulus) return fail(PBF_EINVAL, "bad root of unity");
  nn = normalized_len(num, nn);
  nd = normalized_len(den, nd);
  const bool num_zero = nn == 1 && num[0] == 0;
  if (num_zero || nn < nd) {  // the reference's loop does not run (poly.rs:234): q = 0, r = num,
    q[0] = 0;                 // whatever the divisor is, so 0 / 0 = (0, 0) without a panic
    *lq = 1;
    std::memcpy(r, num, nn * 8);
    *lr = nn;
    return PBF_OK;
  }
  uint64_t lead_inv;
  if (!invmod(den[nd - 1], modulus, &lead_inv))  // zero divisor: the reference panics (poly.rs:238 unwrap)
    return fail(PBF_ENOINV, "leading coefficient of the divisor has no inverse");
  PBF_HIP(hipSetDevice(ctx->device));
  PolyCtx P{ctx, modulus, root, root_log, kind, fa, ctx->host_stream()};
  const size_t k = nn - nd + 1;  // quotient length
  size_t K = 1;
  while (K < k) K <<= 1;
  DevBuf& io = ctx->buf("poly.io");
  // layout: A nn | B nd | revB K | I K | T K | revA k | revQ k | Q k | BQ nd | R nd
  const size_t tot = nn + nd + 3 * K + 3 * k + 2 * nd;
  if ((rc = io.ensure(tot * 8))) return rc;
  uint64_t* dA = (uint64_t*)io.p;
  uint64_t* dB = dA + nn;
  uint64_t* dRevB = dB + nd;
  uint64_t* dI = dRevB + K;
  uint64_t* dT = dI + K;
  uint64_t* dRevA = dT + K;
  uint64_t* dRevQ = dRevA + k;
  uint64_t* dQ = dRevQ + k;
  uint64_t* dBQ = dQ + k;
  uint64_t* dR = dBQ + nd;
  hipStream_t s = P.s;
  PBF_HIP(hipMemcpyAsync(dA, num, nn * 8, hipMemcpyHostToDevice, s));
  PBF_HIP(hipMemcpyAsync(dB, den, nd * 8, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_rev_pad, dim3(grid_for(K)), dim3(256), 0, s, dB, (uint64_t)nd, dRevB, (uint64_t)K);
  PBF_HIP(hipMemcpyAsync(dI, &lead_inv, 8, hipMemcpyHostToDevice, s));
  // Newton: I = rev(den)^-1 mod x^len, len = 1, 2, 4, ... K
  for (size_t len = 1; len < K; len <<= 1) {
    const size_t len2 = 2 * len;
    if ((rc = P.mul(dRevB, len2 < nd ? len2 : nd, dI, len, dT, len2))) return rc;  // rev(den) I
    if ((rc = P.two_minus(dT, len2))) return rc;                                     // 2 - rev(den) I
    if ((rc = P.mul(dI, len, dT, len2, dI, len2))) return rc;                        // I (2 - rev(den) I)
  }
  // rev(q) = rev(num) I mod x^k; q = rev(rev(q))
  hipLaunchKernelGGL(k_rev_pad, dim3(grid_for(k)), dim3(256), 0, s, dA, (uint64_t)nn, dRevA, (uint64_t)k);
  PBF_HIP(hipGetLastError());
  if ((rc = P.mul(dRevA, k, dI, k, dRevQ, k))) return rc;
  hipLaunchKernelGGL(k_rev_pad, dim3(grid_for(k)), dim3(256), 0, s, dRevQ, (uint64_t)k, dQ, (uint64_t)k);
  PBF_HIP(hipGetLastError());
  // r = num - den q, below degree deg den (the higher coefficients cancel exactly)
  size_t nr = nd - 1;
  if (nr > 0) {
    if ((rc = P.mul(dB, nd, dQ, k, dBQ, nr))) return rc;
    if ((rc = P.addsub(dA, nr, dBQ, nr, dR, nr, 1))) return rc;
  }
  PBF_HIP(hipMemcpyAsync(q, dQ, k * 8, hipMemcpyDeviceToHost, s));
  if (nr > 0) PBF_HIP(hipMemcpyAsync(r, dR, nr * 8, hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  *lq = normalized_len(q, k);
  if (nr == 0) {
    r[0] = 0;
    *lr = 1;
  } else {
    *lr = normalized_len(r, nr);
  }
  return PBF_OK;
}

}  // extern "C"
