// C-ABI entry points of libpbf.so (include/pbf.h). Each cites the reference
// function it replaces (paths relative to the adria0/plonk-by-fingers root).
#include <atomic>
#include <cstring>
#include "../../include/pbf.h"
#include "internal.hpp"

namespace pbf {
static thread_local std::string g_last_error;
void set_error(const std::string& s) { g_last_error = s; }
int fail(int code, const std::string& s) {
  g_last_error = s;
  return code;
}
static bool all_canonical(const uint64_t* v, size_t n, uint64_t m) {
  for (size_t i = 0; i < n; ++i)
    if (v[i] >= m) return false;
  return true;
}
}  // namespace pbf

using namespace pbf;
void pbf_internal_drop_plans256(const void* ctx);  // ntt256.hip
void pbf_internal_drop_tl256(const void* ctx);     // ntt256.hip
void pbf_internal_forget_ctx(const pbf_ctx* ctx);  // group.hip
void pbf_internal_release_group_bufs(const pbf_ctx* ctx);  // group.hip

int pbf_ctx::plan(uint64_t m, uint64_t omega, uint64_t n, int inverse, NttPlan** out) {
  auto key = std::make_tuple(m, omega, n, inverse ? 1 : 0);
  auto it = plans.find(key);
  if (it != plans.end()) { *out = it->second.get(); return 0; }
  std::unique_ptr<NttPlan> p(new NttPlan());
  PBF_HIP(hipSetDevice(device));
  p->opts = options;
  int rc = make_plan(m, omega, n, inverse ? 1 : 0, p.get());
  if (rc) return rc;
  *out = p.get();
  plans[key] = std::move(p);
  return 0;
}

int pbf_ctx::roots(uint64_t m, uint64_t root, uint64_t n, TwoLevel** out) {
  auto key = std::make_tuple(m, root, n);
  auto it = two_level.find(key);
  if (it != two_level.end()) { *out = it->second.get(); return 0; }
  std::unique_ptr<TwoLevel> t(new TwoLevel());
  PBF_HIP(hipSetDevice(device));
  int rc = make_two_level(m, root, n, t.get());
  if (rc) return rc;
  *out = t.get();
  two_level[key] = std::move(t);
  return 0;
}

// Validate (modulus, omega, G, nl) of a stride-sharded transform of N = G*nl points.
static int shard_check(uint64_t modulus, uint64_t omega, uint32_t G, size_t nl, FieldKind* k, FieldArgs* fa) {
  if (!field_for(modulus, k, fa)) return fail(PBF_EUNSUPPORTED, "unsupported modulus");
  if (G != 2 && G != 4 && G != 8) return fail(PBF_EINVAL, "world size must be 2, 4 or 8");
  if (nl < G || (nl & (nl - 1))) return fail(PBF_EINVAL, "per-rank size must be a power of two >= G");
  const uint64_t N = (uint64_t)G * nl;
  if (omega >= modulus || hpow(omega, N, modulus) != 1 || hpow(omega, N / 2, modulus) == 1)
    return fail(PBF_EINVAL, "omega does not have order G*nl");
  return 0;
}

extern "C" {

const char* pbf_last_error(void) { return g_last_error.c_str(); }

int pbf_ctx_create(int device, pbf_ctx** out) {
  if (!out) return fail(PBF_EINVAL, "null out");
  int count = 0;
  PBF_HIP(hipGetDeviceCount(&count));
  if (device < 0 || device >= count) return fail(PBF_EINVAL, "device index out of range");
  PBF_HIP(hipSetDevice(device));
  pbf_ctx* c = new pbf_ctx();
  static std::atomic<uint64_t> next_serial{1};
  c->serial = next_serial++;
  c->device = device;
  c->fork.device = device;
  c->msm_tail.device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return fail(PBF_EDEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  *out = c;
  return PBF_OK;
}

void pbf_ctx_destroy(pbf_ctx* ctx) {
  if (!ctx) return;
  pbf_internal_forget_ctx(ctx);  // multi-GPU groups with this member (group.hip)
  pbf_internal_drop_plans256(ctx);
  pbf_internal_drop_tl256(ctx);
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int pbf_ctx_release_caches(pbf_ctx* ctx) {
  if (!ctx) return fail(PBF_EINVAL, "null ctx");
  PBF_HIP(hipSetDevice(ctx->device));
  PBF_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->msm_tail.aux) PBF_HIP(hipStreamSynchronize(ctx->msm_tail.aux));
  if (ctx->msm_tail.prep) PBF_HIP(hipStreamSynchronize(ctx->msm_tail.prep));
  PBF_HIP(hipDeviceSynchronize());  // _dev callers' streams may still read the caches
  pbf_internal_release_group_bufs(ctx);  // the multi-GPU groups' exchange buffers
  ctx->pk_key.clear();
  ctx->vk_key.clear();
  ctx->vk_pts.clear();
  ctx->pair_g2_key.clear();
  ctx->fixed_base.valid = false;
  ctx->fixed_base.n = 0;
  ctx->fixed_base.table.release();
  ctx->fixed_base.inf.release();
  for (const char* name : {"pk.coef", "pk.coset", "pc.lines", "pc.qinf"}) ctx->named.erase(name);
  for (auto it = ctx->named.begin(); it != ctx->named.end();)
    it = it->first.compare(0, 5, "snap.") == 0 ? ctx->named.erase(it) : std::next(it);
  ctx->snap_words.clear();
  ctx->snap_gen.clear();
  ctx->snap_used.clear();
  return PBF_OK;
}

// Context options (include/pbf.h): a value replaces the previous one, NULL removes the option.
// Cached NTT plans were built under the old options, so an ntt* option drops them (after the
// device has finished with them) and they are rebuilt on next use.
int pbf_ctx_set_option(pbf_ctx* ctx, const char* name, const char* value) {
  if (!ctx || !name || !*name) return fail(PBF_EINVAL, "null argument");
  static const char* const known[] = {"ntt.passes",  "ntt.group",       "ntt.streams",   "ntt.twmax_log",
                                      "ntt.twsplit", "ntt.no_rg",       "ntt256.maxr",   "ntt256.twlog",
                                      "msm.fx_c",    "g1.mul_base",     "pair.engine",   "pair.lane_wpe",
                                      "prover.pk",   "prover.timing",   "verifier.vk",   "ntt256.l29"};
  bool ok = false;
  for (const char* k : known) ok = ok || strcmp(k, name) == 0;
  if (!ok) return fail(PBF_EINVAL, std::string("unknown option ") + name);
  if (value) ctx->options.kv[name] = value;
  else ctx->options.kv.erase(name);
  if (strncmp(name, "ntt", 3) == 0) {
    PBF_HIP(hipSetDevice(ctx->device));
    PBF_HIP(hipDeviceSynchronize());
    ctx->plans.clear();
    pbf_internal_drop_plans256(ctx);
  }
  return PBF_OK;
}

int pbf_ctx_set_stream(pbf_ctx* ctx, void* stream) {
  if (!ctx) return fail(PBF_EINVAL, "null ctx");
  ctx->user_stream = (hipStream_t)stream;
  return PBF_OK;
}

int pbf_device_sync(pbf_ctx* ctx) {
  if (!ctx) return fail(PBF_EINVAL, "null ctx");
  PBF_HIP(hipSetDevice(ctx->device));
  PBF_HIP(hipDeviceSynchronize());
  return PBF_OK;
}

// fft.rs:66-78 CooleyTurkey::fft / fft_inv (host buffers, synchronous)
int pbf_ntt_u64(pbf_ctx* ctx, uint64_t modulus, uint64_t omega, const uint64_t* in, uint64_t* out, size_t n,
                int inverse) {
  if (!ctx || (!in && n) || (!out && n)) return fail(PBF_EINVAL, "null argument");
  NttPlan* p;
  int rc = ctx->plan(modulus, omega, n, inverse, &p);
  if (rc) return rc;
  if (!all_canonical(in, n, modulus)) return fail(PBF_EINVAL, "input not canonical");
  hipStream_t s = ctx->host_stream();
  if ((rc = ctx->io0.ensure(n * 8))) return rc;
  PBF_HIP(hipMemcpyAsync(ctx->io0.p, in, n * 8, hipMemcpyHostToDevice, s));
  rc = run_plan(*p, (const uint64_t*)ctx->io0.p, (uint64_t*)ctx->io0.p, 1, ctx->scratch0, ctx->scratch1, s);
  if (rc) return rc;
  PBF_HIP(hipMemcpyAsync(out, ctx->io0.p, n * 8, hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  return PBF_OK;
}

int pbf_ntt_u64_batch_dev(pbf_ctx* ctx, uint64_t modulus, uint64_t omega, const uint64_t* d_in, uint64_t* d_out,
                          size_t n, size_t batch, int inverse, void* stream) {
  if (!ctx || !d_in || !d_out) return fail(PBF_EINVAL, "null argument");
  NttPlan* p;
  int rc = ctx->plan(modulus, omega, n, inverse, &p);
  if (rc) return rc;
  PBF_HIP(hipSetDevice(ctx->device));
  return run_plan(*p, d_in, d_out, batch, ctx->scratch0, ctx->scratch1, ctx->pick(stream), &ctx->fork);
}

// fft.rs:109-132 mul_ntt
int pbf_mul_ntt_u64(pbf_ctx* ctx, uint64_t modulus, uint64_t omega, const uint64_t* a, size_t la, const uint64_t* b,
                    size_t lb, uint64_t* out) {
  if (!ctx || !out || (!a && la) || (!b && lb)) return fail(PBF_EINVAL, "null argument");
  const size_t n = la + lb;
  NttPlan *fw, *iv;
  int rc = ctx->plan(modulus, omega, n, 0, &fw);
  if (!rc) rc = ctx->plan(modulus, omega, n, 1, &iv);
  if (rc) return rc;
  if (!all_canonical(a, la, modulus) || !all_canonical(b, lb, modulus)) return fail(PBF_EINVAL, "input not canonical");
  hipStream_t s = ctx->host_stream();
  if ((rc = ctx->io0.ensure(2 * n * 8))) return rc;
  uint64_t* d = (uint64_t*)ctx->io0.p;  // [a | 0 ... | b | 0 ...], two polynomials of n
  PBF_HIP(hipMemsetAsync(d, 0, 2 * n * 8, s));
  if (la) PBF_HIP(hipMemcpyAsync(d, a, la * 8, hipMemcpyHostToDevice, s));
  if (lb) PBF_HIP(hipMemcpyAsync(d + n, b, lb * 8, hipMemcpyHostToDevice, s));
  if ((rc = run_plan(*fw, d, d, 2, ctx->scratch0, ctx->scratch1, s))) return rc;
  if ((rc = launch_pointwise_mul(fw->kind, fw->fa, d, d + n, d, n, s))) return rc;
  if ((rc = run_plan(*iv, d, d, 1, ctx->scratch0, ctx->scratch1, s))) return rc;
  PBF_HIP(hipMemcpyAsync(out, d, n * 8, hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  return PBF_OK;
}

// poly.rs:71-79 Poly::eval, batched over points
int pbf_poly_eval_u64(pbf_ctx* ctx, uint64_t modulus, const uint64_t* coeffs, size_t n, const uint64_t* xs, size_t nx,
                      uint64_t* ys) {
  if (!ctx || (!coeffs && n) || (!xs && nx) || (!ys && nx)) return fail(PBF_EINVAL, "null argument");
  if (n == 0) return fail(PBF_EINVAL, "a Poly has at least one coefficient (poly.rs:17-21)");
  FieldKind k;
  FieldArgs fa;
  if (!field_for(modulus, &k, &fa)) return fail(PBF_EUNSUPPORTED, "unsupported modulus");
  if (!all_canonical(coeffs, n, modulus) || !all_canonical(xs, nx, modulus)) return fail(PBF_EINVAL, "input not canonical");
  if (nx == 0) return PBF_OK;
  PBF_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->host_stream();
  int rc;
  if ((rc = ctx->io0.ensure(n * 8)) || (rc = ctx->io1.ensure(nx * 8)) || (rc = ctx->io2.ensure(nx * 8))) return rc;
  PBF_HIP(hipMemcpyAsync(ctx->io0.p, coeffs, n * 8, hipMemcpyHostToDevice, s));
  PBF_HIP(hipMemcpyAsync(ctx->io1.p, xs, nx * 8, hipMemcpyHostToDevice, s));
  if ((rc = launch_poly_eval(k, fa, (const uint64_t*)ctx->io0.p, n, (const uint64_t*)ctx->io1.p, nx,
                             (uint64_t*)ctx->io2.p, ctx->partial, s)))
    return rc;
  PBF_HIP(hipMemcpyAsync(ys, ctx->io2.p, nx * 8, hipMemcpyDeviceToHost, s));
  PBF_HIP(hipStreamSynchronize(s));
  return PBF_OK;
}

// c[i] = a[i] * b[i] (the pointwise step of mul_ntt, fft.rs:125-129), device pointers
int pbf_pointwise_mul_u64_dev(pbf_ctx* ctx, uint64_t modulus, const uint64_t* d_a, const uint64_t* d_b, uint64_t* d_c,
                              size_t count, void* stream) {
  if (!ctx || (count && (!d_a || !d_b || !d_c))) return fail(PBF_EINVAL, "null argument");
  FieldKind k;
  FieldArgs fa;
  if (!field_for(modulus, &k, &fa)) return fail(PBF_EUNSUPPORTED, "unsupported modulus");
  PBF_HIP(hipSetDevice(ctx->device));
  return launch_pointwise_mul(k, fa, d_a, d_b, d_c, count, ctx->pick(stream));
}

int pbf_fill_random_u64_dev(pbf_ctx* ctx, uint64_t modulus, uint64_t seed, uint64_t* d_out, size_t count,
                            void* stream) {
  if (!ctx || (!d_out && count)) return fail(PBF_EINVAL, "null argument");
  FieldKind k;
  FieldArgs fa;
  if (!field_for(modulus, &k, &fa)) return fail(PBF_EUNSUPPORTED, "unsupported modulus");
  return launch_fill_random(fa, k, seed, d_out, count, ctx->pick(stream));
}

}  // extern "C"

extern "C" {

// Multi-GPU stride-sharded NTT, local step (the top log2(G) levels of
// the even/odd recursion at fft.rs:94-96 become the rank index).
int pbf_ntt_shard_local_dev(pbf_ctx* ctx, uint64_t modulus, uint64_t omega, uint32_t world, const uint64_t* d_in,
                            uint64_t* d_out, size_t nl, size_t batch, int inverse, void* stream) {
  if (!ctx || !d_in || !d_out) return fail(PBF_EINVAL, "null argument");
  FieldKind k;
  FieldArgs fa;
  int rc = shard_check(modulus, omega, world, nl, &k, &fa);
  if (rc) return rc;
  const uint64_t wl = hpow(omega, world, modulus);  // local root, order nl
  NttPlan* p;
  if ((rc = ctx->plan(modulus, wl, nl, inverse, &p))) return rc;
  hipStream_t s = ctx->pick(stream);
  if (!inverse)
    return run_plan_split(*p, d_in, d_out, batch, world, ctx->scratch0, ctx->scratch1, ctx->scratch2, s);
  if ((rc = ctx->scratch2.ensure(batch * nl * 8))) return rc;
  if ((rc = launch_shard_unsplit(d_in, (uint64_t*)ctx->scratch2.p, nl, (uint32_t)batch, world, s))) return rc;
  return run_plan(*p, (const uint64_t*)ctx->scratch2.p, d_out, batch, ctx->scratch0, ctx->scratch1, s);
}

// Multi-GPU stride-sharded NTT, combine step (twiddle w^(g*k) + radix-G butterfly).
int pbf_ntt_shard_combine_dev(pbf_ctx* ctx, uint64_t modulus, uint64_t omega, uint32_t world, uint32_t rank,
                              const uint64_t* d_in, uint64_t* d_out, size_t nl, size_t batch, int inverse,
                              void* stream) {
  if (!ctx || !d_in || !d_out) return fail(PBF_EINVAL, "null argument");
  if (d_in == d_out) return fail(PBF_EINVAL, "combine is out-of-place");
  FieldKind k;
  FieldArgs fa;
  int rc = shard_check(modulus, omega, world, nl, &k, &fa);
  if (rc) return rc;
  if (rank >= world) return fail(PBF_EINVAL, "rank out of range");
  uint64_t root = omega;
  if (inverse && !hinv(omega, modulus, &root)) return fail(PBF_EINVAL, "omega not invertible");
  TwoLevel* tl;
  if ((rc = ctx->roots(modulus, root, (uint64_t)world * nl, &tl))) return rc;
  return launch_shard_combine(k, fa, *tl, world, rank, d_in, d_out, nl, (uint32_t)batch, inverse, ctx->pick(stream));
}

}  // extern "C"
