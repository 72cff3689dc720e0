// Kernel instantiation, NTT planning and launchers for libpbf.so (gfx950).
#include <cstdlib>
#include <cstring>
#include <mutex>
#include "internal.hpp"
#include "ntt_gl.hpp"

namespace pbf {

// ---------------------------------------------------------------- plans
bool hinv(uint64_t a, uint64_t m, uint64_t* out) {
  // extended gcd in i128 (u64field.rs:10-25 uses i64; the inverse is unique)
  __int128 s = 0, old_s = 1, r = m, old_r = a % m;
  while (r != 0) {
    __int128 q = old_r / r, t;
    t = old_r - q * r; old_r = r; r = t;
    t = old_s - q * s; old_s = s; s = t;
  }
  if (old_r != 1) return false;
  if (old_s < 0) old_s += m;
  *out = (uint64_t)old_s;
  return true;
}

bool field_for(uint64_t m, FieldKind* kind, FieldArgs* fa) {
  fa->m = m;
  fa->mu = 0;
  if (m == GOLDILOCKS) { *kind = FIELD_GOLDILOCKS; return true; }
  if (m >= 3 && m < (1ull << 32) && (m & 1)) {
    *kind = FIELD_MOD32;
    fa->mu = (uint64_t)(((u128)1 << 64) / m);
    return true;
  }
  return false;
}

int DevBuf::ensure(size_t need) {
  if (need <= bytes) return 0;
  if (p) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
  hipError_t e = hipMalloc(&p, need);
  if (e != hipSuccess) { p = nullptr; return fail(3, std::string("hipMalloc: ") + hipGetErrorString(e)); }
  bytes = need;
  return 0;
}
void DevBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
}
DevBuf::~DevBuf() { release(); }

static int upload(DevBuf& b, const std::vector<uint64_t>& v) {
  int rc = b.ensure(v.size() * 8);
  if (rc) return rc;
  PBF_HIP(hipMemcpy(b.p, v.data(), v.size() * 8, hipMemcpyHostToDevice));
  return 0;
}

// radix bits per pass: option "ntt.passes" (e.g. "12,12"; every radix family the planner can
// pick, tests/test_ntt_gpu.py), else passes of at most 2^10 as equal as possible
static std::vector<int> default_passes(uint32_t log_n, const Options& o) {
  const char* env = o.get("ntt.passes");
  if (env && *env) {
    std::vector<int> v;
    int sum = 0;
    for (const char* c = env; *c;) {
      int x = atoi(c);
      v.push_back(x);
      sum += x;
      while (*c && *c != ',') ++c;
      if (*c == ',') ++c;
    }
    bool ok = sum == (int)log_n;
    for (int x : v) ok = ok && x >= 6 && x <= 12;
    if (ok) return v;
  }
  int p = (log_n + 9) / 10;
  std::vector<int> v(p, log_n / p);
  for (int i = 0; i < (int)(log_n % p); ++i) v[i] += 1;
  return v;
}


static int gl_tile(int logr);

int make_plan(uint64_t m, uint64_t omega, uint64_t n, int inverse, NttPlan* p) {
  if (!field_for(m, &p->kind, &p->fa)) return fail(5, "unsupported modulus");
  if (n == 0 || (n & (n - 1))) return fail(1, "n must be a power of two");
  if (n > (1ull << 32)) return fail(1, "n too large");
  if (omega >= m) return fail(1, "omega not canonical");
  uint32_t log_n = 0;
  while ((1ull << log_n) < n) ++log_n;
  if (n > 1) {
    // omega must have order exactly n (the reference assumes it; fft.rs:55-65)
    if (hpow(omega, n, m) != 1 || hpow(omega, n / 2, m) == 1) return fail(1, "omega does not have order n");
  }
  p->m = m; p->omega = omega; p->n = n; p->inverse = inverse; p->log_n = log_n;
  uint64_t w = omega;
  if (inverse) {
    if (!hinv(n % m, m, &p->n_inv)) return fail(2, "n has no inverse modulo M (fft.rs:73 unwrap)");
    if (!hinv(omega, m, &w)) return fail(1, "omega not invertible");
  }
  if (n <= 4096) {
    std::vector<uint64_t> t(n);
    uint64_t x = 1 % m;
    for (uint64_t i = 0; i < n; ++i) { t[i] = x; x = hmul(x, w, m); }
    return upload(p->small_tw, t);
  }
  p->logr = default_passes(log_n, p->opts);
  p->tw_bits = (log_n + 1) / 2;
  // standard Goldilocks root => shift twiddles in the register sub-DFTs
  p->e64 = -1;
  if (p->kind == FIELD_GOLDILOCKS) {
    const uint64_t w64 = hpow(w, n / 64, m);
    if (w64 == hpow(2, 39, m)) p->e64 = 39;
    else if (w64 == hpow(2, 153, m)) p->e64 = 153;
  }
  std::vector<uint64_t> t0(1ull << p->tw_bits), t1(n >> p->tw_bits);
  uint64_t x = 1 % m;
  for (size_t i = 0; i < t0.size(); ++i) { t0[i] = x; x = hmul(x, w, m); }
  uint64_t step = x;  // w^(2^tw_bits)
  x = 1 % m;
  for (size_t i = 0; i < t1.size(); ++i) { t1[i] = x; x = hmul(x, step, m); }
  int rc = upload(p->tw0, t0);
  if (!rc) rc = upload(p->tw1, t1);
  if (rc) return rc;
  // per-pass [r][k] twiddle tables while R*Ns <= 2^ntt.twmax_log (default 24: the last
  // pass of a 2^24 transform reads a 128 MiB table, shared by every polynomial of a batch,
  // in 128-B runs like its data; the two-level table's two random gathers per element were
  // bound by the texture unit: 2^24 x 2 0.545 -> 0.490 ms); larger passes
  // use the two-level table
  {
    uint64_t ns = 1;
    long long tm = p->opts.num("ntt.twmax_log", 24);
    const int twmax = (int)(tm < 0 ? 0 : (tm > 30 ? 30 : tm));
    for (size_t i = 0; i < p->logr.size(); ++i) {
      const uint64_t R = 1ull << p->logr[i];
      auto b = std::make_shared<DevBuf>();
      if (ns > 1 && R * ns <= (1ull << twmax)) {
        const uint64_t step = n / (ns * R);
        std::vector<uint64_t> t(R * ns);
        for (uint64_t r = 0; r < R; ++r) {
          const uint64_t wr = hpow(w, step * r, m);  // (w^(step*r))^k
          uint64_t z = 1 % m;
          for (uint64_t kk = 0; kk < ns; ++kk) { t[r * ns + kk] = z; z = hmul(z, wr, m); }
        }
        int rc1 = upload(*b, t);
        if (rc1) return rc1;
      }
      p->twpass.push_back(b);
      // the last pass of a standard-root plan whose [r][k] table is not built: split table
      // (option ntt.twsplit=1 also replaces a built one, =0 keeps the two-level table: the
      // paths of n > 2^24 exercised at test sizes)
      const bool last = i + 1 == p->logr.size();
      const long long ts = p->opts.num("ntt.twsplit", -1);
      const bool split = ts == 1;
      if (last && ns > 1 && p->e64 >= 0 && ts != 0 && p->logr[i] >= 6 && p->logr[i] <= 10 && (!b->p || split)) {
        const uint64_t W = (uint64_t)gl_tile(p->logr[i]) >> p->logr[i];
        if (ns % W == 0) {
          if (split) p->twpass.back() = std::make_shared<DevBuf>();
          const uint64_t wp = hpow(w, n / (ns * R), m);
          std::vector<uint64_t> ta(R * W), tb((ns / W) * R);
          for (uint64_t r = 0; r < R; ++r) {
            const uint64_t wr = hpow(wp, r, m);
            uint64_t z = 1 % m;
            for (uint64_t c = 0; c < W; ++c) { ta[r * W + c] = z; z = hmul(z, wr, m); }
            const uint64_t wrw = hpow(wr, W, m);  // (w_p^r)^(kb W)
            z = 1 % m;
            for (uint64_t kb = 0; kb < ns / W; ++kb) { tb[kb * R + r] = z; z = hmul(z, wrw, m); }
          }
          p->tws_a = std::make_shared<DevBuf>();
          p->tws_b = std::make_shared<DevBuf>();
          int rc2 = upload(*p->tws_a, ta);
          if (!rc2) rc2 = upload(*p->tws_b, tb);
          if (rc2) return rc2;
          p->tws_w = (int)W;
        }
      }
      ns *= R;
    }
  }
  for (int lr : p->logr) {
    uint64_t R = 1ull << lr;
    uint64_t wr = hpow(w, n / R, m);
    std::vector<uint64_t> rt(R);
    uint64_t y = 1 % m;
    for (uint64_t i = 0; i < R; ++i) { rt[i] = y; y = hmul(y, wr, m); }
    auto b = std::make_shared<DevBuf>();
    rc = upload(*b, rt);
    if (rc) return rc;
    p->rtab.push_back(b);
  }
  // ntt_gl_pass_kernel (standard Goldilocks roots, radices 2^6..2^10): stage-C tables
  // tc[r2][k1] = w_R^(r2*k1), r2 < R/64, k1 < 64; the last pass of an inverse carries n^-1
  p->gl = p->e64 >= 0;
  for (int lr : p->logr) p->gl = p->gl && lr >= 6 && lr <= 10;
  if (p->gl) {
    for (size_t i = 0; i < p->logr.size(); ++i) {
      const uint64_t R = 1ull << p->logr[i], C = R / 64;
      const uint64_t wr = hpow(w, n / R, m);
      const bool scaled = p->inverse && i + 1 == p->logr.size();
      std::vector<uint64_t> tc(C * 64);
      for (uint64_t r2 = 0; r2 < C; ++r2)
        for (uint64_t k1 = 0; k1 < 64; ++k1) {
          const uint64_t z = hpow(wr, r2 * k1, m);
          tc[r2 * 64 + k1] = scaled ? hmul(z, p->n_inv, m) : z;
        }
      auto b = std::make_shared<DevBuf>();
      rc = upload(*b, tc);
      if (rc) return rc;
      p->tc.push_back(b);
    }
  }
  // regrouped 2^24 plan (default for 8,8,8 standard-root plans; option ntt.no_rg=1 keeps the
  // round-2 passes, the tests' cross-check): three twiddle layers of order 4096, 2^18 and 2^24
  // 
  if (p->gl && log_n == 24 && p->logr == std::vector<int>{8, 8, 8} && p->opts.num("ntt.no_rg", 0) == 0) p->rg = true;
  return 0;
}

// ---------------------------------------------------------------- dispatch
typedef void (*PassFn)(PassArgs);

static int cols_for(int logr) {
  // radix 2^10: 8 columns (64-KiB tile, two workgroups per CU overlap each other's HBM
  // and arithmetic phases; measured 0.548 vs 0.585 ms for 16 columns at 2^20 x 32)
  return logr < 10 ? 16 : (logr == 10 ? 8 : (logr == 11 ? 8 : 4));
}

// Kernel configuration of one pass: W columns, register radix 2^LQ, one tile per workgroup
// (the LDS-DMA double-buffered and register-prefetching persistent forms of rounds 1-2 measured
// slower and were removed in round 6: DESIGN.md §3.2)
struct PassCfg {
  int w, lq;
};

static PassCfg pass_cfg(int logr) { return PassCfg{cols_for(logr), 4}; }

#define PBF_PASS(F, LR, W, LQ, E) \
  if (logr == LR && c.w == W && c.lq == LQ) return ntt_pass_kernel<F, LR, W, ((W << LR) >> LQ), LQ, E>;

template <class F, int E>
static PassFn pass_fn_e(int logr, PassCfg c) {
  PBF_PASS(F, 10, 8, 4, E)
  PBF_PASS(F, 11, 8, 4, E)
  PBF_PASS(F, 12, 4, 4, E)
  PBF_PASS(F, 6, 16, 4, E)
  PBF_PASS(F, 7, 16, 4, E)
  PBF_PASS(F, 8, 16, 4, E)
  PBF_PASS(F, 9, 16, 4, E)
  return nullptr;
}

static PassFn pass_fn(FieldKind k, int e64, int logr, PassCfg c) {
  if (k == FIELD_MOD32) return pass_fn_e<Mod32, -1>(logr, c);
  if (e64 == 39) return pass_fn_e<Goldilocks, 39>(logr, c);
  if (e64 == 153) return pass_fn_e<Goldilocks, 153>(logr, c);
  return pass_fn_e<Goldilocks, -1>(logr, c);
}

static int run_plan_impl(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                         DevBuf& s1, hipStream_t stream, uint32_t split_log, ForkSet* fork = nullptr);

int run_plan(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0, DevBuf& s1,
             hipStream_t stream, ForkSet* fork) {
  return run_plan_impl(p, d_in, d_out, batch, s0, s1, stream, 0, fork);
}

// Split a natural-order batch [b][g*S + kk] into the send layout [g][b][kk].
__global__ void shard_split_kernel(const uint64_t* in, uint64_t* out, uint64_t s, uint64_t nl, uint32_t batch) {
  const uint64_t total = nl * batch;
  for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
       id += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = id / nl, k = id % nl;
    out[((k / s) * batch + b) * s + (k % s)] = in[id];
  }
}

static uint64_t grid_for(uint64_t count) {
  uint64_t b = (count + 255) / 256;
  return b > 8192 ? 8192 : (b ? b : 1);
}

int run_plan_split(const NttPlan& p, const uint64_t* d_in, uint64_t* d_send, size_t batch, uint32_t G, DevBuf& s0,
                   DevBuf& s1, DevBuf& s2, hipStream_t stream) {
  const uint64_t S = p.n / G;
  uint32_t sl = 0;
  while ((1ull << sl) < S) ++sl;
  // the last Stockham pass can store the send layout directly when S >= its W columns
  if (!p.logr.empty() && S >= 16 && p.logr.size() >= 2) return run_plan_impl(p, d_in, d_send, batch, s0, s1, stream, sl);
  int rc = s2.ensure(batch * p.n * 8);
  if (rc) return rc;
  if ((rc = run_plan_impl(p, d_in, (uint64_t*)s2.p, batch, s0, s1, stream, 0))) return rc;
  hipLaunchKernelGGL(shard_split_kernel, dim3(grid_for(p.n * batch)), dim3(256), 0, stream, (const uint64_t*)s2.p,
                     d_send, S, p.n, (uint32_t)batch);
  PBF_HIP(hipGetLastError());
  return 0;
}

int launch_shard_unsplit(const uint64_t* recv, uint64_t* out, uint64_t nl, uint32_t batch, uint32_t G,
                         hipStream_t s) {
  hipLaunchKernelGGL(shard_unsplit_kernel, dim3(grid_for(nl * batch)), dim3(256), 0, s, recv, out, nl / G, nl, batch,
                     G);
  PBF_HIP(hipGetLastError());
  return 0;
}

int make_two_level(uint64_t m, uint64_t root, uint64_t n, TwoLevel* t) {
  uint32_t log_n = 0;
  while ((1ull << log_n) < n) ++log_n;
  t->bits = (log_n + 1) / 2;
  t->root = root;
  std::vector<uint64_t> t0(1ull << t->bits), t1((n >> t->bits) ? (n >> t->bits) : 1);
  uint64_t x = 1 % m;
  for (size_t i = 0; i < t0.size(); ++i) { t0[i] = x; x = hmul(x, root, m); }
  uint64_t step = x, y = 1 % m;
  for (size_t i = 0; i < t1.size(); ++i) { t1[i] = y; y = hmul(y, step, m); }
  int rc = upload(t->t0, t0);
  return rc ? rc : upload(t->t1, t1);
}

template <class F>
static int combine_typed(const FieldArgs& fa, const TwoLevel& tl, uint32_t G, uint64_t rank, const uint64_t* in,
                         uint64_t* out, uint64_t nl, uint32_t batch, int inverse, hipStream_t s) {
  CombineArgs a;
  a.recv = in; a.out = out;
  a.tw0 = (const uint64_t*)tl.t0.p; a.tw1 = (const uint64_t*)tl.t1.p; a.tw_bits = tl.bits;
  a.nl = nl; a.s = nl / G; a.rank = rank; a.n_mask = (uint64_t)G * nl - 1; a.batch = batch; a.f = fa;
  a.scale = 1;
  if (inverse) {
    uint64_t ginv;
    if (!hinv(G % fa.m, fa.m, &ginv)) return fail(2, "G has no inverse");
    a.scale = ginv;
  }
  for (int i = 0; i < 8; ++i) a.wg[i] = 0;
  const uint64_t wG = hpow(tl.root, nl, fa.m);  // primitive G-th root (direction-specific)
  uint64_t x = 1 % fa.m;
  for (uint32_t i = 0; i < G; ++i) { a.wg[i] = x; x = hmul(x, wG, fa.m); }
  const uint64_t total = (nl / G) * batch;
  void (*fn)(CombineArgs) = nullptr;
  switch (G) {
    case 2: fn = inverse ? shard_split_inv_kernel<F, 2> : shard_combine_kernel<F, 2>; break;
    case 4: fn = inverse ? shard_split_inv_kernel<F, 4> : shard_combine_kernel<F, 4>; break;
    case 8: fn = inverse ? shard_split_inv_kernel<F, 8> : shard_combine_kernel<F, 8>; break;
    default: return fail(1, "world size must be 2, 4 or 8");
  }
  hipLaunchKernelGGL(fn, dim3(grid_for(total)), dim3(256), 0, s, a);
  PBF_HIP(hipGetLastError());
  return 0;
}

int launch_shard_combine(FieldKind k, const FieldArgs& fa, const TwoLevel& tl, uint32_t G, uint64_t rank,
                         const uint64_t* in, uint64_t* out, uint64_t nl, uint32_t batch, int inverse, hipStream_t s) {
  if (k == FIELD_GOLDILOCKS) return combine_typed<Goldilocks>(fa, tl, G, rank, in, out, nl, batch, inverse, s);
  return combine_typed<Mod32>(fa, tl, G, rank, in, out, nl, batch, inverse, s);
}

typedef void (*GlPassFn)(GlPassArgs);

// Tile of R x W elements per workgroup: radix 2^10 8192 (W = 8: 64-B runs in HBM, two
// workgroups per CU), smaller radices 4096 (W >= 16; four or five workgroups per CU). Wider
// tiles (W = 16 at 2^10: one workgroup per CU) measured slower in round 4.
static int gl_tile(int logr) { return logr >= 10 ? 8192 : 4096; }

template <int E>
static GlPassFn gl_fn_e(int logr, bool first) {
  switch (logr) {
    case 6: return first ? ntt_gl_pass_kernel<6, E, true, 4096> : ntt_gl_pass_kernel<6, E, false, 4096>;
    case 7: return first ? ntt_gl_pass_kernel<7, E, true, 4096> : ntt_gl_pass_kernel<7, E, false, 4096>;
    case 8: return first ? ntt_gl_pass_kernel<8, E, true, 4096> : ntt_gl_pass_kernel<8, E, false, 4096>;
    case 9: return first ? ntt_gl_pass_kernel<9, E, true, 4096> : ntt_gl_pass_kernel<9, E, false, 4096>;
    case 10: return first ? ntt_gl_pass_kernel<10, E, true, 8192> : ntt_gl_pass_kernel<10, E, false, 8192>;
    default: return nullptr;
  }
}

// the regrouped 2^24 plan's three pass kernels
template <int E>
static GlPassFn gl_fn_rg(int pass) {
  if (pass == 0) return ntt_gl_pass_kernel<8, E, true, 4096, 1>;
  if (pass == 1) return ntt_gl_rg2_kernel<E>;
  return ntt_gl_pass_kernel<8, E, false, 4096, 3>;
}

// Passes of a standard-root Goldilocks plan through ntt_gl_pass_kernel (ntt_gl.hpp).
static int run_gl_group(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                        DevBuf& s1, hipStream_t stream, uint32_t split_log, size_t soff = 0);

int ForkSet::ensure(int streams) {
  if (streams > GL_MAX_STREAMS) streams = GL_MAX_STREAMS;
  if (streams > 1 && !fork) PBF_HIP(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  for (int i = 1; i < streams; ++i) {
    if (!aux[i]) PBF_HIP(hipStreamCreateWithFlags(&aux[i], hipStreamNonBlocking));
    if (!join[i]) PBF_HIP(hipEventCreateWithFlags(&join[i], hipEventDisableTiming));
  }
  return 0;
}

ForkSet::~ForkSet() {
  (void)hipSetDevice(device);
  for (int i = 1; i < GL_MAX_STREAMS; ++i) {
    if (aux[i]) {
      (void)hipStreamSynchronize(aux[i]);
      (void)hipStreamDestroy(aux[i]);
    }
    if (join[i]) (void)hipEventDestroy(join[i]);
  }
  if (fork) (void)hipEventDestroy(fork);
}

static int run_gl_passes(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                         DevBuf& s1, hipStream_t stream, uint32_t split_log, ForkSet* fork) {
  // default schedule (measured best at 2^20 x 32): groups of 4 polynomials
  // alternating over the caller's stream and a second one once the batch has at least 8, so the
  // passes of two groups run concurrently and their load / compute / store phases interleave
  // (options ntt.group = polynomials per group, ntt.streams = streams; 0 or >= batch: one group)
  const long long go = p.opts.num("ntt.group", -1);
  const size_t G = go >= 0 ? (size_t)go : (batch >= 8 ? 4 : batch);
  if (split_log != 0 || G == 0 || G >= batch) return run_gl_group(p, d_in, d_out, batch, s0, s1, stream, split_log);
  int ns = (int)p.opts.num("ntt.streams", 2);
  ns = ns < 1 ? 1 : (ns > GL_MAX_STREAMS ? GL_MAX_STREAMS : ns);
  if (!fork) ns = 1;
  hipStream_t sts[GL_MAX_STREAMS];
  sts[0] = stream;
  // Fork and join by events: a stream waiting on an event waits in the command processor
  // (a barrier packet), so it cannot hold the GPU against the work it waits for. Round 5's
  // stream memory-operation joins (hipStreamWaitValue64: a spinning wait kernel) measured 1-4 %
  // faster but never resumed when the queues were serialised (rocprofv3 counter collection,
  // profiles/r05/memop_prof.log); removed in round 6.
  if (ns > 1) {
    int rc = fork->ensure(ns);
    if (rc) return rc;
    for (int i = 1; i < ns; ++i) sts[i] = fork->aux[i];
    PBF_HIP(hipEventRecord(fork->fork, stream));
    for (int i = 1; i < ns; ++i) PBF_HIP(hipStreamWaitEvent(sts[i], fork->fork, 0));
  }
  int gi = 0;
  for (size_t g0 = 0; g0 < batch; g0 += G, ++gi) {
    const size_t b = batch - g0 < G ? batch - g0 : G;
    const int rc = run_gl_group(p, d_in + g0 * p.n, d_out + g0 * p.n, b, s0, s1, sts[gi % ns], 0,
                                ns > 1 ? g0 * p.n : 0);
    if (rc) return rc;
  }
  for (int i = 1; i < ns; ++i) {
    PBF_HIP(hipEventRecord(fork->join[i], sts[i]));
    PBF_HIP(hipStreamWaitEvent(stream, fork->join[i], 0));
  }
  return 0;
}

// The regrouped plan's twiddle tables, built on the first run that takes the regrouped path:
// tc1[a2l][r2][k1] (4096), t2[a1][K] (2^18), and the last pass's C[r2][X] = w^(r2 X) (n^-1
// folded in for the inverse), D[X] = w^(4 X) (X < 2^18: 10 MiB)
static int ensure_rg_tables(const NttPlan& p) {
  if (p.rg_built) return 0;
  const uint64_t m = p.m, n = p.n;
  const int inverse = p.inverse;
  uint64_t w = p.omega;  // the transform's root: omega, or omega^-1 for the inverse (make_plan)
  if (inverse && !hinv(p.omega, m, &w)) return fail(1, "omega not invertible");
  int rc;
  const uint64_t w4096 = hpow(w, n / 4096, m);
  std::vector<uint64_t> tc1(4096);
  for (uint64_t a2l = 0; a2l < 16; ++a2l)
    for (uint64_t r2 = 0; r2 < 4; ++r2)
      for (uint64_t k1 = 0; k1 < 64; ++k1)
        tc1[a2l * 256 + r2 * 64 + k1] = hpow(w4096, ((a2l + 16 * r2) * k1) % 4096, m);
  std::vector<uint64_t> t2(1ull << 18);
  for (uint64_t a1 = 0; a1 < 64; ++a1) {
    const uint64_t st = hpow(w, 64 * a1, m);
    uint64_t y = 1;
    for (uint64_t K = 0; K < 4096; ++K) { t2[(a1 << 12) + K] = y; y = hmul(y, st, m); }
  }
  // the last pass's twiddle w^(a0 X) (a0 = r2 + 4 s2, X = 65536 f + j) as C[r2][X] D[X]^s2 (round
  // 5: from 10 MiB instead of a 2^24-entry, 128 MiB table T3[f][a0][j], profiles/r05/t3geo_ab.log)
  const uint64_t scale = inverse ? p.n_inv : 1;
  std::vector<uint64_t> tgc(4ull << 18), tgb(1ull << 18);
  {
    const uint64_t w4 = hpow(w, 4, m);
    uint64_t x1 = 1, x4 = 1;
    for (uint64_t X = 0; X < (1ull << 18); ++X) {
      tgb[X] = x4;
      uint64_t c = scale;
      for (uint64_t r2 = 0; r2 < 4; ++r2) {
        tgc[(r2 << 18) + X] = c;
        c = hmul(c, x1, m);
      }
      x1 = hmul(x1, w, m);
      x4 = hmul(x4, w4, m);
    }
  }
  if ((rc = upload(p.rg_tc1, tc1)) || (rc = upload(p.rg_t2, t2)) || (rc = upload(p.rg_tgc, tgc)) ||
      (rc = upload(p.rg_tgb, tgb)))
    return rc;
  p.rg_built = true;
  return 0;
}

static int run_gl_group(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                        DevBuf& s1, hipStream_t stream, uint32_t split_log, size_t soff) {
  const size_t P = p.logr.size();
  const bool rg = p.rg && P == 3 && split_log == 0;
  if (rg) {
    const int rc = ensure_rg_tables(p);
    if (rc) return rc;
  }
  uint32_t log_ns = 0;
  for (size_t i = 0; i < P; ++i) {
    const int lr = p.logr[i];
    const int tile = gl_tile(lr);
    GlPassFn fn = p.e64 == 39 ? gl_fn_e<39>(lr, log_ns == 0) : gl_fn_e<153>(lr, log_ns == 0);
    if (rg) fn = p.e64 == 39 ? gl_fn_rg<39>((int)i) : gl_fn_rg<153>((int)i);
    if (!fn) return fail(1, "no Goldilocks pass kernel for this radix");
    const uint64_t W = (uint64_t)tile >> lr;
    if ((p.n >> lr) % W) return fail(1, "transform too small for the pass tile");
    GlPassArgs a;
    a.in = (i == 0) ? d_in : (const uint64_t*)(((i - 1) & 1) ? s1.p : s0.p) + soff;
    a.out = (i == P - 1) ? d_out : (uint64_t*)((i & 1) ? s1.p : s0.p) + soff;
    a.in_pitch = a.out_pitch = p.n;
    a.twpass = (const uint64_t*)p.twpass[i]->p;
    a.tw0 = (const uint64_t*)p.tw0.p;
    a.tw1 = (const uint64_t*)p.tw1.p;
    a.tc = (const uint64_t*)p.tc[i]->p;
    const bool tws = !a.twpass && i == P - 1 && p.tws_a && (uint64_t)p.tws_w == W;
    a.tws_a = tws ? (const uint64_t*)p.tws_a->p : nullptr;
    a.tws_b = tws ? (const uint64_t*)p.tws_b->p : nullptr;
    a.n = p.n;
    a.log_n = p.log_n;
    a.log_ns = log_ns;
    a.tw_bits = p.tw_bits;
    a.blocks_per_poly = (uint32_t)((p.n >> lr) / W);
    a.batch = (uint32_t)batch;
    a.scaled = (p.inverse && i == P - 1) ? 1 : 0;
    a.out_split_log = (i == P - 1) ? split_log : 0;
    const uint64_t tiles = (uint64_t)a.blocks_per_poly * batch;
    if (tiles > 0x7fffffffull) return fail(1, "batch too large");
    // tile order (gl_tile_coords): later passes XCD k-major (the pass-twiddle table's slices
    // fetched into each XCD's L2 once per pass, not once per polynomial)
    a.xcd_kmajor = (log_ns > 0 && batch > 1 && tiles % 8 == 0) ? 1 : 0;
    // two-pass plans apply the second pass's twiddle w^(j k) at the first pass's stores (the
    // first pass hides the product under its memory phase: 2^20 x 32 0.400 -> 0.386 ms,
    // DESIGN.md §3.1), reading that table by column in XCD k-major order too (round 4: 2^20 x 32
    // 0.354-0.357 ms against 0.368-0.371 linear, profiles/r04/ntt_orders_sweep.log)
    a.post_tw = nullptr;
    a.skip_pass_tw = 0;
    if (P == 2 && split_log == 0 && p.twpass[1]->p) {
      if (i == 0) a.post_tw = (const uint64_t*)p.twpass[1]->p;
      else a.skip_pass_tw = 1;
    }
    if (a.post_tw && batch > 1 && tiles % 8 == 0) a.xcd_kmajor = 1;
    if (rg) {
      if (i == 0) a.tc = (const uint64_t*)p.rg_tc1.p;
      if (i == 1) a.twpass = (const uint64_t*)p.rg_t2.p;
      if (i == 2) {
        a.twpass = nullptr;
        a.tws_a = (const uint64_t*)p.rg_tgc.p;
        a.tws_b = (const uint64_t*)p.rg_tgb.p;
      }
      // XCD-blocked order in every pass of the regrouped plan (round 4: 2 x 2^24 0.433-0.437 ms
      // against 0.447-0.453 k-major, 0.462-0.466 linear, profiles/r04/ntt_order24_ab.log; round
      // 5 with the geometric last pass 0.3867-0.3868 against 0.3918-0.3930, order_geo.log)
      if (tiles % 8 == 0) a.xcd_kmajor = 2;
    }
    hipLaunchKernelGGL(fn, dim3((uint32_t)tiles), dim3(tile / 16), 0, stream, a);
    PBF_HIP(hipGetLastError());
    log_ns += lr;
  }
  return 0;
}

static int run_plan_impl(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                         DevBuf& s1, hipStream_t stream, uint32_t split_log, ForkSet* fork) {
  if (batch == 0) return 0;
  if (p.n == 1) {
    if (d_in != d_out) PBF_HIP(hipMemcpyAsync(d_out, d_in, batch * 8, hipMemcpyDeviceToDevice, stream));
    return 0;  // size-1 DFT is the identity; n^-1 = 1
  }
  if (p.logr.empty()) {
    if (p.kind == FIELD_GOLDILOCKS)
      hipLaunchKernelGGL(ntt_small_kernel<Goldilocks>, dim3(batch), dim3(256), 0, stream, d_in, d_out,
                         (const uint64_t*)p.small_tw.p, p.log_n, p.n_inv, (uint32_t)p.inverse, p.fa);
    else
      hipLaunchKernelGGL(ntt_small_kernel<Mod32>, dim3(batch), dim3(256), 0, stream, d_in, d_out,
                         (const uint64_t*)p.small_tw.p, p.log_n, p.n_inv, (uint32_t)p.inverse, p.fa);
    PBF_HIP(hipGetLastError());
    return 0;
  }
  const size_t P = p.logr.size();
  const size_t bytes = batch * p.n * 8;
  int rc = s0.ensure(bytes);
  if (!rc && P > 2) rc = s1.ensure(bytes);
  if (rc) return rc;
  uint32_t log_ns = 0;
  if (p.gl) return run_gl_passes(p, d_in, d_out, batch, s0, s1, stream, split_log, fork);
  for (size_t i = 0; i < P; ++i) {
    const int lr = p.logr[i];
    PassCfg cfg = pass_cfg(lr);
    PassFn fn = pass_fn(p.kind, p.e64, lr, cfg);
    for (int w : {16, 8, 4}) {  // robust fallback: any instantiated single-tile shape
      if (fn) break;
      cfg = PassCfg{w, 4};
      fn = pass_fn(p.kind, p.e64, lr, cfg);
    }
    if (!fn) return fail(1, "no kernel for this radix");
    const int W = cfg.w;
    PassArgs a;
    a.in = (i == 0) ? d_in : (const uint64_t*)(((i - 1) & 1) ? s1.p : s0.p);
    a.out = (i == P - 1) ? d_out : (uint64_t*)((i & 1) ? s1.p : s0.p);
    a.tw0 = (const uint64_t*)p.tw0.p;
    a.tw1 = (const uint64_t*)p.tw1.p;
    a.rtab = (const uint64_t*)p.rtab[i]->p;
    a.twfull = nullptr;
    a.twpass = (const uint64_t*)p.twpass[i]->p;
    a.n = p.n;
    a.n_inv = p.n_inv;
    a.log_n = p.log_n;
    a.log_ns = log_ns;
    a.tw_bits = p.tw_bits;
    a.blocks_per_poly = (uint32_t)((p.n >> lr) / W);
    a.scale = (p.inverse && i == P - 1) ? 1 : 0;
    a.out_split_log = (i == P - 1) ? split_log : 0;
    a.dbg = 0;
    a.batch = (uint32_t)batch;
    a.f = p.fa;
    const int nt = (W << lr) >> cfg.lq;
    const uint64_t blocks = (uint64_t)a.blocks_per_poly * batch;
    if (blocks > 0x7fffffffull) return fail(1, "batch too large");
    const uint32_t grid = (uint32_t)blocks;
    a.xcd_kmajor = (log_ns > 0 && batch > 1 && grid % 8 == 0) ? 1 : 0;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(nt), 0, stream, a);
    PBF_HIP(hipGetLastError());
    log_ns += lr;
  }
  return 0;
}

// ---------------------------------------------------------------- pointwise
int launch_pointwise_mul(FieldKind k, const FieldArgs& fa, const uint64_t* a, const uint64_t* b, uint64_t* c,
                         uint64_t count, hipStream_t s) {
  uint64_t blocks = (count + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) return 0;
  if (k == FIELD_GOLDILOCKS)
    hipLaunchKernelGGL(pointwise_mul_kernel<Goldilocks>, dim3(blocks), dim3(256), 0, s, a, b, c, count, fa);
  else
    hipLaunchKernelGGL(pointwise_mul_kernel<Mod32>, dim3(blocks), dim3(256), 0, s, a, b, c, count, fa);
  PBF_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- poly eval
// Poly::eval (poly.rs:71-79): y = sum_j c_j x^j. Block (point, chunk) computes
// x^start * Horner(chunk) and tree-reduces; a second kernel sums the chunks.
template <class F>
__device__ uint64_t dpow(uint64_t x, uint64_t e, const FieldArgs& f) {
  uint64_t r = 1 % f.m;
  while (e) {
    if (e & 1) r = F::mul(r, x, f);
    x = F::mul(x, x, f);
    e >>= 1;
  }
  return r;
}

constexpr int EVAL_PER_THREAD = 64;
constexpr int EVAL_THREADS = 256;

template <class F>
__global__ void __launch_bounds__(EVAL_THREADS) poly_eval_partial(const uint64_t* c, uint64_t n, const uint64_t* xs,
                                                                  uint64_t chunks, uint64_t* partial, FieldArgs f) {
  __shared__ uint64_t red[EVAL_THREADS];
  const uint64_t pt = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  const uint64_t x = xs[pt];
  const uint64_t start = (ch * EVAL_THREADS + threadIdx.x) * EVAL_PER_THREAD;
  uint64_t acc = 0;
  if (start < n) {
    uint64_t end = start + EVAL_PER_THREAD;
    if (end > n) end = n;
    for (uint64_t j = end; j-- > start;) acc = F::add(F::mul(acc, x, f), c[j], f);
    acc = F::mul(acc, dpow<F>(x, start, f), f);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = EVAL_THREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = F::add(red[threadIdx.x], red[threadIdx.x + s], f);
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

template <class F>
__global__ void poly_eval_final(const uint64_t* partial, uint64_t chunks, uint64_t nx, uint64_t* ys, FieldArgs f) {
  uint64_t pt = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pt >= nx) return;
  uint64_t acc = 0;
  for (uint64_t i = 0; i < chunks; ++i) acc = F::add(acc, partial[pt * chunks + i], f);
  ys[pt] = acc;
}

int launch_poly_eval(FieldKind k, const FieldArgs& fa, const uint64_t* d_coeffs, uint64_t n, const uint64_t* d_xs,
                     uint64_t nx, uint64_t* d_ys, DevBuf& partial, hipStream_t s) {
  const uint64_t per_block = (uint64_t)EVAL_THREADS * EVAL_PER_THREAD;
  const uint64_t chunks = (n + per_block - 1) / per_block;
  int rc = partial.ensure(chunks * nx * 8);
  if (rc) return rc;
  if (k == FIELD_GOLDILOCKS) {
    hipLaunchKernelGGL(poly_eval_partial<Goldilocks>, dim3(chunks * nx), dim3(EVAL_THREADS), 0, s, d_coeffs, n, d_xs,
                       chunks, (uint64_t*)partial.p, fa);
    hipLaunchKernelGGL(poly_eval_final<Goldilocks>, dim3((nx + 255) / 256), dim3(256), 0, s,
                       (const uint64_t*)partial.p, chunks, nx, d_ys, fa);
  } else {
    hipLaunchKernelGGL(poly_eval_partial<Mod32>, dim3(chunks * nx), dim3(EVAL_THREADS), 0, s, d_coeffs, n, d_xs,
                       chunks, (uint64_t*)partial.p, fa);
    hipLaunchKernelGGL(poly_eval_final<Mod32>, dim3((nx + 255) / 256), dim3(256), 0, s, (const uint64_t*)partial.p,
                       chunks, nx, d_ys, fa);
  }
  PBF_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- synthetic inputs
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Element i: z = mix(seed + (i+1)*golden); Goldilocks rejects z >= p by re-mixing
// z + golden; Mod32 reduces z % M. Mirrors tests/golden/gen_golden.py:splitmix_field.
__global__ void fill_random_kernel(uint64_t seed, uint64_t* out, uint64_t count, FieldArgs f, int gold) {
  const uint64_t G = 0x9E3779B97F4A7C15ull;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = splitmix64(seed + (i + 1) * G);
    if (gold) {
      while (z >= f.m) z = splitmix64(z + G);
    } else {
      z %= f.m;
    }
    out[i] = z;
  }
}

int launch_fill_random(const FieldArgs& fa, FieldKind k, uint64_t seed, uint64_t* d_out, uint64_t count,
                       hipStream_t s) {
  if (count == 0) return 0;
  uint64_t blocks = (count + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(fill_random_kernel, dim3(blocks), dim3(256), 0, s, seed, d_out, count, fa,
                     k == FIELD_GOLDILOCKS ? 1 : 0);
  PBF_HIP(hipGetLastError());
  return 0;
}

}  // namespace pbf
