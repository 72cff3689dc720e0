// Kernel instantiation, NTT planning and launchers for libpbf.so (gfx950).
#include <cstdlib>
#include <cstring>
#include <mutex>
#include "internal.hpp"
#include "ntt_gl.hpp"
#include "ntt_r4k.hpp"

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

static std::vector<int> default_passes(uint32_t log_n) {
  const char* env = getenv("PBF_NTT_PASSES");  // e.g. "12,12" (benchmarking override)
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

// ---- round-3 schedule (ntt_ip.hpp) ----------------------------------------------------
int ip_tile_of(int r) { return r >= 10 ? 8192 : 4096; }
int ip_w(int r) { return ip_tile_of(r) >> r; }

// radix bits per pass, top slot first; empty when the schedule does not apply
static std::vector<int> ip_radices(uint32_t L) {
  std::vector<int> v;
  if (const char* env = getenv("PBF_NTT_IP_PASSES")) {  // A/B override, e.g. "8,8,8"
    int sum = 0;
    for (const char* c = env; *c;) {
      v.push_back(atoi(c));
      sum += v.back();
      while (*c && *c != ',') ++c;
      if (*c == ',') ++c;
    }
    if (sum != (int)L) v.clear();
  } else if (L >= 12 && L <= 30) {
    const int P = L <= 20 ? 2 : 3;
    v.assign(P, (int)L / P);
    for (int i = 0; i < (int)(L % P); ++i) v[i] += 1;
  }
  if (v.size() < 2 || v.size() > 4) return {};  // IP_MAXP (ntt_ip.hpp)
  int lo = (int)L;
  for (size_t i = 0; i < v.size(); ++i) {
    if (v[i] < 6 || v[i] > 10) return {};
    lo -= v[i];
    if (i + 1 < v.size() && (1 << lo) < ip_w(v[i])) return {};  // column blocks of W
  }
  if ((1 << v[0]) < ip_w(v.back())) return {};  // row pass: W consecutive K vary k_0 only
  return v;
}

static int make_ip_plan(NttPlan* p, uint64_t w) {
  const uint64_t m = p->m, n = p->n;
  const uint32_t L = p->log_n;
  p->ip_r = ip_radices(L);
  if (p->ip_r.empty()) return 0;
  const size_t P = p->ip_r.size();
  std::vector<int> lo(P);
  {
    int l = (int)L;
    for (size_t i = 0; i < P; ++i) { l -= p->ip_r[i]; lo[i] = l; }
  }
  const uint64_t scale = p->inverse ? p->n_inv : 1;
  for (size_t i = 0; i < P; ++i) {
    const int r = p->ip_r[i];
    const uint64_t R = 1ull << r, C = R / 64, W = (uint64_t)ip_w(r);
    // stage-C table w_R^(r2 k1) (unscaled: the inverse scales in the row pass's twiddles)
    {
      const uint64_t wr = hpow(w, n / R, m);
      std::vector<uint64_t> tc(C * 64);
      for (uint64_t r2 = 0; r2 < C; ++r2)
        for (uint64_t k1 = 0; k1 < 64; ++k1) tc[r2 * 64 + k1] = hpow(wr, r2 * k1, m);
      auto b = std::make_shared<DevBuf>();
      int rc = upload(*b, tc);
      if (rc) return rc;
      p->ip_tc.push_back(b);
    }
    auto tb = std::make_shared<DevBuf>();
    if (i > 0 && i + 1 < P) {
      // column pass: T[h][x] = w^(2^lo_i x K(h)), K(h) = the earlier digits, k_0 lowest
      const uint64_t H = 1ull << (L - lo[i] - r);
      std::vector<uint64_t> t(H * R);
      for (uint64_t h = 0; h < H; ++h) {
        uint64_t K = 0, sh = 0;
        for (size_t j = 0; j < i; ++j) {
          const uint64_t kj = (h >> (lo[j] - lo[i] - r)) & ((1ull << p->ip_r[j]) - 1);
          K |= kj << sh;
          sh += (uint64_t)p->ip_r[j];
        }
        const uint64_t z = hpow(w, (((uint64_t)1 << lo[i]) * K) % n, m);
        uint64_t y = 1;
        for (uint64_t x = 0; x < R; ++x) { t[h * R + x] = y; y = hmul(y, z, m); }
      }
      int rc = upload(*tb, t);
      if (rc) return rc;
    } else if (i + 1 == P) {
      // row pass: w^(x K) (x n^-1 for the inverse), K < n / R
      const uint64_t NK = n / R;
      const bool full = n <= (1ull << 21) && !getenv("PBF_NTT_IP_SPLIT");
      std::vector<uint64_t> t(full ? NK * R : (NK / W) * R);
      for (uint64_t kb = 0; kb < (full ? NK : NK / W); ++kb) {
        const uint64_t z = hpow(w, full ? kb : kb * W, m);
        uint64_t y = scale;
        for (uint64_t x = 0; x < R; ++x) { t[kb * R + x] = y; y = hmul(y, z, m); }
      }
      int rc = upload(*tb, t);
      if (rc) return rc;
      if (!full) {
        std::vector<uint64_t> ta(R * W);
        for (uint64_t x = 0; x < R; ++x) {
          const uint64_t z = hpow(w, x, m);
          uint64_t y = 1;
          for (uint64_t c = 0; c < W; ++c) { ta[x * W + c] = y; y = hmul(y, z, m); }
        }
        p->ip_twa = std::make_shared<DevBuf>();
        if ((rc = upload(*p->ip_twa, ta))) return rc;
      }
    }
    p->ip_tw.push_back(tb);
  }
  p->ip = true;
  return 0;
}

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
  p->logr = default_passes(log_n);
  p->tw_bits = (log_n + 1) / 2;
  // standard Goldilocks root => shift twiddles in the register sub-DFTs
  p->e64 = -1;
  if (p->kind == FIELD_GOLDILOCKS && !getenv("PBF_NTT_NO_SHIFT")) {
    const uint64_t w64 = hpow(w, n / 64, m);
    if (w64 == hpow(2, 39, m)) p->e64 = 39;
    else if (w64 == hpow(2, 153, m)) p->e64 = 153;
  }
  // scattered full twiddle table: measured slower than the two-level table (kept for A/B)
  if (log_n <= 22 && getenv("PBF_NTT_TWFULL")) {
    std::vector<uint64_t> tf(n);
    uint64_t z = 1 % m;
    for (uint64_t i = 0; i < n; ++i) { tf[i] = z; z = hmul(z, w, m); }
    int rc0 = upload(p->twfull, tf);
    if (rc0) return rc0;
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
  // per-pass [r][k] twiddle tables while R*Ns <= 2^PBF_NTT_TWMAX_LOG (default 24: the last
  // pass of a 2^24 transform reads a 128 MiB table, shared by every polynomial of a batch,
  // in 128-B runs like its data; the two-level table's two random gathers per element were
  // bound by the texture unit: 2^24 x 2 0.545 -> 0.490 ms); larger passes
  // use the two-level table
  {
    uint64_t ns = 1;
    const char* tm = getenv("PBF_NTT_TWMAX_LOG");
    const int twmax = tm ? atoi(tm) : 24;
    for (size_t i = 0; i < p->logr.size(); ++i) {
      const uint64_t R = 1ull << p->logr[i];
      auto b = std::make_shared<DevBuf>();
      if (ns > 1 && R * ns <= (1ull << twmax) && !getenv("PBF_NTT_TWO_LEVEL")) {
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
      // (A/B: PBF_NTT_TWSPLIT=1 also replaces a built one)
      const bool last = i + 1 == p->logr.size();
      const bool split = getenv("PBF_NTT_TWSPLIT") != nullptr;
      if (last && ns > 1 && p->e64 >= 0 && !getenv("PBF_NTT_NO_TWSPLIT") && p->logr[i] >= 6 && p->logr[i] <= 10 && (!b->p || split)) {
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
  p->gl = p->e64 >= 0 && !getenv("PBF_NTT_LEGACY");
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
  // regrouped 2^24 plan (default for 8,8,8 standard-root plans; PBF_NTT_NO_RG=1 restores the
  // round-2 passes): three twiddle layers of order 4096, 2^18 and 2^24
  if (p->gl && log_n == 24 && p->logr == std::vector<int>{8, 8, 8} && !getenv("PBF_NTT_NO_RG")) p->rg = true;
  // two-pass 4096 x 4096 plan (ntt_r4k.hpp)
  if (p->gl && log_n == 24 && getenv("PBF_NTT_R4K")) p->r4k = true;
  // round-3 in-place schedule: opt-in (PBF_NTT_IP=1) while it measures slower than the
  // round-2 Stockham plan
  if (p->gl && getenv("PBF_NTT_IP") && !getenv("PBF_NTT_V2")) {
    int rc2 = make_ip_plan(p, w);
    if (rc2) return rc2;
  }
  return 0;
}

// ---------------------------------------------------------------- dispatch
typedef void (*PassFn)(PassArgs);

static int cols_for(int logr) {
  // radix 2^10: 8 columns (64-KiB tile, two workgroups per CU overlap each other's HBM
  // and arithmetic phases; measured 0.548 vs 0.585 ms for 16 columns at 2^20 x 32)
  return logr < 10 ? 16 : (logr == 10 ? 8 : (logr == 11 ? 8 : 4));
}

// Kernel configuration of one pass: W columns, register radix 2^LQ, double-buffered
// persistent (DB) or one tile per workgroup.
struct PassCfg {
  int w, lq, db, nt;  // nt != 0: threads per workgroup other than R*W/2^lq
};

static PassCfg pass_cfg(int logr) {
  // default: one tile per workgroup (measured faster than the LDS-DMA
  // double-buffered kernel, whose two tiles halve occupancy: DESIGN.md "NTT")
  PassCfg def = PassCfg{cols_for(logr), 4, 0, 0};
  const char* env = getenv("PBF_NTT_CFG");  // "W,LQ,DB" e.g. "16,4,0" (benchmarking override)
  if (env && *env) {
    int v[4] = {def.w, def.lq, def.db, 0}, i = 0;
    for (const char* c = env; *c && i < 4;) {
      v[i++] = atoi(c);
      while (*c && *c != ',') ++c;
      if (*c == ',') ++c;
    }
    return PassCfg{v[0], v[1], v[2], v[3]};
  }
  return def;
}

#define PBF_PASS(F, LR, W, LQ, E)                                                              \
  if (logr == LR && c.w == W && c.lq == LQ && !c.db && !c.nt) return ntt_pass_kernel<F, LR, W, ((W << LR) >> LQ), LQ, E>;
#define PBF_PASS_DB(F, LR, W, LQ, E)                                                           \
  if (logr == LR && c.w == W && c.lq == LQ && c.db == 1) return ntt_pass_db_kernel<F, LR, W, ((W << LR) >> LQ), LQ, E>;
#define PBF_PASS_NT(F, LR, W, LQ, NTH, E)                                                      \
  if (logr == LR && c.w == W && c.lq == LQ && !c.db && c.nt == NTH) return ntt_pass_kernel<F, LR, W, NTH, LQ, E>;
#define PBF_PASS_RP(F, LR, W, LQ, E)                                                           \
  if (logr == LR && c.w == W && c.lq == LQ && c.db == 2) return ntt_pass_rp_kernel<F, LR, W, ((W << LR) >> LQ), LQ, E>;

template <class F, int E>
static PassFn pass_fn_e(int logr, PassCfg c) {
  PBF_PASS_DB(F, 10, 8, 4, E)  // A/B only (PBF_NTT_CFG=8,4,1): measured slower, DESIGN.md "NTT"
  PBF_PASS_RP(F, 10, 8, 4, E)  // A/B only (PBF_NTT_CFG=8,4,2)
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

// Persistent grid: every resident workgroup slot once (blocks per CU from the
// occupancy query x CUs), never more than there are tiles.
// The answer depends only on the kernel, the block size and the device, never on a context's
// state, so one process-wide table under a lock serves every context (pbf.h: contexts share
// no mutable state a caller could observe).
uint32_t persistent_grid(const void* fn, int nt, uint64_t tiles) {
  static std::mutex mu;
  static std::map<std::tuple<const void*, int, int>, uint32_t> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const auto key = std::make_tuple(fn, nt, dev);
  uint32_t slots;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) {
      slots = it->second;
    } else {
      int cus = 256, per_cu = 1;
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, nt, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
      slots = (uint32_t)(cus * per_cu);
      cache[key] = slots;
    }
  }
  const char* env = getenv("PBF_NTT_GRID_MULT");  // A/B: oversubscribe the persistent grid
  if (env) slots *= (uint32_t)atoi(env);
  return (uint32_t)(tiles < slots ? tiles : slots);
}

typedef void (*GlPassFn)(GlPassArgs);

#define PBF_GL_K(LR, FIRST, T) (persist ? ntt_gl_pass_pkernel<LR, E, FIRST, T> : ntt_gl_pass_kernel<LR, E, FIRST, T>)

template <int E, int T>
static GlPassFn gl_fn_t(int logr, bool first, bool persist) {
  switch (logr) {
    case 6: return first ? PBF_GL_K(6, true, T) : PBF_GL_K(6, false, T);
    case 7: return first ? PBF_GL_K(7, true, T) : PBF_GL_K(7, false, T);
    case 8: return first ? PBF_GL_K(8, true, T) : PBF_GL_K(8, false, T);
    case 9: return first ? PBF_GL_K(9, true, T) : PBF_GL_K(9, false, T);
    default: return nullptr;
  }
}

// Tile of R x W elements per workgroup: 4096 (four workgroups per CU) or 8192 (two);
// radix 2^10 always 8192 (W >= 8: 64-B runs in HBM).
static int gl_tile(int logr) {
  const char* env = getenv("PBF_NTT_TILE");  // A/B override
  const int e = env ? atoi(env) : 0;
  if (logr >= 10) return e == 16384 ? 16384 : 8192;
  return e == 8192 ? 8192 : 4096;
}

template <int E>
static GlPassFn gl_fn_e(int logr, bool first, int tile, bool persist) {
  if (logr == 10 && tile == 16384) return first ? PBF_GL_K(10, true, 16384) : PBF_GL_K(10, false, 16384);
  if (logr == 10) return first ? PBF_GL_K(10, true, 8192) : PBF_GL_K(10, false, 8192);
  return tile == 8192 ? gl_fn_t<E, 8192>(logr, first, persist) : gl_fn_t<E, 4096>(logr, first, persist);
}
#undef PBF_GL_K

// blocked-intermediate variants (two-pass plans), the default tile of each radix
template <int E>
static GlPassFn gl_fn_blk(int logr, bool first) {
#define PBF_GL_B(LR, T) (first ? ntt_gl_pass_kernel<LR, E, true, T, true> : ntt_gl_pass_kernel<LR, E, false, T, true>)
  switch (logr) {
    case 6: return PBF_GL_B(6, 4096);
    case 7: return PBF_GL_B(7, 4096);
    case 8: return PBF_GL_B(8, 4096);
    case 9: return PBF_GL_B(9, 4096);
    case 10: return PBF_GL_B(10, 8192);
    default: return nullptr;
  }
#undef PBF_GL_B
}

// the regrouped 2^24 plan's three pass kernels
template <int E>
static GlPassFn gl_fn_rg(int pass) {
  if (pass == 0) return ntt_gl_pass_kernel<8, E, true, 4096, false, 1>;
  if (pass == 1) return getenv("PBF_NTT_T2GEO") ? ntt_gl_rg2_kernel<E, true> : ntt_gl_rg2_kernel<E, false>;
  return ntt_gl_pass_kernel<8, E, false, 4096, false, 3>;
}

// one pass launch of a group, recorded instead of launched (the dual-group schedule below)
struct GlLaunch {
  GlPassFn fn;
  uint32_t grid, block;
  size_t lds;
  GlPassArgs a;
};

// Passes of a standard-root Goldilocks plan through ntt_gl_pass_kernel (ntt_gl.hpp).
static int run_gl_group(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                        DevBuf& s1, hipStream_t stream, uint32_t split_log, size_t soff = 0,
                        std::vector<GlLaunch>* rec = nullptr);

// Padded intermediates (PBF_NTT_PAD = elements per row, A/B): the scratch between passes i and
// i+1 keeps each of its rows (n / R_(i+1) elements: what pass i+1 reads as one row r) `pad`
// elements apart, breaking the power-of-two strides of the strided reads. Not with the
// persistent or blocked variants.
static uint64_t gl_pad(const NttPlan& p) {
  const char* e = getenv("PBF_NTT_PAD");
  if (!e || !p.gl || p.logr.size() < 2 || getenv("PBF_NTT_PERSIST") || getenv("PBF_NTT_BLK")) return 0;
  const long long v = atoll(e);
  return v > 0 && v <= 4096 ? (uint64_t)v : 0;
}
// elements per polynomial in the scratch buffers
static uint64_t gl_pitch(const NttPlan& p) {
  const uint64_t pad = gl_pad(p);
  uint64_t rows = 0;
  for (size_t i = 1; i < p.logr.size(); ++i) rows = std::max<uint64_t>(rows, 1ull << p.logr[i]);
  return p.n + rows * pad;
}

int ForkSet::ensure(int streams) {
  if (streams > GL_MAX_STREAMS) streams = GL_MAX_STREAMS;
  if (streams > 1 && !fork) PBF_HIP(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  for (int i = 1; i < streams; ++i) {
    if (!aux[i]) PBF_HIP(hipStreamCreateWithFlags(&aux[i], hipStreamNonBlocking));
    if (!join[i]) PBF_HIP(hipEventCreateWithFlags(&join[i], hipEventDisableTiming));
  }
  if (!flags) {
    PBF_HIP(hipMalloc((void**)&flags, GL_MAX_STREAMS * sizeof(uint64_t)));
    PBF_HIP(hipMemset(flags, 0, GL_MAX_STREAMS * sizeof(uint64_t)));
    PBF_HIP(hipDeviceSynchronize());
  }
  return 0;
}

int ForkSet::ensure_q(size_t n) {
  if (n <= qctr_n) return 0;
  if (qctr) {
    PBF_HIP(hipDeviceSynchronize());  // a launch still using the old counters
    PBF_HIP(hipFree(qctr));
    qctr = nullptr;
    qctr_n = 0;
  }
  PBF_HIP(hipMalloc((void**)&qctr, n * sizeof(uint32_t)));
  PBF_HIP(hipMemset(qctr, 0, n * sizeof(uint32_t)));
  PBF_HIP(hipDeviceSynchronize());
  qctr_n = n;
  return 0;
}

ForkSet::~ForkSet() {
  (void)hipSetDevice(device);
  if (qctr) {
    (void)hipDeviceSynchronize();
    (void)hipFree(qctr);
  }
  for (int i = 1; i < GL_MAX_STREAMS; ++i) {
    if (aux[i]) {
      (void)hipStreamSynchronize(aux[i]);
      (void)hipStreamDestroy(aux[i]);
    }
    if (join[i]) (void)hipEventDestroy(join[i]);
  }
  if (fork) (void)hipEventDestroy(fork);
  if (flags) (void)hipFree(flags);
}

// Dual-group schedule of a two-pass plan (round 5, opt-in PBF_NTT_DUAL=1): ONE stream, launches
// {pass 1 of group 0}, {pass 2 of group g-1 + pass 1 of group g} (one launch, the two roles
// interleaved in runs of 8 workgroups so both run at once on every XCD: ntt_gl_dual_kernel),
// ..., {pass 2 of the last group}. Two groups' passes overlap as with the two-stream schedule,
// without its per-call fork and join (cross-queue event waits, ~20 us of idle GPU per call at
// 2^20 x 32: profiles/r04/ntt_2p20_timeline.txt). Measured slower (2^20 x 32: 0.411 against
// 0.357 ms, profiles/r05/dual_ab.log): each launch ends in a tail of its last workgroups that the
// two-stream schedule fills with the other stream's kernel. Returns -1 when the plan has no
// dual-group kernel (the caller falls back to the stream schedule).
typedef void (*GlDualFn)(GlPassArgs, GlPassArgs);
template <int E>
static GlDualFn gl_fn_dual(int logr, int tile) {
  if (logr == 10 && tile == 8192) return ntt_gl_dual_kernel<10, E, 8192>;
  if (logr == 9 && tile == 4096) return ntt_gl_dual_kernel<9, E, 4096>;
  if (logr == 8 && tile == 4096) return ntt_gl_dual_kernel<8, E, 4096>;
  return nullptr;
}

static int run_gl_dual(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, size_t G, DevBuf& s0,
                       DevBuf& s1, hipStream_t stream) {
  if (p.logr.size() != 2 || p.logr[0] != p.logr[1] || batch <= G || p.r4k || gl_pad(p) || getenv("PBF_NTT_BLK") ||
      getenv("PBF_NTT_PERSIST"))
    return -1;
  const int tile = gl_tile(p.logr[0]);
  const GlDualFn dual = p.e64 == 39 ? gl_fn_dual<39>(p.logr[0], tile) : gl_fn_dual<153>(p.logr[0], tile);
  if (!dual) return -1;
  const size_t groups = (batch + G - 1) / G;  // the last one may be smaller
  std::vector<std::vector<GlLaunch>> L(groups);
  for (size_t g = 0; g < groups; ++g) {
    const size_t b = std::min(G, batch - g * G);
    const int rc = run_gl_group(p, d_in + g * G * p.n, d_out + g * G * p.n, b, s0, s1, stream, 0, g * G * gl_pitch(p),
                                &L[g]);
    if (rc) return rc;
    if (L[g].size() != 2 || L[g][0].block != L[g][1].block) return -1;
  }
  auto launch = [&](const GlLaunch& l) -> int {
    hipLaunchKernelGGL(l.fn, dim3(l.grid), dim3(l.block), l.lds, stream, l.a);
    PBF_HIP(hipGetLastError());
    return 0;
  };
  int rc = launch(L[0][0]);
  for (size_t g = 1; g < groups && !rc; ++g) {
    const GlLaunch &sec = L[g - 1][1], &fst = L[g][0];
    if (sec.grid == fst.grid && sec.grid % 8 == 0 && !sec.lds && !fst.lds) {
      hipLaunchKernelGGL(dual, dim3(2 * fst.grid), dim3(fst.block), 0, stream, sec.a, fst.a);
      PBF_HIP(hipGetLastError());
    } else {  // unequal groups (the remainder): the two passes one after the other
      if (!(rc = launch(sec))) rc = launch(fst);
    }
  }
  if (!rc) rc = launch(L[groups - 1][1]);
  return rc;
}

// Work-queue schedule (ntt_gl.hpp ntt_gl_queue_kernel): both passes of an equal-radix two-pass
// plan for the whole batch in one launch on the caller's stream. Returns -1 when the plan or
// batch has no queue form (the caller falls back to the stream schedule).
typedef void (*GlQueueFn)(GlQueueArgs);
template <int E>
static GlQueueFn gl_fn_queue(int logr, int tile, int pub) {
#define PBF_GL_Q(LR, T)                                                                                      \
  if (logr == LR && tile == T)                                                                               \
    return pub == 0 ? ntt_gl_queue_kernel<LR, E, T, 0> : pub == 1 ? ntt_gl_queue_kernel<LR, E, T, 1>        \
                                                                   : ntt_gl_queue_kernel<LR, E, T, 2>;
  PBF_GL_Q(10, 8192)
  PBF_GL_Q(9, 4096)
  PBF_GL_Q(8, 4096)
#undef PBF_GL_Q
  return nullptr;
}

static int run_gl_queue(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                        DevBuf& s1, hipStream_t stream, ForkSet* fork) {
  if (!fork || p.logr.size() != 2 || p.logr[0] != p.logr[1] || p.r4k || gl_pad(p) || getenv("PBF_NTT_BLK") ||
      getenv("PBF_NTT_PERSIST") || getenv("PBF_NTT_NO_PRETW"))
    return -1;
  const int tile = gl_tile(p.logr[0]);
  const char* pe = getenv("PBF_NTT_QPUB");
  const int pub = pe ? atoi(pe) : 1;
  const GlQueueFn fn = p.e64 == 39 ? gl_fn_queue<39>(p.logr[0], tile, pub) : gl_fn_queue<153>(p.logr[0], tile, pub);
  if (!fn) return -1;
  size_t G = batch % 4 == 0 ? 4 : (batch % 2 == 0 ? 2 : 1);
  if (const char* g = getenv("PBF_NTT_QG")) {
    const size_t v = (size_t)atoll(g);
    if (v >= 1 && batch % v == 0) G = v;
  }
  const uint64_t T = p.n / (uint64_t)tile;  // tiles per polynomial and pass
  if ((G * T) % 8 || batch * T * 2 > 0x7fffffffull) return -1;
  std::vector<GlLaunch> L;
  int rc = run_gl_group(p, d_in, d_out, G, s0, s1, stream, 0, 0, &L);
  if (rc) return rc;
  if (L.size() != 2 || L[0].lds || L[1].lds || L[0].block != L[1].block || !L[0].a.post_tw || !L[1].a.skip_pass_tw)
    return -1;
  const size_t groups = batch / G;
  if ((rc = fork->ensure_q(9 + groups))) return rc;
  GlQueueArgs q;
  q.p1 = L[0].a;
  q.p2 = L[1].a;
  q.p1.xcd_kmajor = q.p2.xcd_kmajor = 1;
  q.ctr = fork->qctr;
  q.in_gs = q.out_gs = G * p.n;
  q.scr_gs = G * gl_pitch(p);
  q.per_class = (uint32_t)(G * T / 8);
  q.groups = (uint32_t)groups;
  const char* le = getenv("PBF_NTT_QLAG");
  q.lag = le ? (uint32_t)atoi(le) : 1;
  if (q.lag < 1) q.lag = 1;
  q.total = (uint32_t)(2 * batch * T);
  hipLaunchKernelGGL(fn, dim3(q.total), dim3(L[0].block), 0, stream, q);
  PBF_HIP(hipGetLastError());
  return 0;
}

static int run_gl_passes(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                         DevBuf& s1, hipStream_t stream, uint32_t split_log, ForkSet* fork) {
  // round 6 default: the work-queue schedule (one launch, no second stream) for batches of >= 2
  if (split_log == 0 && batch >= 2 && !env_default_off("PBF_NTT_NO_QUEUE") && !getenv("PBF_NTT_DUAL")) {
    const int rc = run_gl_queue(p, d_in, d_out, batch, s0, s1, stream, fork);
    if (rc != -1) return rc;
  }
  // default schedule (measured best at 2^20 x 32): groups of 4
  // polynomials alternating over two streams once the batch has at least 8
  size_t G = batch >= 8 ? 4 : batch;
  if (const char* g = getenv("PBF_NTT_GROUP")) G = (size_t)atoll(g);
  if (split_log != 0 || G == 0 || G >= batch) return run_gl_group(p, d_in, d_out, batch, s0, s1, stream, split_log);
  if (getenv("PBF_NTT_DUAL") && !getenv("PBF_NTT_STREAMS")) {
    const int rc = run_gl_dual(p, d_in, d_out, batch, G, s0, s1, stream);
    if (rc != -1) return rc;  // -1: this plan has no dual-group form
  }
  // PBF_NTT_STREAMS=k: groups round-robin over the caller's stream and k-1 more (disjoint
  // scratch), so the passes of k groups run concurrently and their phases interleave
  // (the extra streams are the context's own ForkSet; without one everything stays on `stream`)
  int ns = getenv("PBF_NTT_STREAMS") ? atoi(getenv("PBF_NTT_STREAMS")) : 2;
  ns = ns < 1 ? 1 : (ns > GL_MAX_STREAMS ? GL_MAX_STREAMS : ns);
  if (!fork) ns = 1;
  hipStream_t sts[GL_MAX_STREAMS];
  sts[0] = stream;
  // fork / join by stream memory operations (round 5 default; PBF_NTT_EVENTS=1 restores hipEvent
  // waits): a flag written by one stream and waited on by the other resolves faster than an
  // event wait across hardware queues: 2^20 x 32 0.349-0.352 against 0.357-0.360 ms, three
  // alternations on one box (profiles/r05/memop_ab.log)
  // Under rocprofv3 counter collection (ROCPROF_COUNTER_COLLECTION, which serialises dispatches
  // across queues) a stream waiting on a flag that another queue writes never resumes: events
  // there (profiles/r05/memop_prof.log).
  const bool memop = getenv("PBF_NTT_EVENTS") == nullptr && getenv("ROCPROF_COUNTER_COLLECTION") == nullptr;
  uint64_t seq = 0;
  if (ns > 1) {
    int rc = fork->ensure(ns);
    if (rc) return rc;
    for (int i = 1; i < ns; ++i) sts[i] = fork->aux[i];
    if (memop) {
      seq = ++fork->seq;
      PBF_HIP(hipStreamWriteValue64(stream, fork->flags, seq, 0));
      for (int i = 1; i < ns; ++i) PBF_HIP(hipStreamWaitValue64(sts[i], fork->flags, seq, hipStreamWaitValueGte, ~0ull));
    } else {
      PBF_HIP(hipEventRecord(fork->fork, stream));
      for (int i = 1; i < ns; ++i) PBF_HIP(hipStreamWaitEvent(sts[i], fork->fork, 0));
    }
  }
  int gi = 0;
  for (size_t g0 = 0; g0 < batch; g0 += G, ++gi) {
    const size_t b = batch - g0 < G ? batch - g0 : G;
    const int rc = run_gl_group(p, d_in + g0 * p.n, d_out + g0 * p.n, b, s0, s1, sts[gi % ns], 0,
                                ns > 1 ? g0 * gl_pitch(p) : 0);
    if (rc) return rc;
  }
  if (ns > 1) {
    for (int i = 1; i < ns; ++i) {
      if (memop) {
        PBF_HIP(hipStreamWriteValue64(sts[i], fork->flags + i, seq, 0));
        PBF_HIP(hipStreamWaitValue64(stream, fork->flags + i, seq, hipStreamWaitValueGte, ~0ull));
      } else {
        PBF_HIP(hipEventRecord(fork->join[i], sts[i]));
        PBF_HIP(hipStreamWaitEvent(stream, fork->join[i], 0));
      }
    }
  }
  return 0;
}

// The regrouped plan's twiddle tables, built on the first run that takes the regrouped path:
// tc1[a2l][r2][k1] (4096), t2[a1][K] (2^18), t3[f][a0][j] (2^24, n^-1 folded in for the inverse)
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
  std::vector<uint64_t> t3(1ull << 24);
  const uint64_t scale = inverse ? p.n_inv : 1;
  for (uint64_t fq = 0; fq < 4; ++fq)
    for (uint64_t a0 = 0; a0 < 64; ++a0) {
      const uint64_t st = hpow(w, a0, m);
      uint64_t y = hmul(hpow(w, (65536 * a0 * fq) % n, m), scale, m);
      uint64_t* row = t3.data() + ((fq * 64 + a0) << 16);
      for (uint64_t j = 0; j < 65536; ++j) { row[j] = y; y = hmul(y, st, m); }
    }
  // the last pass's twiddle w^(a0 X) (a0 = r2 + 4 s2, X = 65536 f + j) as C[r2][X] D[X]^s2 with
  // C = w^(r2 X) (n^-1 folded in for the inverse), D = w^(4 X): 10 MiB instead of 128
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
  std::vector<uint64_t> t2d(64);
  for (uint64_t a1 = 0; a1 < 64; ++a1) t2d[a1] = hpow(w, (16384 * a1) % n, m);
  if ((rc = upload(p.rg_tc1, tc1)) || (rc = upload(p.rg_t2, t2)) || (rc = upload(p.rg_t3, t3)) ||
      (rc = upload(p.rg_tgc, tgc)) || (rc = upload(p.rg_tgb, tgb)) || (rc = upload(p.rg_t2d, t2d)))
    return rc;
  p.rg_built = true;
  return 0;
}

// The two-pass plan's tables (ntt_r4k.hpp): tst[b][c] = w_4096^(b c) for pass 1, the same times
// n^-1 for an inverse's pass 2, post[j][k] = w^(j k) (2^24 entries) for pass 1's stores
static int ensure_r4k_tables(const NttPlan& p) {
  if (p.r4k_built) return 0;
  const uint64_t m = p.m;
  uint64_t w = p.omega;
  if (p.inverse && !hinv(p.omega, m, &w)) return fail(1, "omega not invertible");
  const uint64_t w4096 = hpow(w, 4096, m);
  std::vector<uint64_t> t1(4096), t2(4096);
  for (uint64_t b = 0; b < 64; ++b)
    for (uint64_t c = 0; c < 64; ++c) {
      t1[b * 64 + c] = hpow(w4096, b * c, m);
      t2[b * 64 + c] = p.inverse ? hmul(t1[b * 64 + c], p.n_inv, m) : t1[b * 64 + c];
    }
  std::vector<uint64_t> post(1ull << 24);
  for (uint64_t j = 0; j < 4096; ++j) {
    const uint64_t st = hpow(w, j, m);
    uint64_t y = 1;
    uint64_t* row = post.data() + (j << 12);
    for (uint64_t k = 0; k < 4096; ++k) { row[k] = y; y = hmul(y, st, m); }
  }
  int rc;
  if ((rc = upload(p.r4k_tst1, t1)) || (rc = upload(p.r4k_tst2, t2)) || (rc = upload(p.r4k_post, post))) return rc;
  p.r4k_built = true;
  return 0;
}

// ntt_r4k.hip
int launch_r4k_pass(const R4kArgs& a, bool first, int e64, uint32_t tiles, bool persist, hipStream_t stream);

static int run_r4k(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                   hipStream_t stream, size_t soff) {
  int rc = ensure_r4k_tables(p);
  if (rc) return rc;
  if (batch * 512 > 0x7fffffffull) return fail(1, "batch too large");
  R4kArgs a;
  a.batch = (uint32_t)batch;
  a.kmajor = batch > 1 && !getenv("PBF_NTT_NO_KMAJOR") ? 1 : 0;
  const uint32_t grid = (uint32_t)(512 * batch);
  // pass 1: in -> s0 (inter-pass twiddle applied at the stores)
  a.in = d_in;
  a.out = (uint64_t*)s0.p + soff;
  a.tst = (const uint64_t*)p.r4k_tst1.p;
  a.post = (const uint64_t*)p.r4k_post.p;
  a.scaled = 0;
  const char* mode = getenv("PBF_NTT_R4K");
  const bool persist = mode && mode[0] == '2';
  if ((rc = launch_r4k_pass(a, true, p.e64, grid, persist, stream))) return rc;
  // pass 2: s0 -> out (n^-1 in the stage table of an inverse)
  a.in = (const uint64_t*)s0.p + soff;
  a.out = d_out;
  a.tst = (const uint64_t*)p.r4k_tst2.p;
  a.post = nullptr;
  a.scaled = p.inverse ? 1 : 0;
  if ((rc = launch_r4k_pass(a, false, p.e64, grid, persist, stream))) return rc;
  return 0;
}

static int run_gl_group(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                        DevBuf& s1, hipStream_t stream, uint32_t split_log, size_t soff, std::vector<GlLaunch>* rec) {
  if (p.r4k && split_log == 0 && gl_pad(p) == 0) return run_r4k(p, d_in, d_out, batch, s0, stream, soff);
  const size_t P = p.logr.size();
  // two-pass plans with equal tile widths may keep the intermediate blocked (ntt_gl.hpp BLK)
  bool blk = false;
  uint32_t blk_log = 0;
  // opt-in (PBF_NTT_BLK): measured level with the natural layout
  if (P == 2 && getenv("PBF_NTT_BLK") && !getenv("PBF_NTT_PERSIST")) {
    const int t0 = gl_tile(p.logr[0]), t1 = gl_tile(p.logr[1]);
    const uint64_t w0 = (uint64_t)t0 >> p.logr[0], w1 = (uint64_t)t1 >> p.logr[1];
    const bool dflt = (t0 == (p.logr[0] >= 10 ? 8192 : 4096)) && (t1 == (p.logr[1] >= 10 ? 8192 : 4096));
    if (w0 == w1 && dflt && (p.n >> p.logr[0]) % w0 == 0 && (p.n >> p.logr[1]) % w1 == 0) {
      blk = true;
      while ((1ull << blk_log) < w1) ++blk_log;
    }
  }
  const bool rg = p.rg && P == 3 && split_log == 0 && !blk && gl_pad(p) == 0 && !getenv("PBF_NTT_PERSIST") &&
                  gl_tile(8) == 4096;
  if (rg) {
    const int rc = ensure_rg_tables(p);
    if (rc) return rc;
  }
  uint32_t log_ns = 0;
  for (size_t i = 0; i < P; ++i) {
    const int lr = p.logr[i];
    const int tile = gl_tile(lr);
    const bool persist = getenv("PBF_NTT_PERSIST") != nullptr;  // A/B: pipelined persistent kernel
    GlPassFn fn =
        p.e64 == 39 ? gl_fn_e<39>(lr, log_ns == 0, tile, persist) : gl_fn_e<153>(lr, log_ns == 0, tile, persist);
    if (blk) fn = p.e64 == 39 ? gl_fn_blk<39>(lr, log_ns == 0) : gl_fn_blk<153>(lr, log_ns == 0);
    if (rg) fn = p.e64 == 39 ? gl_fn_rg<39>((int)i) : gl_fn_rg<153>((int)i);
    if (!fn) return fail(1, "no Goldilocks pass kernel for this radix");
    const uint64_t W = (uint64_t)tile >> lr;
    if ((p.n >> lr) % W) return fail(1, "transform too small for the pass tile");
    GlPassArgs a;
    a.in = (i == 0) ? d_in : (const uint64_t*)(((i - 1) & 1) ? s1.p : s0.p) + soff;
    a.out = (i == P - 1) ? d_out : (uint64_t*)((i & 1) ? s1.p : s0.p) + soff;
    const uint64_t pad = blk ? 0 : gl_pad(p), pitch = gl_pitch(p);
    a.in_pitch = (i == 0) ? p.n : pitch;
    a.out_pitch = (i == P - 1) ? p.n : pitch;
    a.in_pad = (i == 0) ? 0 : (uint32_t)pad;
    a.out_pad = (i == P - 1) ? 0 : (uint32_t)pad;
    a.out_rows_log = (i == P - 1) ? 0 : p.log_n - (uint32_t)p.logr[i + 1];
    a.twpass = (const uint64_t*)p.twpass[i]->p;
    a.tw0 = (const uint64_t*)p.tw0.p;
    a.tw1 = (const uint64_t*)p.tw1.p;
    a.tc = (const uint64_t*)p.tc[i]->p;
    const bool tws = !a.twpass && i == P - 1 && p.tws_a && (uint64_t)p.tws_w == W && !blk;
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
    a.xcd_kmajor = (log_ns > 0 && batch > 1 && tiles % 8 == 0 && !getenv("PBF_NTT_NO_KMAJOR")) ? 1 : 0;
    a.blk_log = blk_log;
    // two-pass plans apply the second pass's twiddle w^(j k) at the first pass's stores (the
    // first pass hides the product under its memory phase: 2^20 x 32 0.400 -> 0.386 ms,
    // DESIGN.md §3.1); PBF_NTT_NO_PRETW=1 restores it at the second pass's loads
    a.post_tw = nullptr;
    a.skip_pass_tw = 0;
    if (P == 2 && !blk && pad == 0 && split_log == 0 && !persist && !getenv("PBF_NTT_NO_PRETW") && p.twpass[1]->p) {
      if (i == 0) a.post_tw = (const uint64_t*)p.twpass[1]->p;
      else a.skip_pass_tw = 1;
    }
    // the first pass of a 2-pass plan reads the second pass's twiddle table by column too
    // (post_tw): k-major keeps its rows in the XCD's L2 across the polynomials of a block
    // (round 4: 2^20 x 32 0.354-0.357 ms against 0.368-0.371 linear, profiles/r04/ntt_orders_sweep.log)
    if (a.post_tw && batch > 1 && tiles % 8 == 0 && !getenv("PBF_NTT_NO_KMAJOR")) a.xcd_kmajor = 1;
    if (rg && i == 0) a.tc = (const uint64_t*)p.rg_tc1.p;
    if (rg && i == 1) a.twpass = (const uint64_t*)p.rg_t2.p;
    if (rg && i == 1 && getenv("PBF_NTT_T2GEO")) a.tws_b = (const uint64_t*)p.rg_t2d.p;  // A/B (ntt_gl_rg2_kernel)
    if (rg && i == 2) a.twpass = (const uint64_t*)p.rg_t3.p;
    // round 5: the last pass forms its twiddles as C[r2][X] D[X]^s2 from 10 MiB of tables instead
    // of reading the 128 MiB T3 (one more product per element): 2 x 2^24 0.390-0.392 against
    // 0.411-0.412 ms, three alternations (profiles/r05/t3geo_ab.log); PBF_NTT_T3GEO=0 reads T3
    const char* geo_env = getenv("PBF_NTT_T3GEO");
    if (rg && i == 2 && !(geo_env && geo_env[0] == '0')) {
      a.twpass = nullptr;
      a.tws_a = (const uint64_t*)p.rg_tgc.p;
      a.tws_b = (const uint64_t*)p.rg_tgb.p;
    }
    // the regrouped 2^24 plan takes the XCD-blocked order in every pass (round 4: 2 x 2^24
    // 0.433-0.437 ms against 0.447-0.453 k-major, 0.462-0.466 linear, five alternations on one
    // box, profiles/r04/ntt_order24_ab.log); the 2-pass plans keep k-major (2^20 x 32: 0.352-0.355
    // k-major against 0.362-0.364, profiles/r04/ntt_order_ab.log)
    if (rg && tiles % 8 == 0) a.xcd_kmajor = 2;
    // round 5: the last pass takes XCD k-major instead (both polynomials of a column block on one
    // XCD, so each slice of its 128 MiB T3 table is read into one L2 once, not once per XCD of
    // each polynomial): calibrated traffic 1.886 -> 1.753 GB per 2 x 2^24 step, time level
    // (0.4375-0.4433 against 0.4362-0.4379 ms, profiles/r05/order24.log)
    // With the geometric last pass (below) there is no T3 to share: XCD-blocked again (orders 222
    // 0.3867-0.3868 against 221 0.3918-0.3930 ms, profiles/r05/order_geo.log)
    const char* geo_off = getenv("PBF_NTT_T3GEO");
    if (rg && i == 2 && batch > 1 && tiles % 8 == 0 && geo_off && geo_off[0] == '0') a.xcd_kmajor = 1;
    if (const char* o = getenv("PBF_NTT_ORDER")) {  // A/B: 0 linear, 1 k-major per XCD, 2 XCD-blocked
      const uint32_t ord = (uint32_t)atoi(o);
      a.xcd_kmajor = (tiles % 8 == 0 && (ord != 1 || batch > 1)) ? ord : 0;
    }
    if (const char* o = getenv("PBF_NTT_ORDERS")) {  // A/B: one digit per pass, e.g. "021"
      if (strlen(o) > i && o[i] >= '0' && o[i] <= '2') {
        const uint32_t ord = (uint32_t)(o[i] - '0');
        a.xcd_kmajor = (tiles % 8 == 0 && (ord != 1 || batch > 1)) ? ord : 0;
      }
    }
    const uint32_t grid = persist ? persistent_grid((const void*)fn, tile / 16, tiles) : (uint32_t)tiles;
    // A/B diagnostic: extra dynamic LDS per workgroup (PBF_NTT_LDSPAD bytes) lowers the
    // workgroups resident per CU without changing the code
    const size_t ldspad = getenv("PBF_NTT_LDSPAD") ? (size_t)atoll(getenv("PBF_NTT_LDSPAD")) : 0;
    if (rec) {
      rec->push_back(GlLaunch{fn, grid, (uint32_t)(tile / 16), ldspad, a});
    } else {
      hipLaunchKernelGGL(fn, dim3(grid), dim3(tile / 16), ldspad, stream, a);
      PBF_HIP(hipGetLastError());
    }
    log_ns += lr;
  }
  return 0;
}

static int run_plan_impl(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0,
                         DevBuf& s1, hipStream_t stream, uint32_t split_log, ForkSet* fork) {
  if (batch == 0) return 0;
  if (p.ip && split_log == 0 && p.n > 1) return run_ip(p, d_in, d_out, batch, s0, stream);
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
  const size_t bytes = batch * (p.gl ? gl_pitch(p) : p.n) * 8;
  int rc = s0.ensure(bytes);
  if (!rc && P > 2 && !(p.r4k && split_log == 0 && gl_pad(p) == 0)) rc = s1.ensure(bytes);
  if (rc) return rc;
  uint32_t log_ns = 0;
  if (p.gl) return run_gl_passes(p, d_in, d_out, batch, s0, s1, stream, split_log, fork);
  for (size_t i = 0; i < P; ++i) {
    const int lr = p.logr[i];
    PassCfg cfg = pass_cfg(lr);
    PassFn fn = pass_fn(p.kind, p.e64, lr, cfg);
    for (int w : {16, 8, 4}) {  // robust fallback: any instantiated single-tile shape
      if (fn) break;
      cfg = PassCfg{w, 4, 0};
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
    a.twfull = (const uint64_t*)p.twfull.p;
    a.twpass = (const uint64_t*)p.twpass[i]->p;
    a.n = p.n;
    a.n_inv = p.n_inv;
    a.log_n = p.log_n;
    a.log_ns = log_ns;
    a.tw_bits = p.tw_bits;
    a.blocks_per_poly = (uint32_t)((p.n >> lr) / W);
    a.scale = (p.inverse && i == P - 1) ? 1 : 0;
    a.out_split_log = (i == P - 1) ? split_log : 0;
    a.dbg = getenv("PBF_NTT_DBG") ? (uint32_t)atoi(getenv("PBF_NTT_DBG")) : 0;
    a.batch = (uint32_t)batch;
    a.f = p.fa;
    const int nt = cfg.nt ? cfg.nt : (W << lr) >> cfg.lq;
    const uint64_t blocks = (uint64_t)a.blocks_per_poly * batch;
    if (blocks > 0x7fffffffull) return fail(1, "batch too large");
    const uint32_t grid = cfg.db ? persistent_grid((const void*)fn, nt, blocks) : (uint32_t)blocks;  // modes 1, 2: persistent
    a.xcd_kmajor = (!cfg.db && log_ns > 0 && batch > 1 && grid % 8 == 0 && !getenv("PBF_NTT_NO_KMAJOR")) ? 1 : 0;
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
