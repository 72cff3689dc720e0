// Host-side internals of libpbf.so shared by the translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>
#include "field.hpp"

struct pbf_ctx;

namespace pbf {

typedef unsigned __int128 u128;
static const uint64_t GOLDILOCKS = 0xFFFFFFFF00000001ull;

enum FieldKind { FIELD_GOLDILOCKS = 0, FIELD_MOD32 = 1 };

void set_error(const std::string& s);

// Context options (pbf_ctx_set_option, include/pbf.h): named string values that select among
// product code paths (plan shapes, schedules, the proving-key and verification-key caches),
// set per context by the caller. The library never reads them from the environment, so a
// stray variable cannot change what a context computes or how. A plan
// keeps a copy of its context's options from when it was built.
struct Options {
  std::map<std::string, std::string> kv;
  const char* get(const char* name) const {
    auto it = kv.find(name);
    return it == kv.end() ? nullptr : it->second.c_str();
  }
  long long num(const char* name, long long dflt) const {
    const char* v = get(name);
    return v && *v ? atoll(v) : dflt;
  }
};

// A/B switches of measured-negative or diagnostic variants kept for experiments: read from the
// environment ONLY in the A/B build (make ab: -DPBF_AB, libpbf_ab.so). The product build
// compiles them to their defaults and ignores the environment.
inline const char* ab_env(const char* name) {
#ifdef PBF_AB
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}
// A/B switch that is on by default: off only when the variable parses as the integer 0.
inline bool env_default_on(const char* name) {
  const char* e = ab_env(name);
  return !(e && *e && atoi(e) == 0);
}
// A/B switch that is off by default: on only when the variable parses as a nonzero integer.
inline bool env_default_off(const char* name) {
  const char* e = ab_env(name);
  return e && *e && atoi(e) != 0;
}
int fail(int code, const std::string& s);

#define PBF_HIP(expr)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return ::pbf::fail(3 /*PBF_EDEVICE*/, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ---- host modular arithmetic (table generation, validation) ----
inline uint64_t hmul(uint64_t a, uint64_t b, uint64_t m) { return (uint64_t)(((u128)a * b) % m); }
inline uint64_t hpow(uint64_t a, uint64_t e, uint64_t m) {
  uint64_t r = 1 % m;
  while (e) {
    if (e & 1) r = hmul(r, a, m);
    a = hmul(a, a, m);
    e >>= 1;
  }
  return r;
}
// extended gcd inverse; false when gcd != 1 (u64field.rs:52-63 returns None)
bool hinv(uint64_t a, uint64_t m, uint64_t* out);

// Classify a modulus into a device field; false if unsupported.
bool field_for(uint64_t m, FieldKind* kind, FieldArgs* fa);

// Device buffer that grows on demand (freed by the context).
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t need);
  void release();  // frees the allocation (ensure() allocates again)
  ~DevBuf();
};

// A planned NTT: (modulus, omega, n, direction) -> passes + device twiddle tables.
struct NttPlan {
  uint64_t m = 0, omega = 0, n = 0;
  int inverse = 0;
  FieldKind kind = FIELD_GOLDILOCKS;
  FieldArgs fa{};
  uint32_t log_n = 0;
  uint64_t n_inv = 1;
  Options opts;            // the context's options when the plan was built
  std::vector<int> logr;   // radix per pass (empty => small kernel)
  int e64 = -1;            // w_64 = 2^e64 for a standard Goldilocks root, else -1
  std::vector<std::shared_ptr<DevBuf>> twpass;  // per-pass [r][k] twiddles (empty buffer => two-level)
  int w = 16;              // columns per workgroup
  uint32_t tw_bits = 0;
  DevBuf tw0, tw1, small_tw;
  std::vector<std::shared_ptr<DevBuf>> rtab;  // per pass
  bool gl = false;         // passes run on ntt_gl_pass_kernel (standard Goldilocks roots)
  std::vector<std::shared_ptr<DevBuf>> tc;    // per pass: stage-C tables of ntt_gl_pass_kernel
  // last pass without a full [r][k] table: w^(r k) = B[kb][r] * A[r][w] for k = kb*W + w
  // (A: R x W, B: Ns/W x R; null when unused), W = tws_w columns per tile
  std::shared_ptr<DevBuf> tws_a, tws_b;
  int tws_w = 0;
  // regrouped 2^24 plan (ntt_gl.hpp ntt_gl_rg2_kernel): 8,8,8 passes with the general
  // twiddles between 64-point blocks only; tables tc1[a2l][r2][k1] (4096), t2[a1][K] (2^18),
  // and the last pass's geometric factors C[r2][X], D[X] (X < 2^18, n^-1 folded into C for the
  // inverse). rg: the plan qualifies; the tables (~12 MiB) are built the first time a run takes
  // the regrouped path (ntt_launch.hip ensure_rg_tables), never for runs that cannot
  bool rg = false;
  mutable bool rg_built = false;
  mutable DevBuf rg_tc1, rg_t2;
  mutable DevBuf rg_tgc, rg_tgb;
};

// Extra streams and events of the multi-stream NTT group schedule (ntt_launch.hip
// run_gl_passes). Owned by one context (created lazily on its device, destroyed with it),
// so distinct contexts never share or race on them (include/pbf.h "Streams").
constexpr int GL_MAX_STREAMS = 8;
struct ForkSet {
  int device = 0;
  hipStream_t aux[GL_MAX_STREAMS] = {};  // aux[0] unused: slot 0 is the caller's stream
  hipEvent_t fork = nullptr, join[GL_MAX_STREAMS] = {};
  int ensure(int streams);               // streams 1..streams-1 and the event pair exist
  ~ForkSet();
};

// The asynchronous tail of the fixed-base MSM (msm.hip msm_fixed_device): after the
// accumulation, the latency-bound bucket join and reduction run on a context-owned side
// stream while the caller's stream goes on; MSM_TAIL_SLOTS workspaces rotate between the
// MSMs in flight. msm_fixed_wait orders a stream after every tail enqueued so far.
constexpr int MSM_TAIL_SLOTS = 3;
// The prep stream (round 4, opt-in PBF_MSM_PREP=1: measured no faster, msm.hip
// msm_scalars_ready): a caller that commits several polynomials that are all ready
// (msm_scalars_ready, then msm_fixed_device with that event) gets each MSM's digits, sort and
// bucket bounds enqueued on `prep`, so they run while the caller's stream accumulates the
// previous MSM (the sort is memory-bound, the accumulation VALU-bound). MSM_PREP_SLOTS sets of
// sort buffers rotate; prep_free[p] (recorded after the accumulation that read slot p) orders
// their reuse.
constexpr int MSM_PREP_SLOTS = 2;
struct MsmTail {
  int device = 0;
  hipStream_t aux = nullptr;
  hipEvent_t ready[MSM_TAIL_SLOTS] = {}, done[MSM_TAIL_SLOTS] = {};
  bool used[MSM_TAIL_SLOTS] = {};
  int next = 0, last = -1;
  hipStream_t prep = nullptr;
  hipEvent_t prep_done[MSM_PREP_SLOTS] = {}, prep_free[MSM_PREP_SLOTS] = {}, sc_ready = nullptr;
  bool prep_used[MSM_PREP_SLOTS] = {};
  int prep_next = 0;
  int ensure();
  ~MsmTail();  // waits for the side streams (declared after the buffers they use)
};

// Build a plan (validates omega's order and n^-1). Returns PBF status.
int make_plan(uint64_t m, uint64_t omega, uint64_t n, int inverse, NttPlan* p);
// Enqueue a batched transform of a planned size on `stream` (d_in may equal d_out).
// `fork` (the context's ForkSet) allows the multi-stream group schedule for large
// Goldilocks batches; null keeps every launch on `stream`.
int run_plan(const NttPlan& p, const uint64_t* d_in, uint64_t* d_out, size_t batch, DevBuf& s0, DevBuf& s1,
             hipStream_t stream, ForkSet* fork = nullptr);
// Kernel launchers (ntt_launch.hip)
int launch_pointwise_mul(FieldKind k, const FieldArgs& fa, const uint64_t* a, const uint64_t* b, uint64_t* c,
                         uint64_t count, hipStream_t s);
int launch_poly_eval(FieldKind k, const FieldArgs& fa, const uint64_t* d_coeffs, uint64_t n, const uint64_t* d_xs,
                     uint64_t nx, uint64_t* d_ys, DevBuf& partial, hipStream_t s);
// Multi-GPU stride-sharded NTT pieces
struct TwoLevel {
  DevBuf t0, t1;
  uint64_t root = 0;
  uint32_t bits = 0;
};
int make_two_level(uint64_t m, uint64_t root, uint64_t n, TwoLevel* t);
int run_plan_split(const NttPlan& p, const uint64_t* d_in, uint64_t* d_send, size_t batch, uint32_t G, DevBuf& s0,
                   DevBuf& s1, DevBuf& s2, hipStream_t stream);
int launch_shard_combine(FieldKind k, const FieldArgs& fa, const TwoLevel& tl, uint32_t G, uint64_t rank,
                         const uint64_t* in, uint64_t* out, uint64_t nl, uint32_t batch, int inverse, hipStream_t s);
int launch_shard_unsplit(const uint64_t* recv, uint64_t* out, uint64_t nl, uint32_t batch, uint32_t G,
                         hipStream_t s);
int launch_fill_random(const FieldArgs& fa, FieldKind k, uint64_t seed, uint64_t* d_out, uint64_t count,
                       hipStream_t s);

// Plonk::verify's KZG pairing check on a given stream (pairing.hip)
int pairing_check_on_stream(pbf_ctx* ctx, const uint64_t* g1, const uint64_t* g2, size_t n, int* ok, hipStream_t s);

}  // namespace pbf

struct pbf_ctx {
  int device = 0;
  pbf::Options options;  // pbf_ctx_set_option
  uint64_t serial = 0;  // creation order (multi-GPU groups match contexts by pointer and serial)
  hipStream_t stream = nullptr;
  hipStream_t user_stream = nullptr;
  std::map<std::tuple<uint64_t, uint64_t, uint64_t, int>, std::unique_ptr<pbf::NttPlan>> plans;
  pbf::DevBuf scratch0, scratch1, scratch2, io0, io1, io2, partial;
  pbf::ForkSet fork;  // aux streams of the NTT group schedule (this context only)
  // fixed-base MSM window table (msm.hip msm_fixed_table): the points it was built from
  struct FixedBase {
    bool valid = false;  // built from the points in snapshot "fx.pts" (msm.hip snapshot_check)
    uint64_t n = 0;
    int c = 16;  // window bits of the table (msm.hip FxGeom): ceil(255 / c) windows of n points
    pbf::DevBuf table;
    pbf::DevBuf inf;  // per point: 1 = the identity (contributes nothing)
  } fixed_base;
  std::map<std::tuple<uint64_t, uint64_t, uint64_t>, std::unique_ptr<pbf::TwoLevel>> two_level;
  int roots(uint64_t m, uint64_t root, uint64_t n, pbf::TwoLevel** out);
  // `_dev` entry points enqueue on exactly the stream they are given (NULL = the
  // HIP null stream); the synchronous host-pointer entry points use host_stream().
  static hipStream_t pick(void* s) { return (hipStream_t)s; }
  hipStream_t host_stream() const { return user_stream ? user_stream : stream; }
  int plan(uint64_t m, uint64_t omega, uint64_t n, int inverse, pbf::NttPlan** out);
  // named scratch buffers of the larger pipelines (prover), freed with the context
  std::map<std::string, std::unique_ptr<pbf::DevBuf>> named;
  pbf::DevBuf& buf(const std::string& name) {
    auto& b = named[name];
    if (!b) b.reset(new pbf::DevBuf());
    return *b;
  }
  // snapshots of cache inputs (msm.hpp snapshot_check): device copies in buf("snap." + name),
  // their lengths in u64 words here
  std::map<std::string, uint64_t> snap_words;
  // one snapshot per input (named after the data: "q", "copies", "g1pts"), shared by every
  // cache derived from it; snap_gen[name] changes whenever the copy is replaced, and
  // snap_used[consumer + "/" + name] is the generation that consumer's cache was built from
  std::map<std::string, uint64_t> snap_gen, snap_used;
  uint64_t snap_next_gen = 1;
  // pairing check: the G2 inputs whose prepared lines sit in buf("pc.lines") (pairing.hip)
  std::vector<uint64_t> pair_g2_key;
  // prover proving key: the preprocessed polynomials' coefficients and coset evaluations
  // in buf("pk.coef") / buf("pk.coset"), valid for this key (n, world, rank, k1 k2) while the
  // gates and copies equal their snapshots "pk.q" / "pk.copies"
  std::vector<uint64_t> pk_key;
  // verifier verification key: the 8 preprocessed commitments (vk_pts, 8 x 8 u64) of the
  // circuit and SRS in vk_key (n, srs_m, k1 k2) while q, copies and the SRS equal their
  // snapshots "vk.q" / "vk.copies" / "vk.srs"
  std::vector<uint64_t> vk_key, vk_pts;
  pbf::MsmTail msm_tail;  // destroyed before `named`: its stream drains first
};
