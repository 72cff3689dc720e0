// Multi-GPU entry points driven by ONE host process (include/pbf.h "multi-GPU from one
// process"): SURVEY.md §8b's pbf_ntt_u64_multi(ctx[], G, ...) and its Fr, mul_ntt and
// prover analogues. The reference is single-threaded and single-device; these split the top
// log2(G) levels of its even/odd recursion (src/fft.rs:94-96) across G contexts.
//
// The exchange lives in the library. A group of G contexts gets one communicator:
//  * contexts on G distinct devices: RCCL (librccl, loaded at run time with dlopen so the
//    library has no link-time dependency on it), communicators from ncclCommInitAll, every
//    all-to-all as grouped ncclSend / ncclRecv per peer and every all-gather as ncclAllGather,
//    on the rank's stream;
//  * contexts sharing one device (virtual ranks: tests, rehearsals): stream-ordered device
//    copies between the ranks' buffers, ordered by events (no host synchronisation).
// Each rank runs in its own host thread (the prover's rounds synchronise on the host between
// collectives), calling the same stream-ordered kernels as one process per GPU does.
#include <dlfcn.h>
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>
#include "../../include/pbf.h"
#include "internal.hpp"

namespace {
using namespace pbf;

// ---- RCCL, resolved at run time (the subset the group uses; types from rccl.h)
typedef void* nccl_comm_t;
typedef int nccl_result_t;
constexpr int NCCL_UINT8 = 1;  // ncclDataType_t: ncclInt8 = 0, ncclUint8 = 1 (stable in the RCCL / NCCL ABI)
struct Rccl {
  std::string path;  // "" = the process's / ROCm's librccl; else PBF_RCCL_LIB
  void* h = nullptr;
  nccl_result_t (*comm_init_all)(nccl_comm_t*, int, const int*) = nullptr;
  nccl_result_t (*comm_destroy)(nccl_comm_t) = nullptr;
  nccl_result_t (*comm_abort)(nccl_comm_t) = nullptr;
  nccl_result_t (*send)(const void*, size_t, int, int, nccl_comm_t, hipStream_t) = nullptr;
  nccl_result_t (*recv)(void*, size_t, int, int, nccl_comm_t, hipStream_t) = nullptr;
  nccl_result_t (*all_gather)(const void*, void*, size_t, int, nccl_comm_t, hipStream_t) = nullptr;
  nccl_result_t (*group_start)() = nullptr;
  nccl_result_t (*group_end)() = nullptr;
  const char* (*err)(nccl_result_t) = nullptr;
  bool load() {
    if (h) return true;
    if (!path.empty()) {
      h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    } else {
      // reuse a copy already in the process (torch's), else the ROCm one
      for (const char* name : {"librccl.so.1", "librccl.so"})
        if ((h = dlopen(name, RTLD_NOW | RTLD_NOLOAD))) break;
      if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    }
    if (!h) return false;
    comm_init_all = (decltype(comm_init_all))dlsym(h, "ncclCommInitAll");
    comm_destroy = (decltype(comm_destroy))dlsym(h, "ncclCommDestroy");
    comm_abort = (decltype(comm_abort))dlsym(h, "ncclCommAbort");
    send = (decltype(send))dlsym(h, "ncclSend");
    recv = (decltype(recv))dlsym(h, "ncclRecv");
    all_gather = (decltype(all_gather))dlsym(h, "ncclAllGather");
    group_start = (decltype(group_start))dlsym(h, "ncclGroupStart");
    group_end = (decltype(group_end))dlsym(h, "ncclGroupEnd");
    err = (decltype(err))dlsym(h, "ncclGetErrorString");
    return comm_init_all && comm_destroy && comm_abort && send && recv && all_gather && group_start && group_end && err;
  }
};
// one loaded library per path: PBF_RCCL_LIB (read when a group is built) selects a stand-in
// implementation of the same entry points (tests/native/fake_rccl.cpp: exercises this branch
// on one device, where RCCL itself refuses two ranks)
std::mutex g_rccl_mu;
Rccl* rccl_lib() {
  static std::vector<std::unique_ptr<Rccl>> libs;
  const char* e = getenv("PBF_RCCL_LIB");
  const std::string path = e ? e : "";
  std::lock_guard<std::mutex> l(g_rccl_mu);
  for (auto& r : libs)
    if (r->path == path) return r->load() ? r.get() : nullptr;
  libs.emplace_back(new Rccl());
  libs.back()->path = path;
  return libs.back()->load() ? libs.back().get() : nullptr;
}

// reusable barrier for the rank threads of one call; abort() releases every waiter with false
class Barrier {
 public:
  explicit Barrier(uint32_t n) : n_(n) {}
  bool wait() {
    std::unique_lock<std::mutex> l(m_);
    if (aborted_) return false;
    const uint64_t gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
      return true;
    }
    cv_.wait(l, [&] { return gen_ != gen || aborted_; });
    return !aborted_;
  }
  void abort() {
    std::lock_guard<std::mutex> l(m_);
    aborted_ = true;
    cv_.notify_all();
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  uint32_t n_, count_ = 0;
  uint64_t gen_ = 0;
  bool aborted_ = false;
};

struct Group;
// one rank's view (the pbf_comm user pointer)
struct RankComm {
  Group* grp;
  uint32_t rank;
};

struct Group {
  std::vector<pbf_ctx*> ctx;
  std::vector<uint64_t> serial;  // the contexts' creation serials (a destroyed context never matches)
  uint32_t G = 0;
  bool same_device = true;
  bool use_rccl = false;             // distinct devices, or PBF_GROUP_FORCE_RCCL=1 (stand-in tests)
  std::atomic<bool> broken{false};   // communicators aborted after a failure: dropped by group_for
  Rccl* R = nullptr;
  std::vector<nccl_comm_t> nccl;
  std::vector<DevBuf> send, recv;   // per rank, on its device
  std::vector<hipEvent_t> ev_ready, ev_done;
  std::vector<hipStream_t> stream;  // per rank, the stream of the current call
  std::vector<RankComm> rc;
  std::unique_ptr<Barrier> bar;
  // post_mu[r]: held by rank r's thread while it is inside RCCL calls on its communicator
  // (group start .. group end, all-gather), and by abort_all while it aborts that communicator,
  // so no communicator is aborted (freed) while its rank's thread is using it
  std::unique_ptr<std::timed_mutex[]> post_mu;
  size_t capacity = 0;

  ~Group() {
    for (uint32_t g = 0; g < G; ++g) {
      (void)hipSetDevice(ctx_device(g));
      if (g < ev_ready.size() && ev_ready[g]) (void)hipEventDestroy(ev_ready[g]);
      if (g < ev_done.size() && ev_done[g]) (void)hipEventDestroy(ev_done[g]);
      if (g < send.size()) send[g].release();
      if (g < recv.size()) recv[g].release();
    }
    if (!broken)  // aborted communicators are already freed
      for (nccl_comm_t c : nccl)
        if (c) (void)R->comm_destroy(c);
  }
  // a rank failed: release every rank waiting on a host barrier and every collective in flight
  // (ncclCommAbort unblocks peers whose partner never posts its half); the group is then dropped
  // by group_for. `broken` is set first, and a rank checks it under its post_mu before posting,
  // so once abort_all holds post_mu[g], rank g is outside RCCL and never posts again: its
  // communicator is aborted with no other thread inside it. A rank still inside a blocking RCCL
  // call after 5 s (a rendezvous whose partner failed) is aborted anyway, which is how a blocked
  // NCCL / RCCL call is released (the communicator is not freed under the abort of its own
  // call: the stand-in, tests/native/fake_rccl.cpp, keeps that contract too).
  void abort_all() {
    if (bar) bar->abort();
    if (!use_rccl || broken.exchange(true)) return;
    for (uint32_t g = 0; g < G; ++g) {
      if (!nccl[g]) continue;
      std::unique_lock<std::timed_mutex> l(post_mu[g], std::defer_lock);
      (void)l.try_lock_for(std::chrono::seconds(5));
      (void)R->comm_abort(nccl[g]);
    }
  }
  std::vector<int> devs;
  int ctx_device(uint32_t g) const { return devs[g]; }

  int init(pbf_ctx* const* ctxs, uint32_t world) {
    G = world;
    for (uint32_t g = 0; g < G; ++g) {
      ctx.push_back(ctxs[g]);
      serial.push_back(ctxs[g]->serial);
      devs.push_back(ctxs[g]->device);
    }
    for (uint32_t g = 1; g < G; ++g) same_device = same_device && devs[g] == devs[0];
    if (!same_device) {
      std::vector<int> sorted(devs);
      std::sort(sorted.begin(), sorted.end());
      if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
        return fail(PBF_EINVAL, "multi-GPU group: contexts must share one device or all be on distinct devices");
    }
    const char* force = getenv("PBF_GROUP_FORCE_RCCL");  // test only: the RCCL branch on one device
    use_rccl = !same_device || (force && force[0] == '1');
    if (use_rccl) {
      if (!(R = rccl_lib())) {
        const char* e = dlerror();
        return fail(PBF_ECOMM, std::string("multi-GPU group: cannot load librccl: ") + (e ? e : "missing symbols"));
      }
      nccl.assign(G, nullptr);
      const nccl_result_t r = R->comm_init_all(nccl.data(), (int)G, devs.data());
      if (r) return fail(PBF_ECOMM, std::string("ncclCommInitAll: ") + R->err(r));
    }
    send.resize(G);
    recv.resize(G);
    ev_ready.assign(G, nullptr);
    ev_done.assign(G, nullptr);
    stream.assign(G, nullptr);
    for (uint32_t g = 0; g < G; ++g) {
      PBF_HIP(hipSetDevice(devs[g]));
      PBF_HIP(hipEventCreateWithFlags(&ev_ready[g], hipEventDisableTiming));
      PBF_HIP(hipEventCreateWithFlags(&ev_done[g], hipEventDisableTiming));
      rc.push_back(RankComm{this, g});
    }
    bar.reset(new Barrier(G));
    post_mu.reset(new std::timed_mutex[G]);
    return 0;
  }
  int ensure(size_t bytes) {
    for (uint32_t g = 0; g < G; ++g) {
      PBF_HIP(hipSetDevice(devs[g]));
      int r;
      if ((r = send[g].ensure(bytes)) || (r = recv[g].ensure(bytes))) return r;
    }
    capacity = std::min(send[0].bytes, recv[0].bytes);
    return 0;
  }
  // rank r's side of an exchange: `piece(g)` = (source offset in send[g], bytes) of what rank g
  // sends to r, placed at recv[r] + g * b. Same device: wait for every rank's send buffer
  // (events), copy, then every rank waits for every reader before its send buffer is reused.
  int copy_exchange(uint32_t r, size_t b, bool gather) {
    hipStream_t s = stream[r];
    PBF_HIP(hipEventRecord(ev_ready[r], s));
    if (!bar->wait()) return fail(PBF_ECOMM, "multi-GPU group: a rank failed");
    for (uint32_t g = 0; g < G; ++g) {
      PBF_HIP(hipStreamWaitEvent(s, ev_ready[g], 0));
      const char* src = (const char*)send[g].p + (gather ? 0 : (size_t)r * b);
      if (b) PBF_HIP(hipMemcpyAsync((char*)recv[r].p + (size_t)g * b, src, b, hipMemcpyDeviceToDevice, s));
    }
    PBF_HIP(hipEventRecord(ev_done[r], s));
    if (!bar->wait()) return fail(PBF_ECOMM, "multi-GPU group: a rank failed");
    // every reader of send[r] is done before rank r's stream writes it again; the events are
    // recorded again only after the next exchange's first barrier, i.e. after these waits
    for (uint32_t g = 0; g < G; ++g) PBF_HIP(hipStreamWaitEvent(s, ev_done[g], 0));
    return 0;
  }
  // RCCL: every rank passes a host barrier before it posts, so a rank that failed earlier (an
  // allocation, a launch, an input check) releases the others instead of leaving their halves
  // of the exchange without a partner (their stream would never drain)
  int rccl_ready() {
    if (!bar->wait() || broken) return fail(PBF_ECOMM, "multi-GPU group: a rank failed");
    return 0;
  }
  int all_to_all(uint32_t r, size_t b) {
    if (!use_rccl) return copy_exchange(r, b, false);
    if (int rc = rccl_ready()) return rc;
    std::lock_guard<std::timed_mutex> l(post_mu[r]);
    if (broken) return fail(PBF_ECOMM, "multi-GPU group: a rank failed");
    nccl_result_t e = R->group_start();
    for (uint32_t g = 0; g < G && !e; ++g) {
      if ((e = R->send((const char*)send[r].p + (size_t)g * b, b, NCCL_UINT8, (int)g, nccl[r], stream[r]))) break;
      e = R->recv((char*)recv[r].p + (size_t)g * b, b, NCCL_UINT8, (int)g, nccl[r], stream[r]);
    }
    const nccl_result_t e2 = R->group_end();
    if (e || e2) return fail(PBF_ECOMM, std::string("RCCL all-to-all: ") + R->err(e ? e : e2));
    return 0;
  }
  int all_gather(uint32_t r, size_t b) {
    if (!use_rccl) return copy_exchange(r, b, true);
    if (int rc = rccl_ready()) return rc;
    std::lock_guard<std::timed_mutex> l(post_mu[r]);
    if (broken) return fail(PBF_ECOMM, "multi-GPU group: a rank failed");
    const nccl_result_t e = R->all_gather(send[r].p, recv[r].p, b, NCCL_UINT8, nccl[r], stream[r]);
    if (e) return fail(PBF_ECOMM, std::string("ncclAllGather: ") + R->err(e));
    return 0;
  }
  pbf_comm comm(uint32_t r);
  // run fn(rank) on G host threads (device selected); the first failure aborts the others'
  // barriers and is reported with its message
  int run(const std::function<int(uint32_t)>& fn) {
    bar.reset(new Barrier(G));
    std::vector<int> rcs(G, 0);
    std::vector<std::string> msgs(G);
    std::vector<std::thread> ts;
    for (uint32_t g = 0; g < G; ++g)
      ts.emplace_back([&, g] {
        if (hipSetDevice(devs[g]) != hipSuccess) rcs[g] = PBF_EDEVICE;
        else rcs[g] = fn(g);
        if (rcs[g]) {
          msgs[g] = pbf_last_error();
          abort_all();
        }
      });
    for (auto& t : ts) t.join();
    for (uint32_t g = 0; g < G; ++g)  // the root cause: a failure other than a released barrier
      if (rcs[g] && msgs[g].find("a rank failed") == std::string::npos) return fail(rcs[g], "rank " + std::to_string(g) + ": " + msgs[g]);
    for (uint32_t g = 0; g < G; ++g)
      if (rcs[g]) return fail(rcs[g], "rank " + std::to_string(g) + ": " + msgs[g]);
    return 0;
  }
};

int cb_a2a(void* user, size_t b, void* stream) {
  RankComm* rc = (RankComm*)user;
  rc->grp->stream[rc->rank] = (hipStream_t)stream;
  return rc->grp->all_to_all(rc->rank, b);
}
int cb_ag(void* user, size_t b, void* stream) {
  RankComm* rc = (RankComm*)user;
  rc->grp->stream[rc->rank] = (hipStream_t)stream;
  return rc->grp->all_gather(rc->rank, b);
}
pbf_comm Group::comm(uint32_t r) {
  pbf_comm c;
  c.world = G;
  c.rank = r;
  c.user = &rc[r];
  c.send = send[r].p;
  c.recv = recv[r].p;
  c.capacity = capacity;
  c.all_to_all = cb_a2a;
  c.all_gather = cb_ag;
  return c;
}

// groups by their exact member list (pointers and creation serials); a destroyed member drops
// every group it belongs to (pbf_internal_forget_ctx, called by pbf_ctx_destroy)
std::mutex g_groups_mu;
std::vector<std::unique_ptr<Group>>& groups() {
  static std::vector<std::unique_ptr<Group>> v;
  return v;
}
int group_for(pbf_ctx* const* ctxs, uint32_t world, Group** out) {
  if (!ctxs) return fail(PBF_EINVAL, "null context array");
  if (world != 2 && world != 4 && world != 8) return fail(PBF_EINVAL, "world size must be 2, 4 or 8");
  for (uint32_t g = 0; g < world; ++g)
    if (!ctxs[g]) return fail(PBF_EINVAL, "null context");
  for (uint32_t g = 0; g < world; ++g)
    for (uint32_t h = g + 1; h < world; ++h)
      if (ctxs[g] == ctxs[h]) return fail(PBF_EINVAL, "a context appears twice (one context per rank)");
  std::lock_guard<std::mutex> l(g_groups_mu);
  auto& v = groups();  // a group whose communicators were aborted is rebuilt
  v.erase(std::remove_if(v.begin(), v.end(), [](const std::unique_ptr<Group>& g) { return g->broken.load(); }),
          v.end());
  for (auto& gp : groups()) {
    if (gp->G != world) continue;
    bool same = true;
    for (uint32_t g = 0; g < world && same; ++g) same = gp->ctx[g] == ctxs[g] && gp->serial[g] == ctxs[g]->serial;
    if (same) { *out = gp.get(); return 0; }
  }
  std::unique_ptr<Group> gp(new Group());
  int rc = gp->init(ctxs, world);
  if (rc) return rc;
  *out = gp.get();
  groups().push_back(std::move(gp));
  return 0;
}

// ---- host-vector helpers: stride shards out of / blocks into natural order (W u64 per element)
template <int W>
void gather_stride(const uint64_t* in, uint64_t* out, size_t nl, uint32_t G, uint32_t g) {
  for (size_t m = 0; m < nl; ++m) memcpy(out + W * m, in + W * (g + (size_t)G * m), 8 * W);
}
template <int W>
void scatter_stride(const uint64_t* in, uint64_t* out, size_t nl, uint32_t G, uint32_t g) {
  for (size_t m = 0; m < nl; ++m) memcpy(out + W * (g + (size_t)G * m), in + W * m, 8 * W);
}

// One rank's sharded NTT step sequence on device buffers (forward: stride shard -> blocks).
struct NttOps {
  int words;  // u64 per element
  std::function<int(pbf_ctx*, const uint64_t*, uint64_t*, size_t, size_t, int, hipStream_t)> local;
  std::function<int(pbf_ctx*, uint32_t, const uint64_t*, uint64_t*, size_t, size_t, int, hipStream_t)> combine;
};
int sharded_ntt_rank(Group* grp, uint32_t r, const NttOps& ops, const uint64_t* d_in, uint64_t* d_out, size_t nl,
                     size_t batch, int inverse, hipStream_t s) {
  pbf_ctx* c = grp->ctx[r];
  const size_t per = batch * (nl / grp->G) * ops.words * 8;  // bytes per peer
  uint64_t* snd = (uint64_t*)grp->send[r].p;
  const uint64_t* rcv = (const uint64_t*)grp->recv[r].p;
  grp->stream[r] = s;
  int rc;
  if (!inverse) {
    if ((rc = ops.local(c, d_in, snd, nl, batch, 0, s))) return rc;
    if ((rc = grp->all_to_all(r, per))) return rc;
    return ops.combine(c, r, rcv, d_out, nl, batch, 0, s);
  }
  if ((rc = ops.combine(c, r, d_in, snd, nl, batch, 1, s))) return rc;
  if ((rc = grp->all_to_all(r, per))) return rc;
  return ops.local(c, rcv, d_out, nl, batch, 1, s);
}

NttOps u64_ops(uint64_t modulus, uint64_t omega, uint32_t G) {
  NttOps o;
  o.words = 1;
  o.local = [=](pbf_ctx* c, const uint64_t* in, uint64_t* out, size_t nl, size_t b, int inv, hipStream_t s) {
    return pbf_ntt_shard_local_dev(c, modulus, omega, G, in, out, nl, b, inv, s);
  };
  o.combine = [=](pbf_ctx* c, uint32_t r, const uint64_t* in, uint64_t* out, size_t nl, size_t b, int inv,
                  hipStream_t s) { return pbf_ntt_shard_combine_dev(c, modulus, omega, G, r, in, out, nl, b, inv, s); };
  return o;
}
NttOps fr_ops(const uint64_t* omega, uint32_t G) {
  std::array<uint64_t, 4> w;
  memcpy(w.data(), omega, 32);
  NttOps o;
  o.words = 4;
  o.local = [=](pbf_ctx* c, const uint64_t* in, uint64_t* out, size_t nl, size_t b, int inv, hipStream_t s) {
    return pbf_ntt_fr256_shard_local_dev(c, w.data(), G, in, out, nl, b, inv, s);
  };
  o.combine = [=](pbf_ctx* c, uint32_t r, const uint64_t* in, uint64_t* out, size_t nl, size_t b, int inv,
                  hipStream_t s) { return pbf_ntt_fr256_shard_combine_dev(c, w.data(), G, r, in, out, nl, b, inv, s); };
  return o;
}

// whole host vectors through the G ranks: forward NTT (in natural order -> out natural order)
// or inverse; W u64 words per element
int host_ntt_multi(Group* grp, const NttOps& ops, const uint64_t* in, uint64_t* out, size_t n, int inverse) {
  const uint32_t G = grp->G;
  if (n % G || (n / G) < G || ((n / G) & (n / G - 1))) return fail(PBF_EINVAL, "n must be G * (a power of two >= G)");
  const size_t nl = n / G, S = nl / G, W = (size_t)ops.words;
  int rc = grp->ensure(nl * W * 8);
  if (rc) return rc;
  return grp->run([&](uint32_t r) -> int {
    pbf_ctx* c = grp->ctx[r];
    const hipStream_t s = c->host_stream();
    DevBuf &din = c->buf("multi.in"), &dout = c->buf("multi.out");
    int e;
    if ((e = din.ensure(nl * W * 8)) || (e = dout.ensure(nl * W * 8))) return e;
    std::vector<uint64_t> h(nl * W);
    if (!inverse) {  // this rank's stride shard in[r + G m]
      if (W == 1) gather_stride<1>(in, h.data(), nl, G, r);
      else gather_stride<4>(in, h.data(), nl, G, r);
    } else {  // this rank's blocks: X[q nl + r S + kk] at q S + kk
      for (size_t q = 0; q < G; ++q) memcpy(h.data() + W * q * S, in + W * (q * nl + r * S), 8 * W * S);
    }
    PBF_HIP(hipMemcpyAsync(din.p, h.data(), nl * W * 8, hipMemcpyHostToDevice, s));
    if ((e = sharded_ntt_rank(grp, r, ops, (const uint64_t*)din.p, (uint64_t*)dout.p, nl, 1, inverse, s))) return e;
    PBF_HIP(hipMemcpyAsync(h.data(), dout.p, nl * W * 8, hipMemcpyDeviceToHost, s));
    PBF_HIP(hipStreamSynchronize(s));
    if (!inverse) {
      for (size_t q = 0; q < G; ++q) memcpy(out + W * (q * nl + r * S), h.data() + W * q * S, 8 * W * S);
    } else {
      if (W == 1) scatter_stride<1>(h.data(), out, nl, G, r);
      else scatter_stride<4>(h.data(), out, nl, G, r);
    }
    return 0;
  });
}

// mul_ntt (fft.rs:109-132) across the ranks: both operands forward-sharded, pointwise product on
// each rank's blocks, one inverse-sharded transform; out has la + lb = n entries
int host_mul_ntt_multi(Group* grp, const NttOps& ops,
                       const std::function<int(pbf_ctx*, const uint64_t*, const uint64_t*, uint64_t*, size_t,
                                               hipStream_t)>& pointwise,
                       const uint64_t* a, size_t la, const uint64_t* b, size_t lb, uint64_t* out) {
  const uint32_t G = grp->G;
  const size_t n = la + lb;
  if (!la || !lb || n % G || (n / G) < G || ((n / G) & (n / G - 1)))
    return fail(PBF_EINVAL, "la + lb must be G * (a power of two >= G)");
  const size_t nl = n / G, W = (size_t)ops.words;
  int rc = grp->ensure(2 * nl * W * 8);
  if (rc) return rc;
  return grp->run([&](uint32_t r) -> int {
    pbf_ctx* c = grp->ctx[r];
    const hipStream_t s = c->host_stream();
    DevBuf &din = c->buf("multi.in"), &dout = c->buf("multi.out");
    int e;
    if ((e = din.ensure(2 * nl * W * 8)) || (e = dout.ensure(2 * nl * W * 8))) return e;
    std::vector<uint64_t> h(2 * nl * W, 0);
    for (size_t m = 0; m < nl; ++m) {  // zero-padded stride shards of a and b (fft.rs:114-118)
      const size_t j = r + (size_t)G * m;
      if (j < la) memcpy(h.data() + W * m, a + W * j, 8 * W);
      if (j < lb) memcpy(h.data() + W * (nl + m), b + W * j, 8 * W);
    }
    PBF_HIP(hipMemcpyAsync(din.p, h.data(), 2 * nl * W * 8, hipMemcpyHostToDevice, s));
    uint64_t* dI = (uint64_t*)din.p;
    uint64_t* dO = (uint64_t*)dout.p;
    if ((e = sharded_ntt_rank(grp, r, ops, dI, dO, nl, 2, 0, s))) return e;
    if ((e = pointwise(c, dO, dO + W * nl, dI, nl, s))) return e;
    if ((e = sharded_ntt_rank(grp, r, ops, dI, dO, nl, 1, 1, s))) return e;
    PBF_HIP(hipMemcpyAsync(h.data(), dO, nl * W * 8, hipMemcpyDeviceToHost, s));
    PBF_HIP(hipStreamSynchronize(s));
    if (W == 1) scatter_stride<1>(h.data(), out, nl, G, r);
    else scatter_stride<4>(h.data(), out, nl, G, r);
    return 0;
  });
}

// BN254 r (little-endian u64 limbs): Fr inputs are canonical residues, as in the single-GPU calls
bool fr_canonical(const uint64_t* v, size_t n) {
  static const uint64_t R[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull,
                                0x30644e72e131a029ull};
  for (size_t i = 0; i < n; ++i) {
    const uint64_t* x = v + 4 * i;
    int k = 3;
    while (k >= 0 && x[k] == R[k]) --k;
    if (k < 0 || x[k] > R[k]) return false;
  }
  return true;
}
// the _dev forms: every rank holds nl elements per polynomial, a power of two >= G (the
// stride-shard layout and the per-peer blocks of nl / G)
int check_nl(size_t nl, uint32_t G) {
  if (nl < G || (nl & (nl - 1)) || nl % G) return fail(PBF_EINVAL, "nl must be a power of two >= world");
  return 0;
}

}  // namespace

// pbf_ctx_release_caches: the exchange buffers of every group with this member are freed (the
// communicators stay; the next call allocates again)
void pbf_internal_release_group_bufs(const pbf_ctx* c) {
  std::lock_guard<std::mutex> l(g_groups_mu);
  for (auto& g : groups()) {
    if (std::find(g->ctx.begin(), g->ctx.end(), c) == g->ctx.end()) continue;
    for (uint32_t r = 0; r < g->G; ++r) {
      (void)hipSetDevice(g->devs[r]);
      g->send[r].release();
      g->recv[r].release();
    }
    g->capacity = 0;
  }
}

void pbf_internal_forget_ctx(const pbf_ctx* c) {
  std::lock_guard<std::mutex> l(g_groups_mu);
  auto& v = groups();
  v.erase(std::remove_if(v.begin(), v.end(),
                         [&](const std::unique_ptr<Group>& g) {
                           return std::find(g->ctx.begin(), g->ctx.end(), c) != g->ctx.end();
                         }),
          v.end());
}

extern "C" {

int pbf_ntt_u64_multi(pbf_ctx* const* ctxs, uint32_t world, uint64_t modulus, uint64_t omega, const uint64_t* in,
                      uint64_t* out, size_t n, int inverse) {
  if (!in || !out) return fail(PBF_EINVAL, "null argument");
  Group* g;
  int rc = group_for(ctxs, world, &g);
  if (rc) return rc;
  FieldKind k;
  FieldArgs fa;
  if (!field_for(modulus, &k, &fa)) return fail(PBF_EUNSUPPORTED, "unsupported modulus");
  for (size_t i = 0; i < n; ++i)
    if (in[i] >= modulus) return fail(PBF_EINVAL, "input not canonical");
  if (in == out) {  // every rank reads all of `in` before the outputs land: stage a copy
    std::vector<uint64_t> tmp(in, in + n);
    return host_ntt_multi(g, u64_ops(modulus, omega, world), tmp.data(), out, n, inverse);
  }
  return host_ntt_multi(g, u64_ops(modulus, omega, world), in, out, n, inverse);
}

int pbf_ntt_u64_multi_dev(pbf_ctx* const* ctxs, uint32_t world, uint64_t modulus, uint64_t omega,
                          const uint64_t* const* d_in, uint64_t* const* d_out, size_t nl, size_t batch, int inverse,
                          void* const* streams) {
  if (!d_in || !d_out) return fail(PBF_EINVAL, "null argument");
  Group* g;
  int rc = group_for(ctxs, world, &g);
  if (rc) return rc;
  if ((rc = check_nl(nl, world))) return rc;
  if ((rc = g->ensure(batch * nl * 8))) return rc;
  const NttOps ops = u64_ops(modulus, omega, world);
  return g->run([&](uint32_t r) {
    return sharded_ntt_rank(g, r, ops, d_in[r], d_out[r], nl, batch, inverse,
                            streams ? (hipStream_t)streams[r] : (hipStream_t) nullptr);
  });
}

int pbf_ntt_fr256_multi(pbf_ctx* const* ctxs, uint32_t world, const uint64_t* omega, const uint64_t* in, uint64_t* out,
                        size_t n, int inverse) {
  if (!omega || !in || !out) return fail(PBF_EINVAL, "null argument");
  Group* g;
  int rc = group_for(ctxs, world, &g);
  if (rc) return rc;
  if (!fr_canonical(in, n)) return fail(PBF_EINVAL, "input not canonical");
  if (in == out) {
    std::vector<uint64_t> tmp(in, in + 4 * n);
    return host_ntt_multi(g, fr_ops(omega, world), tmp.data(), out, n, inverse);
  }
  return host_ntt_multi(g, fr_ops(omega, world), in, out, n, inverse);
}

int pbf_ntt_fr256_multi_dev(pbf_ctx* const* ctxs, uint32_t world, const uint64_t* omega, const uint64_t* const* d_in,
                            uint64_t* const* d_out, size_t nl, size_t batch, int inverse, void* const* streams) {
  if (!omega || !d_in || !d_out) return fail(PBF_EINVAL, "null argument");
  Group* g;
  int rc = group_for(ctxs, world, &g);
  if (rc) return rc;
  if ((rc = check_nl(nl, world))) return rc;
  if ((rc = g->ensure(batch * nl * 32))) return rc;
  const NttOps ops = fr_ops(omega, world);
  return g->run([&](uint32_t r) {
    return sharded_ntt_rank(g, r, ops, d_in[r], d_out[r], nl, batch, inverse,
                            streams ? (hipStream_t)streams[r] : (hipStream_t) nullptr);
  });
}

int pbf_mul_ntt_u64_multi(pbf_ctx* const* ctxs, uint32_t world, uint64_t modulus, uint64_t omega, const uint64_t* a,
                          size_t la, const uint64_t* b, size_t lb, uint64_t* out) {
  if (!a || !b || !out) return fail(PBF_EINVAL, "null argument");
  Group* g;
  int rc = group_for(ctxs, world, &g);
  if (rc) return rc;
  FieldKind k;
  FieldArgs fa;
  if (!field_for(modulus, &k, &fa)) return fail(PBF_EUNSUPPORTED, "unsupported modulus");
  for (size_t i = 0; i < la; ++i)
    if (a[i] >= modulus) return fail(PBF_EINVAL, "input not canonical");
  for (size_t i = 0; i < lb; ++i)
    if (b[i] >= modulus) return fail(PBF_EINVAL, "input not canonical");
  return host_mul_ntt_multi(
      g, u64_ops(modulus, omega, world),
      [=](pbf_ctx* c, const uint64_t* x, const uint64_t* y, uint64_t* z, size_t cnt, hipStream_t s) {
        return pbf_pointwise_mul_u64_dev(c, modulus, x, y, z, cnt, s);
      },
      a, la, b, lb, out);
}

int pbf_mul_ntt_fr256_multi(pbf_ctx* const* ctxs, uint32_t world, const uint64_t* omega, const uint64_t* a, size_t la,
                            const uint64_t* b, size_t lb, uint64_t* out) {
  if (!omega || !a || !b || !out) return fail(PBF_EINVAL, "null argument");
  Group* g;
  int rc = group_for(ctxs, world, &g);
  if (rc) return rc;
  if (!fr_canonical(a, la) || !fr_canonical(b, lb)) return fail(PBF_EINVAL, "input not canonical");
  return host_mul_ntt_multi(
      g, fr_ops(omega, world),
      [](pbf_ctx* c, const uint64_t* x, const uint64_t* y, uint64_t* z, size_t cnt, hipStream_t s) {
        return pbf_pointwise_mul_fr256_dev(c, x, y, z, cnt, s);
      },
      a, la, b, lb, out);
}

int pbf_plonk_prove_bn254_multi_dev(pbf_ctx* const* ctxs, uint32_t world, size_t n, const uint64_t* const* d_q,
                                    const uint64_t* const* d_copies, const uint64_t* const* d_abc, const uint64_t* chal,
                                    const uint64_t* rnd, const uint64_t* k1k2, const uint64_t* const* d_srs,
                                    size_t srs_m, int mode, uint64_t* out_pts, uint64_t* out_f, void* const* streams) {
  if (!d_q || !d_copies || !d_abc || !d_srs || !out_pts || !out_f) return fail(PBF_EINVAL, "null argument");
  Group* g;
  int rc = group_for(ctxs, world, &g);
  if (rc) return rc;
  if ((rc = g->ensure((size_t)5 * (4 * n / world) * 32))) return rc;
  std::vector<uint64_t> pts((size_t)world * 72), fs((size_t)world * 28);
  rc = g->run([&](uint32_t r) {
    const pbf_comm c = g->comm(r);
    return pbf_plonk_prove_bn254_sharded_dev(g->ctx[r], &c, n, d_q[r], d_copies[r], d_abc[r], chal, rnd, k1k2, d_srs[r],
                                             srs_m, mode, pts.data() + 72 * r, fs.data() + 28 * r,
                                             streams ? streams[r] : nullptr);
  });
  if (rc) return rc;
  for (uint32_t r = 1; r < world; ++r)
    if (memcmp(pts.data(), pts.data() + 72 * r, 72 * 8) || memcmp(fs.data(), fs.data() + 28 * r, 28 * 8))
      return fail(PBF_ECOMM, "ranks disagree on the proof");
  memcpy(out_pts, pts.data(), 72 * 8);
  memcpy(out_f, fs.data(), 28 * 8);
  return 0;
}

int pbf_plonk_prove_bn254_multi(pbf_ctx* const* ctxs, uint32_t world, size_t n, const uint64_t* q, const uint64_t* copies,
                                const uint64_t* abc, const uint64_t* chal, const uint64_t* rnd, const uint64_t* k1k2,
                                const uint64_t* srs, size_t srs_m, int mode, uint64_t* out_pts, uint64_t* out_f) {
  if (!q || !copies || !abc || !srs) return fail(PBF_EINVAL, "null argument");
  Group* g;
  int rc = group_for(ctxs, world, &g);
  if (rc) return rc;
  // the circuit, witness and SRS on every rank's device (one copy per device)
  std::vector<const uint64_t*> dq(world), dc(world), dabc(world), dsrs(world);
  std::vector<void*> st(world);
  for (uint32_t r = 0; r < world; ++r) {
    pbf_ctx* c = g->ctx[r];
    PBF_HIP(hipSetDevice(c->device));
    DevBuf &bq = c->buf("pv.q"), &bc = c->buf("pv.copies"), &babc = c->buf("pv.abc"), &bs = c->buf("pv.srs");
    if ((rc = bq.ensure(5 * n * 32)) || (rc = bc.ensure(3 * n * 16)) || (rc = babc.ensure(3 * n * 32)) ||
        (rc = bs.ensure(srs_m * 64)))
      return rc;
    const hipStream_t s = c->host_stream();
    PBF_HIP(hipMemcpyAsync(bq.p, q, 5 * n * 32, hipMemcpyHostToDevice, s));
    PBF_HIP(hipMemcpyAsync(bc.p, copies, 3 * n * 16, hipMemcpyHostToDevice, s));
    PBF_HIP(hipMemcpyAsync(babc.p, abc, 3 * n * 32, hipMemcpyHostToDevice, s));
    PBF_HIP(hipMemcpyAsync(bs.p, srs, srs_m * 64, hipMemcpyHostToDevice, s));
    dq[r] = (const uint64_t*)bq.p; dc[r] = (const uint64_t*)bc.p; dabc[r] = (const uint64_t*)babc.p;
    dsrs[r] = (const uint64_t*)bs.p;
    st[r] = (void*)s;
  }
  rc = pbf_plonk_prove_bn254_multi_dev(ctxs, world, n, dq.data(), dc.data(), dabc.data(), chal, rnd, k1k2, dsrs.data(),
                                       srs_m, mode, out_pts, out_f, st.data());
  for (uint32_t r = 0; r < world; ++r) {
    (void)hipSetDevice(g->ctx[r]->device);
    (void)hipStreamSynchronize((hipStream_t)st[r]);
  }
  return rc;
}

int pbf_multi_backend(pbf_ctx* const* ctxs, uint32_t world, int* backend) {
  if (!backend) return fail(PBF_EINVAL, "null argument");
  Group* g;
  int rc = group_for(ctxs, world, &g);
  if (rc) return rc;
  *backend = g->use_rccl ? 1 : 0;
  return 0;
}

}  // extern "C"
