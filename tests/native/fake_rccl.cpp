// TEST INFRASTRUCTURE ONLY. A stand-in for the subset of librccl that
// plonk-by-fingers_amd/csrc/group.hip calls, so the library's RCCL branch (grouped
// ncclSend / ncclRecv all-to-alls, ncclAllGather, ncclCommInitAll, ncclCommAbort) runs on
// a one-GPU box, where RCCL itself refuses two ranks on one device ("Duplicate GPU detected",
// profiles/r02/rccl_probe_one_gpu.log). Selected by PBF_RCCL_LIB=<this .so> together with
// PBF_GROUP_FORCE_RCCL=1 (tests/test_rccl_branch_gpu.py); never linked into the product.
//
// Semantics kept from RCCL / NCCL:
//  * ncclGroupStart / ncclGroupEnd are per host thread; sends and receives posted inside a
//    group are issued together at ncclGroupEnd (outside a group each call is its own group);
//  * every operation is ordered on the stream it was posted on: a receive's copy waits (by an
//    event) for the work the sender's stream queued before the send, and the sender's stream
//    does not pass the send until the receiver's copy has read the buffer;
//  * a send and its receive must agree on the byte count (else ncclInvalidUsage);
//  * ncclCommAbort releases every rank waiting in a collective of the clique.
// Restriction: every rank of the clique takes part in every grouped call (true of group.hip:
// its all-to-alls and all-gathers span the whole group). The rendezvous is a host barrier per
// grouped call, so a rank that never arrives leaves the others waiting until ncclCommAbort (or
// a 120 s timeout, reported as ncclSystemError).
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

namespace {

enum : int {
  ncclSuccess = 0,
  ncclUnhandledCudaError = 1,
  ncclSystemError = 2,
  ncclInternalError = 3,
  ncclInvalidArgument = 4,
  ncclInvalidUsage = 5,
};

size_t dtype_bytes(int t) {
  switch (t) {
    case 0: case 1: return 1;          // int8, uint8
    case 2: case 3: case 7: return 4;  // int32, uint32, float32
    case 4: case 5: case 8: return 8;  // int64, uint64, float64
    case 6: case 9: return 2;          // float16, bfloat16
    default: return 0;
  }
}

struct Clique;
struct Comm {
  Clique* cq;
  int rank;
  int sends = 0;  // ncclSend calls on this communicator (failure injection below)
};

struct Slot {  // what rank s posted for peer d
  const void* buf = nullptr;
  size_t bytes = 0;
  bool set = false;
};

struct Clique {
  int n = 0;
  int device = 0;
  std::vector<std::unique_ptr<Comm>> comms;
  std::vector<hipEvent_t> ready, done;
  std::vector<Slot> slots;  // [src * n + dst]
  std::mutex m;
  std::condition_variable cv;
  int count = 0;
  uint64_t gen = 0;
  bool aborted = false;
  int alive = 0;
  int barrier() {
    std::unique_lock<std::mutex> l(m);
    if (aborted) return ncclSystemError;
    const uint64_t g = gen;
    if (++count == n) {
      count = 0;
      ++gen;
      cv.notify_all();
      return ncclSuccess;
    }
    if (!cv.wait_for(l, std::chrono::seconds(120), [&] { return gen != g || aborted; })) return ncclSystemError;
    return aborted ? ncclSystemError : ncclSuccess;
  }
};

struct Op {
  bool is_send;
  void* buf;
  size_t bytes;
  int peer;
  Comm* comm;
  hipStream_t stream;
};

thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;

#define HIPCHK(x)                          \
  do {                                     \
    if ((x) != hipSuccess) return ncclUnhandledCudaError; \
  } while (0)

// issue one rank's grouped operations (all on one communicator and stream)
int issue(std::vector<Op>& ops) {
  if (ops.empty()) return ncclSuccess;
  Comm* c = ops[0].comm;
  Clique* q = c->cq;
  const hipStream_t s = ops[0].stream;
  for (const Op& o : ops)
    if (o.comm->cq != q || o.stream != s) return ncclInvalidUsage;  // one clique and stream per group here
  const int r = c->rank;
  for (int d = 0; d < q->n; ++d) q->slots[(size_t)r * q->n + d].set = false;
  for (const Op& o : ops)
    if (o.is_send) q->slots[(size_t)r * q->n + o.peer] = Slot{o.buf, o.bytes, true};
  HIPCHK(hipEventRecord(q->ready[r], s));
  int e;
  if ((e = q->barrier())) return e;  // every rank's sends are published and its ready event recorded
  int bad = ncclSuccess;
  for (const Op& o : ops) {
    if (o.is_send) continue;
    const Slot& sl = q->slots[(size_t)o.peer * q->n + r];
    if (!sl.set || sl.bytes != o.bytes) { bad = ncclInvalidUsage; continue; }
    HIPCHK(hipStreamWaitEvent(s, q->ready[o.peer], 0));
    if (o.bytes) HIPCHK(hipMemcpyAsync(o.buf, sl.buf, o.bytes, hipMemcpyDeviceToDevice, s));
  }
  HIPCHK(hipEventRecord(q->done[r], s));
  if ((e = q->barrier())) return e;  // every receiver's copies are queued behind its done event
  for (const Op& o : ops)
    if (o.is_send) HIPCHK(hipStreamWaitEvent(s, q->done[o.peer], 0));  // the send completes when read
  return bad;
}

int post(const Op& o) {
  if (!o.comm || o.peer < 0 || o.peer >= o.comm->cq->n) return ncclInvalidArgument;
  t_ops.push_back(o);
  if (t_depth > 0) return ncclSuccess;
  std::vector<Op> ops;
  ops.swap(t_ops);
  return issue(ops);
}

}  // namespace

extern "C" {

const char* ncclGetErrorString(int r) {
  switch (r) {
    case ncclSuccess: return "no error (stand-in)";
    case ncclUnhandledCudaError: return "HIP call failed (stand-in)";
    case ncclSystemError: return "aborted or timed out (stand-in)";
    case ncclInvalidArgument: return "invalid argument (stand-in)";
    case ncclInvalidUsage: return "invalid usage: unmatched send / receive (stand-in)";
    default: return "internal error (stand-in)";
  }
}

int ncclCommInitAll(void** comms, int ndev, const int* devlist) {
  if (!comms || ndev <= 0 || !devlist) return ncclInvalidArgument;
  for (int i = 1; i < ndev; ++i)
    if (devlist[i] != devlist[0]) return ncclInvalidUsage;  // the stand-in serves one shared device
  Clique* q = new Clique();
  q->n = ndev;
  q->device = devlist[0];
  q->alive = ndev;
  q->ready.assign(ndev, nullptr);
  q->done.assign(ndev, nullptr);
  q->slots.assign((size_t)ndev * ndev, Slot{});
  if (hipSetDevice(q->device) != hipSuccess) return ncclUnhandledCudaError;
  for (int i = 0; i < ndev; ++i) {
    if (hipEventCreateWithFlags(&q->ready[i], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&q->done[i], hipEventDisableTiming) != hipSuccess)
      return ncclUnhandledCudaError;
    q->comms.emplace_back(new Comm{q, i});
    comms[i] = q->comms.back().get();
  }
  return ncclSuccess;
}

static int release(void* comm, bool abort) {
  if (!comm) return ncclInvalidArgument;
  Clique* q = ((Comm*)comm)->cq;
  bool last;
  {
    std::lock_guard<std::mutex> l(q->m);
    if (abort) {
      q->aborted = true;
      q->cv.notify_all();
    }
    last = --q->alive == 0 && !q->aborted;  // after an abort, waiters may still be waking: keep q
  }
  if (last) {
    (void)hipSetDevice(q->device);
    for (hipEvent_t e : q->ready) (void)hipEventDestroy(e);
    for (hipEvent_t e : q->done) (void)hipEventDestroy(e);
    delete q;
  }
  return ncclSuccess;
}

int ncclCommDestroy(void* comm) { return release(comm, false); }
int ncclCommAbort(void* comm) { return release(comm, true); }

int ncclGroupStart() {
  ++t_depth;
  return ncclSuccess;
}

int ncclGroupEnd() {
  if (t_depth <= 0) return ncclInvalidUsage;
  if (--t_depth > 0) return ncclSuccess;
  std::vector<Op> ops;
  ops.swap(t_ops);
  return issue(ops);
}

// Failure injection (tests only): FAKE_RCCL_FAIL_SEND="r,k" makes the k-th ncclSend call on
// rank r's communicator fail (ncclSystemError, nothing posted) -- a rank failing inside its half
// of a collective after every rank has passed the library's pre-post barrier.
int ncclSend(const void* buf, size_t count, int dtype, int peer, void* comm, hipStream_t stream) {
  const size_t b = dtype_bytes(dtype);
  if (!b || !comm) return ncclInvalidArgument;
  Comm* c = (Comm*)comm;
  if (const char* f = getenv("FAKE_RCCL_FAIL_SEND")) {  // counted from when the variable is set
    int fr = -1, fk = -1;
    if (sscanf(f, "%d,%d", &fr, &fk) == 2 && c->rank == fr && ++c->sends == fk) return ncclSystemError;
  } else {
    c->sends = 0;
  }
  return post(Op{true, const_cast<void*>(buf), count * b, peer, (Comm*)comm, stream});
}

int ncclRecv(void* buf, size_t count, int dtype, int peer, void* comm, hipStream_t stream) {
  const size_t b = dtype_bytes(dtype);
  if (!b) return ncclInvalidArgument;
  return post(Op{false, buf, count * b, peer, (Comm*)comm, stream});
}

// every rank's sendbuf lands at recvbuf + rank * bytes on every rank
int ncclAllGather(const void* sendbuf, void* recvbuf, size_t count, int dtype, void* comm, hipStream_t stream) {
  const size_t b = dtype_bytes(dtype) * count;
  if (!dtype_bytes(dtype) || !comm) return ncclInvalidArgument;
  if (t_depth > 0) return ncclInvalidUsage;  // not used inside groups by group.hip
  Comm* c = (Comm*)comm;
  std::vector<Op> ops;
  for (int g = 0; g < c->cq->n; ++g) {
    ops.push_back(Op{true, const_cast<void*>(sendbuf), b, g, c, stream});
    ops.push_back(Op{false, (char*)recvbuf + (size_t)g * b, b, g, c, stream});
  }
  return issue(ops);
}

}  // extern "C"
