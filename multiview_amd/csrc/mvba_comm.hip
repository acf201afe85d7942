// mvba_comm.hip — communicators for landmark-sharded solves.
//
// mvba_solve exchanges the camera-side partial sums of its shards (one
// all-reduce per linearization, one per CG iteration, a few scalars per LM
// step; mvba_solve.cpp Solver::exchange). The exchange is STREAM-ORDERED: it is
// enqueued on the solver's stream and the host never waits for it, so the
// device-resident CG (batched iterations, device-side step control) runs
// unchanged in sharded mode. Two transports behind one mvba_allreduce_fn:
//
//   * RCCL (one process per GPU, torchrun): ncclAllReduce on the solver's
//     stream over xGMI. The unique id is created by rank 0
//     (mvba_comm_unique_id) and broadcast by the caller (torch.distributed).
//     Ring all-reduce hands every rank the same bits, so the replicated
//     camera-side CG state stays identical and every rank takes the same
//     number of iterations (the collectives stay matched).
//   * local (several shards in ONE process, one host thread and one stream
//     per shard, on one or several devices: the rig_calibrator CLI's
//     --num_gpus, and two shards on one GPU where RCCL refuses duplicate
//     devices): every shard copies its buffer into its slot (double-buffered
//     by call parity), records an event, meets the other host threads at a
//     barrier (enqueue-time only: no GPU wait), makes its stream wait for
//     every shard's event and sums the slots in rank order into its buffer —
//     the same bits on every shard. A shard reuses a slot parity only after
//     every shard's sum of the previous use has completed (done events).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <thread>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

// mvba_solve.cpp: drops the captured graphs that hold a communicator's collectives
extern "C" void mvba_drop_comm_graphs(const void* comm);

#include "../../include/mvba/mvba.h"

namespace {

constexpr int kMaxLocalRanks = 64;

struct SlotArgs {
  const double* p[kMaxLocalRanks];
};

__global__ void __launch_bounds__(256) k_slot_reduce(SlotArgs a, int32_t nranks, int64_t n, int32_t op,
                                                     double* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    double v = a.p[0][e];
    for (int r = 1; r < nranks; r++) {
      const double w = a.p[r][e];
      v = op == MVBA_REDUCE_MAX ? fmax(v, w) : v + w;
    }
    out[e] = v;
  }
}

struct LocalGroup {
  int nranks = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  struct Rank {
    int device = 0;
    hipEvent_t ready[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    double* slot[2] = {nullptr, nullptr};
    int64_t cap[2] = {0, 0};
    int64_t count[2] = {0, 0};  // this rank's element count of its current use of slot p
  };
  std::vector<Rank> ranks;
  int refs = 0;

  // host rendezvous of all ranks (enqueue order only); false if aborted
  bool barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (aborted) return false;
    const uint64_t g = gen;
    if (++arrived == nranks) {
      arrived = 0;
      gen++;
      cv.notify_all();
      return true;
    }
    cv.wait(lk, [&] { return gen != g || aborted; });
    return !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(m);
    aborted = true;
    cv.notify_all();
  }
};

}  // namespace

struct mvba_comm {
  int kind = 0;  // 0 RCCL, 1 local
  int rank = 0, nranks = 1, device = 0;
  ncclComm_t nccl = nullptr;   // non-blocking RCCL communicator (config.blocking = 0)
  // Every NCCL call on nccl (enqueue, async-error poll, abort, destroy) runs
  // under nccl_m, and `aborted` is checked under it: mvba_comm_abort may come
  // from a watchdog thread while the owner enqueues or polls, and ncclCommAbort
  // frees the communicator. The lock is never held across a sleep or a stream
  // wait, so an abort is never blocked behind a long wait.
  std::mutex nccl_m;
  std::atomic<bool> aborted{false};
  double timeout_s = 0.0;      // deadline of every host-side RCCL wait
  std::shared_ptr<LocalGroup> grp;
  uint64_t calls = 0;
  std::string err;
};

namespace {

thread_local std::string g_comm_err;

mvba_status comm_fail(const std::string& msg) {
  g_comm_err = msg;
  return MVBA_E_INVALID;
}

// Default deadline of the RCCL waits (communicator init, collective enqueue):
// MVBA_COMM_TIMEOUT_S, else 300 s.
double default_timeout_s() {
  const char* v = std::getenv("MVBA_COMM_TIMEOUT_S");
  const double t = v ? std::atof(v) : 0.0;
  return t > 0.0 ? t : 300.0;
}

// A non-blocking communicator's calls may return ncclInProgress: poll its
// asynchronous state until it settles, an abort is requested, or the deadline
// passes (then the communicator is aborted, so no rank stays stuck in it).
ncclResult_t settle(mvba_comm* c, ncclResult_t r, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  while (r == ncclInProgress) {
    std::this_thread::sleep_for(std::chrono::microseconds(50));
    std::lock_guard<std::mutex> lk(c->nccl_m);
    if (c->aborted.load()) return ncclInvalidUsage;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c->timeout_s) {
      g_comm_err = std::string(what) + ": no progress within " + std::to_string(c->timeout_s) +
                   " s (MVBA_COMM_TIMEOUT_S); communicator aborted";
      c->aborted.store(true);
      (void)ncclCommAbort(c->nccl);
      return ncclSystemError;
    }
    if (ncclCommGetAsyncError(c->nccl, &r) != ncclSuccess) return ncclSystemError;
  }
  if (r != ncclSuccess && g_comm_err.empty()) g_comm_err = std::string(what) + ": " + ncclGetErrorString(r);
  return r;
}

int32_t local_allreduce(mvba_comm* c, double* buf, int64_t n, int32_t op, hipStream_t s) {
  LocalGroup& G = *c->grp;
  LocalGroup::Rank& me = G.ranks[(size_t)c->rank];
  const int p = (int)(c->calls & 1);
  c->calls++;
  if (hipSetDevice(c->device) != hipSuccess) return 1;
  // slot p is free once every shard's sum of its previous use is done
  for (int j = 0; j < G.nranks; j++)
    if (G.ranks[(size_t)j].done[p] && hipStreamWaitEvent(s, G.ranks[(size_t)j].done[p], 0) != hipSuccess) return 1;
  if (me.cap[p] < n) {
    // grows at most a few times (the first linearization exchange is the largest);
    // the old slot may still be read by earlier sums: wait for the device first
    if (me.slot[p]) {
      // the stream waits for every shard's previous sum on this slot (above)
      if (hipStreamSynchronize(s) != hipSuccess || hipFree(me.slot[p]) != hipSuccess) return 1;
      me.slot[p] = nullptr;
    }
    if (hipMalloc(reinterpret_cast<void**>(&me.slot[p]), (size_t)std::max<int64_t>(n, 1024) * sizeof(double)) !=
        hipSuccess)
      return 1;
    me.cap[p] = std::max<int64_t>(n, 1024);
  }
  if (n > 0 && hipMemcpyAsync(me.slot[p], buf, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, s) != hipSuccess)
    return 1;
  if (hipEventRecord(me.ready[p], s) != hipSuccess) return 1;
  {
    std::lock_guard<std::mutex> lk(G.m);
    me.count[p] = n;
  }
  if (!G.barrier()) return 1;
  // every rank compares every rank's count (a rank cannot overwrite count[p]
  // before all ranks passed the next barrier, on the other slot), so a
  // mismatch fails all of them before any reduce over a smaller peer slot
  {
    std::lock_guard<std::mutex> lk(G.m);
    for (int j = 0; j < G.nranks; j++)
      if (G.ranks[(size_t)j].count[p] != n) {
        comm_fail("mvba_comm_allreduce: ranks passed different element counts");
        G.aborted = true;
        G.cv.notify_all();
        return 1;
      }
  }
  SlotArgs a{};
  for (int j = 0; j < G.nranks; j++) {
    if (hipStreamWaitEvent(s, G.ranks[(size_t)j].ready[p], 0) != hipSuccess) return 1;
    a.p[j] = G.ranks[(size_t)j].slot[p];
  }
  if (n > 0) {
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_slot_reduce, dim3(blocks), dim3(256), 0, s, a, (int32_t)G.nranks, n, op, buf);
    if (hipGetLastError() != hipSuccess) return 1;
  }
  if (hipEventRecord(me.done[p], s) != hipSuccess) return 1;
  return 0;
}

}  // namespace

extern "C" {

const char* mvba_comm_error(void) { return g_comm_err.c_str(); }

mvba_status mvba_comm_unique_id(uint8_t* id) {
  if (!id) return comm_fail("null id");
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return comm_fail(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(id, u.internal, MVBA_COMM_ID_BYTES);
  return MVBA_OK;
}

mvba_status mvba_comm_init_rccl_deadline(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device,
                                         double timeout_s, mvba_comm** out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return comm_fail("invalid communicator arguments");
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return comm_fail("hipSetDevice failed");
  ncclUniqueId u;
  std::memcpy(u.internal, id, MVBA_COMM_ID_BYTES);
  auto* c = new mvba_comm();
  c->kind = 0;
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  c->timeout_s = timeout_s > 0.0 ? timeout_s : default_timeout_s();
  g_comm_err.clear();
  // non-blocking: the init returns at once and is polled against the deadline,
  // so a rank whose peers never join gets an error instead of a hang
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t r = ncclCommInitRankConfig(&c->nccl, nranks, u, rank, &cfg);
  if (r == ncclSuccess || r == ncclInProgress) {
    // c is not published yet (no other thread can abort it): no lock needed
    if (r == ncclSuccess && ncclCommGetAsyncError(c->nccl, &r) != ncclSuccess) r = ncclSystemError;
    r = settle(c, r, "ncclCommInitRankConfig");
  } else {
    g_comm_err = std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r);
  }
  if (r != ncclSuccess) {
    if (c->nccl && !c->aborted.load()) (void)ncclCommAbort(c->nccl);
    delete c;
    return MVBA_E_INVALID;
  }
  *out = c;
  return MVBA_OK;
}

mvba_status mvba_comm_init_rccl(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device, mvba_comm** out) {
  return mvba_comm_init_rccl_deadline(id, nranks, rank, device, 0.0, out);
}

mvba_status mvba_comm_init_local(int32_t nranks, const int32_t* devices, mvba_comm** out) {
  if (!devices || !out || nranks < 1 || nranks > kMaxLocalRanks) return comm_fail("invalid communicator arguments");
  auto G = std::make_shared<LocalGroup>();
  G->nranks = nranks;
  G->ranks.resize((size_t)nranks);
  for (int r = 0; r < nranks; r++) out[r] = nullptr;
  for (int r = 0; r < nranks; r++) {
    LocalGroup::Rank& R = G->ranks[(size_t)r];
    R.device = devices[r];
    if (hipSetDevice(R.device) != hipSuccess) return comm_fail("hipSetDevice failed");
    for (int p = 0; p < 2; p++)
      if (hipEventCreateWithFlags(&R.ready[p], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&R.done[p], hipEventDisableTiming) != hipSuccess)
        return comm_fail("hipEventCreate failed");
    // shards on different devices read each other's slots over xGMI
    for (int j = 0; j < nranks; j++)
      if (devices[j] != R.device) {
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, R.device, devices[j]) != hipSuccess || !can)
          return comm_fail("no peer access between the devices of a local communicator");
        const hipError_t e = hipDeviceEnablePeerAccess(devices[j], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return comm_fail("hipDeviceEnablePeerAccess failed");
        (void)hipGetLastError();
      }
  }
  G->refs = nranks;
  for (int r = 0; r < nranks; r++) {
    auto* c = new mvba_comm();
    c->kind = 1;
    c->rank = r;
    c->nranks = nranks;
    c->device = devices[r];
    c->grp = G;
    out[r] = c;
  }
  return MVBA_OK;
}

mvba_status mvba_comm_abort(mvba_comm* c) {
  if (!c) return MVBA_E_INVALID;
  if (c->kind == 0) {
    // callable from another thread while the owner waits on a collective
    // (a watchdog): RCCL's abort makes the pending kernels return. Under
    // nccl_m: the owner is then never inside an NCCL call on the handle this
    // frees, and its next call sees `aborted` before touching it.
    std::lock_guard<std::mutex> lk(c->nccl_m);
    if (c->nccl && !c->aborted.exchange(true)) (void)ncclCommAbort(c->nccl);
  } else {
    c->grp->abort();
  }
  return MVBA_OK;
}

void mvba_comm_destroy(mvba_comm* c) {
  if (!c) return;
  mvba_drop_comm_graphs(c);  // graphs holding this communicator's collectives go first
  if (c->kind == 0) {
    std::lock_guard<std::mutex> lk(c->nccl_m);
    if (c->nccl && !c->aborted.exchange(true)) (void)ncclCommDestroy(c->nccl);
  } else {
    std::shared_ptr<LocalGroup> G = c->grp;
    c->grp.reset();
    bool last = false;
    {
      std::lock_guard<std::mutex> lk(G->m);
      last = --G->refs == 0;
    }
    if (last) {
      (void)hipDeviceSynchronize();
      for (auto& R : G->ranks) {
        (void)hipSetDevice(R.device);
        for (int p = 0; p < 2; p++) {
          if (R.ready[p]) (void)hipEventDestroy(R.ready[p]);
          if (R.done[p]) (void)hipEventDestroy(R.done[p]);
          if (R.slot[p]) (void)hipFree(R.slot[p]);
        }
      }
    }
  }
  delete c;
}

int32_t mvba_comm_rank(const mvba_comm* c) { return c ? c->rank : -1; }
int32_t mvba_comm_capturable(const mvba_comm* c) { return c && c->kind == 0 && c->nccl ? 1 : 0; }
int32_t mvba_comm_size(const mvba_comm* c) { return c ? c->nranks : 0; }

int32_t mvba_comm_allreduce(double* device_buf, int64_t count, int32_t op, void* hip_stream, void* comm) {
  auto* c = static_cast<mvba_comm*>(comm);
  if (!c || count < 0 || (op != MVBA_REDUCE_SUM && op != MVBA_REDUCE_MAX)) return 1;
  const hipStream_t s = static_cast<hipStream_t>(hip_stream);
  if (c->kind == 1) return local_allreduce(c, device_buf, count, op, s);
  if (!c->nccl) return 1;
  c->calls++;
  if (count == 0) return c->aborted.load() ? 1 : 0;
  ncclResult_t r;
  {
    std::lock_guard<std::mutex> lk(c->nccl_m);
    if (c->aborted.load()) return 1;
    r = ncclAllReduce(device_buf, device_buf, (size_t)count, ncclDouble, op == MVBA_REDUCE_MAX ? ncclMax : ncclSum,
                      c->nccl, s);
    if (r == ncclSuccess && ncclCommGetAsyncError(c->nccl, &r) != ncclSuccess) r = ncclSystemError;
  }
  if (r == ncclInProgress) r = settle(c, r, "ncclAllReduce");
  return r == ncclSuccess ? 0 : 1;
}

}  // extern "C"
