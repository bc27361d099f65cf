// tgsim_comm.cpp — the engine's own RCCL exchange (include/tgsim.h tgsim_comm_*).
//
// Shaping is egress-only and per source (pkg/sidecar/link.go:22-40), so every rank's engine owns a
// contiguous range of sources and computes their verdicts and delivery times; the only exchange is
// the hand-off of scheduled 24-B records to the destination's engine.  In the reference, packets
// between instances on different k8s nodes cross the weave CNI (pkg/sidecar/k8s_network.go:266-314);
// here they cross xGMI through RCCL, driven from inside the library so that a host (the Go runner
// through cgo) calls nothing but tgsim_*:
//
//   simulate stream   k_sim (or k_sim_fused) of window k, dispatch order of k+1
//   routing stream    records of window k grouped by destination rank (tgsim_step_sim_launch*)
//   exchange stream   (high priority) count all-to-all, grouped ncclSend/ncclRecv of the records
//                     to and from every other rank; the own rank's records are copied on the device;
//                     records an event
//   delivery stream   waits for that event: per-destination sort of the inbound records
//
// At one rank the engine owns every destination: nothing is routed or moved, and tgsim_comm_step /
// tgsim_comm_run are the single-shard tgsim_step / tgsim_step_n (local delivery, fused groups).
// TGSIM_COMM_ROUTE1=1 keeps the routed path at one rank (routing, then the delivery reads the routed
// records in place), to time the N > 1 step's own kernels on one GPU.
//
// Buffers: out[k % 3] holds window k's routed records (two launched windows + one being exchanged),
// in[k % 2] the inbound ones; ev_out[j] is the last reader of out[j] (the exchange), ev_in[i] the
// delivery that last read in[i].  Every wait is an event on a stream; the host blocks only where RCCL
// needs sizes it cannot know (the count exchange of tgsim_comm_step).
#include <dlfcn.h>
#include <sched.h>
#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include <rccl/rccl.h>  // types only: the functions are resolved from librccl.so.1 at run time

#include "tgsim_launch.h"

using namespace tgsim;

namespace {

constexpr size_t kRec = sizeof(tgsim_delivery);
// Grid of the sharded fused groups at N > 1: the exchange's kernels (RCCL) and the group delivery need
// CU slots while the next group simulates, so the persistent grid holds 90 % of the resident
// workgroups (the rest stay free for them).  Timed at one rank (TGSIM_COMM_ROUTE1, grid fractions A/B'd,
// profiles/r04/grids): turnover (one workgroup per ticket) 31.2-31.3 G pkt/s, 80 % 31.8-32.1, 90 %
// 34.0-34.4, the whole grid 34.0-34.2.
constexpr uint32_t kRoutedGridPct = 90;

// librccl.so.1, loaded once per process (when torch has loaded it already, dlopen returns that
// same instance, so one process never holds two RCCL runtimes).  The test build of this file
// (-DTGSIM_COMM_TEST_TRANSPORT, tests/mockrccl: a separate library the product never contains)
// binds the linked-in ranks-as-threads transport instead, since RCCL refuses two ranks on one GPU.
struct Rccl {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;  // optional: frees a communicator whose peer never came
  const char* (*GetErrorString)(ncclResult_t);
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  ncclResult_t (*AllToAll)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*GroupStart)();
  ncclResult_t (*GroupEnd)();
  bool ok = false;
  std::string why;
};

#ifdef TGSIM_COMM_TEST_TRANSPORT
#define MOCK_DECL(ret, name, ...) extern "C" ret mockrccl_##name(__VA_ARGS__);
MOCK_DECL(ncclResult_t, GetUniqueId, ncclUniqueId*)
MOCK_DECL(ncclResult_t, CommInitRank, ncclComm_t*, int, ncclUniqueId, int)
MOCK_DECL(ncclResult_t, CommDestroy, ncclComm_t)
MOCK_DECL(ncclResult_t, CommAbort, ncclComm_t)
MOCK_DECL(const char*, GetErrorString, ncclResult_t)
MOCK_DECL(ncclResult_t, AllReduce, const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t)
MOCK_DECL(ncclResult_t, AllGather, const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t)
MOCK_DECL(ncclResult_t, AllToAll, const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t)
MOCK_DECL(ncclResult_t, Send, const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t)
MOCK_DECL(ncclResult_t, Recv, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t)
MOCK_DECL(ncclResult_t, GroupStart, void)
MOCK_DECL(ncclResult_t, GroupEnd, void)
#undef MOCK_DECL

Rccl load_rccl() {
  Rccl r;
  r.GetUniqueId = mockrccl_GetUniqueId;
  r.CommInitRank = mockrccl_CommInitRank;
  r.CommDestroy = mockrccl_CommDestroy;
  r.CommAbort = mockrccl_CommAbort;
  r.GetErrorString = mockrccl_GetErrorString;
  r.AllReduce = mockrccl_AllReduce;
  r.AllGather = mockrccl_AllGather;
  r.AllToAll = mockrccl_AllToAll;
  r.Send = mockrccl_Send;
  r.Recv = mockrccl_Recv;
  r.GroupStart = mockrccl_GroupStart;
  r.GroupEnd = mockrccl_GroupEnd;
  r.ok = true;
  return r;
}
#else
Rccl load_rccl() {
  Rccl r;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    r.why = std::string("librccl.so.1 not loadable: ") + dlerror();
    return r;
  }
  bool all = true;
  auto get = [&](auto& fp, const char* name) {
    fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
    if (!fp) {
      all = false;
      r.why = std::string("librccl.so.1 lacks ") + name;
    }
  };
  get(r.GetUniqueId, "ncclGetUniqueId");
  get(r.CommInitRank, "ncclCommInitRank");
  get(r.CommDestroy, "ncclCommDestroy");
  get(r.GetErrorString, "ncclGetErrorString");
  get(r.AllReduce, "ncclAllReduce");
  get(r.AllGather, "ncclAllGather");
  get(r.AllToAll, "ncclAllToAll");
  get(r.Send, "ncclSend");
  get(r.Recv, "ncclRecv");
  get(r.GroupStart, "ncclGroupStart");
  get(r.GroupEnd, "ncclGroupEnd");
  r.ok = all;
  r.CommAbort = reinterpret_cast<ncclResult_t (*)(ncclComm_t)>(dlsym(h, "ncclCommAbort"));
  return r;
}
#endif

const Rccl* rccl(std::string* err) {
  static const Rccl r = load_rccl();  // thread-safe one-time initialisation
  if (!r.ok && err) *err = r.why;
  return r.ok ? &r : nullptr;
}

struct DevMem {
  uint8_t* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct Comm {
  void* eng = nullptr;
  const Rccl* R = nullptr;
  ncclComm_t nc = nullptr;
  int rank = 0, nranks = 1, dev = 0;
  uint32_t bounds[9] = {};
  hipStream_t xs = nullptr;  // exchange stream, high priority (its own hardware queue)
  DevMem out[3], in[2];
  hipEvent_t ev_out[3] = {}, ev_in[2] = {}, ev_routed[3] = {}, ev_sig = nullptr;
  bool out_busy[3] = {}, in_busy[2] = {};
  uint64_t k = 0;  // launched windows (groups) so far
  DevMem d_cnt;    // count exchange and reductions: 2 x 8 u64
  uint64_t* dm_cnt = nullptr;  // h_cnt's device address (the publish kernels store through it)
  uint64_t* h_cnt = nullptr;  // pinned, coherent and mapped (the device publishes into it from a running
                              // kernel): [0..8) sent, [8..8 + nranks) received + their sequence word,
                              // [17] reduction result, [18] its sequence word
  uint64_t cnt_seq = 0;       // sequence of the received counts published into h_cnt[8 + nranks]
  uint64_t red_seq = 0;       // sequence of the reduction results published into h_cnt[18]
  hipEvent_t ev_red = nullptr;  // after the last reduction's publish
  // TGSIM_COMM_TIMEOUT_MS: how long the host waits for a collective whose peers may have stopped
  // (a rank that died before the count all-to-all leaves the others' RCCL kernels waiting forever)
  uint64_t timeout_ms = 300000;
  bool timed_out = false;  // a collective never completed: the communicator is aborted, not drained
  hipEvent_t ev_cnt = nullptr;  // after the last count all-to-all's publish (tells a fault from a slow step)
  uint64_t route1_cap[3] = {};  // TGSIM_COMM_ROUTE1: the capacity-sized chunk of out[j]
  uint64_t exchanged = 0, max_count = 0, slot_cap = 0;
  bool launched = false;  // tgsim_comm_launch without its tgsim_comm_finish yet
  bool local = false;     // one rank, not TGSIM_COMM_ROUTE1: the single-shard step
};

int fail(Comm* C, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int fail(Comm* C, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return engine_fail(C->eng, code, buf);
}

#define CHIP(expr)                                                                        \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) return fail(C, -EIO, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)
#define CNCCL(expr)                                                                                    \
  do {                                                                                                 \
    ncclResult_t _r = (expr);                                                                          \
    if (_r != ncclSuccess) return fail(C, -EIO, "%s: %s", #expr, C->R->GetErrorString(_r));          \
  } while (0)
#define CRC(expr)          \
  do {                     \
    int _rc = (expr);      \
    if (_rc) return _rc;   \
  } while (0)

void comm_free(void* p) {
  Comm* C = static_cast<Comm*>(p);
  if (!C) return;
  (void)hipSetDevice(C->dev);
  if (C->timed_out && C->nc && C->R->CommAbort) {
    // a collective on xs waits for a peer that will never come: abort the communicator (its kernels
    // leave), and only then drain the stream
    (void)C->R->CommAbort(C->nc);
    C->nc = nullptr;
  }
  if (C->timed_out && C->nc) {
    // no ncclCommAbort in this RCCL: the stream would never drain and a destroy would wait for it, so
    // the communicator, its stream and the buffers its kernels may still touch are left behind
    fprintf(stderr, "tgsim: communicator of rank %d leaked after a timed-out exchange (no ncclCommAbort)\n", C->rank);
    delete C;
    return;
  }
  if (C->xs) (void)hipStreamSynchronize(C->xs);
  if (C->nc) (void)C->R->CommDestroy(C->nc);
  for (auto& b : C->out) b.release();
  for (auto& b : C->in) b.release();
  C->d_cnt.release();
  for (hipEvent_t e : C->ev_out)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : C->ev_in)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : C->ev_routed)
    if (e) (void)hipEventDestroy(e);
  if (C->ev_sig) (void)hipEventDestroy(C->ev_sig);
  if (C->ev_cnt) (void)hipEventDestroy(C->ev_cnt);
  if (C->ev_red) (void)hipEventDestroy(C->ev_red);
  if (C->h_cnt) (void)hipHostFree(C->h_cnt);
  if (C->xs) (void)hipStreamDestroy(C->xs);
  delete C;
}

Comm* comm_of(void* e) {
  CommSlot* s = engine_comm_slot(e);
  return s ? static_cast<Comm*>(s->state) : nullptr;
}

// A buffer about to be rewritten: wait (host) for its last reader when it has to grow, since the
// old block is freed; otherwise the writer's stream waits for that reader on the device.
int grow(Comm* C, DevMem& b, hipEvent_t last_reader, bool busy, size_t bytes) {
  if (bytes <= b.cap) return 0;
  if (busy) CHIP(hipEventSynchronize(last_reader));
  CHIP(b.ensure(bytes));
  return 0;
}

// Moves out's per-rank segments (send[r] records at soff[r]) to the ranks and the ranks' segments
// for this one into in (recv[r] records at roff[r]), on the exchange stream.  The own segment is
// a device copy: it never crosses the fabric.
int exchange(Comm* C, const uint8_t* out, uint8_t* in, const uint64_t* send, const uint64_t* soff,
             const uint64_t* recv, const uint64_t* roff) {
  if (C->nranks > 1) {
    CNCCL(C->R->GroupStart());
    for (int r = 0; r < C->nranks; ++r) {
      if (r == C->rank) continue;
      if (send[r]) CNCCL(C->R->Send(out + soff[r] * kRec, send[r] * kRec, ncclUint8, r, C->nc, C->xs));
      if (recv[r]) CNCCL(C->R->Recv(in + roff[r] * kRec, recv[r] * kRec, ncclUint8, r, C->nc, C->xs));
    }
    CNCCL(C->R->GroupEnd());
  }
  const uint64_t n_self = send[C->rank];
  if (n_self)
    CHIP(hipMemcpyAsync(in + roff[C->rank] * kRec, out + soff[C->rank] * kRec, n_self * kRec,
                        hipMemcpyDeviceToDevice, C->xs));
  return 0;
}

// Spins until the device publishes `want` into the pinned word (system-scope release), bounded by
// TGSIM_COMM_TIMEOUT_MS: a peer rank that stopped before the collective leaves it waiting forever, so
// the rank fails with -ETIMEDOUT (rank and window in tgsim_last_error) instead of hanging; the event
// recorded after the publish tells a fault from a slow exchange.
int wait_word(Comm* C, const uint64_t* w, uint64_t want, hipEvent_t ev, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t it = 1;; ++it) {
    if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == want) return 0;
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
    if ((it & 255) == 0) {
      const hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) {
        if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == want) return 0;
        return fail(C, -EIO, "comm: the %s finished without publishing", what);
      }
      if (q != hipErrorNotReady) return fail(C, -EIO, "comm: %s: %s", what, hipGetErrorString(q));
      const uint64_t ms = static_cast<uint64_t>(
          std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count());
      if (ms >= C->timeout_ms) {
        C->timed_out = true;
        return fail(C, -ETIMEDOUT, "comm: rank %d of %d waited %llu ms for the %s of window %llu (a peer rank "
                    "stopped?); the communicator is aborted at tgsim_destroy", C->rank, C->nranks,
                    static_cast<unsigned long long>(ms), what, static_cast<unsigned long long>(C->k));
      }
      if (it > (1u << 16)) sched_yield();  // (a yield on a loaded host costs a scheduler slice per wait)
    }
  }
}

// The count all-to-all's publish of the received counts (h_cnt[8..8+nranks), sequence word
// h_cnt[8 + nranks]).
int wait_counts(Comm* C) { return wait_word(C, C->h_cnt + 8 + C->nranks, C->cnt_seq, C->ev_cnt, "count all-to-all"); }

// Sum (or max) of one u64 over the ranks, on the exchange stream; the result is published to pinned
// memory behind it and the host spins on its sequence word (bounded, as above).
int allreduce_u64(Comm* C, const void* dev_src, uint64_t* result, ncclRedOp_t op) {
  const uint64_t* red = reinterpret_cast<const uint64_t*>(C->d_cnt.p + 24 * sizeof(uint64_t));
  CNCCL(C->R->AllReduce(dev_src, const_cast<uint64_t*>(red), 1, ncclUint64, op, C->nc, C->xs));
  launch_publish_words(red, 1, C->dm_cnt + 17, ++C->red_seq, C->xs);
  CHIP(hipGetLastError());
  CHIP(hipEventRecord(C->ev_red, C->xs));
  CRC(wait_word(C, C->h_cnt + 18, C->red_seq, C->ev_red, "all-reduce"));
  *result = __atomic_load_n(C->h_cnt + 17, __ATOMIC_ACQUIRE);
  return 0;
}

}  // namespace

extern "C" {
int tgsim_step(void*, uint32_t);
int tgsim_step_n(void*, uint32_t, uint32_t);
int tgsim_step_sim_launch(void*, uint32_t, uint32_t, const uint32_t*, void*, size_t);
int tgsim_step_sim_counts(void*, uint64_t*);
int tgsim_step_sim_launch_slotted_n(void*, uint32_t, uint32_t, uint32_t, const uint32_t*, void*, uint64_t, void*);
int tgsim_step_sim_launch_slotted(void*, uint32_t, uint32_t, const uint32_t*, void*, uint64_t, void*);
int tgsim_deliver_slotted_async(void*, const void*, uint32_t, uint64_t, void*);
int tgsim_step_sim_release(void*);
int tgsim_deliver_async(void*, const void*, size_t, void*);
int tgsim_deliver_slotted_n_async(void*, const void*, uint32_t, uint32_t, uint64_t, void*);
int tgsim_delivery_event(void*, void*);
int tgsim_wait_event(void*, void*);
int64_t tgsim_sim_capacity(void*);
int tgsim_sync_counters(void*, void**, uint32_t*, void*);

int tgsim_comm_id(void* out_id) {
  if (!out_id) return -EINVAL;
  std::string why;
  const Rccl* R = rccl(&why);
  if (!R) return -ENOSYS;
  ncclUniqueId id;
  if (R->GetUniqueId(&id) != ncclSuccess) return -EIO;
  memcpy(out_id, &id, TGSIM_COMM_ID_BYTES);
  return 0;
}

}  // extern "C"

namespace {

// Builds the communicator; the engine owns it only once every step succeeded (a failed init leaves
// nothing attached, so a retry is possible and no later call sees a half-built one).
int comm_build(Comm* C, const void* id) {
  void* e = C->eng;
  const int nranks = C->nranks;
  CHIP(hipSetDevice(C->dev));
  int lo = 0, hi = 0;
  CHIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  CHIP(hipStreamCreateWithPriority(&C->xs, hipStreamNonBlocking, hi));
  for (auto& ev : C->ev_out) CHIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (auto& ev : C->ev_in) CHIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (auto& ev : C->ev_routed) CHIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CHIP(hipEventCreateWithFlags(&C->ev_sig, hipEventDisableTiming));
  CHIP(hipEventCreateWithFlags(&C->ev_cnt, hipEventDisableTiming));
  CHIP(hipEventCreateWithFlags(&C->ev_red, hipEventDisableTiming));
  // coherent and mapped, as every other word the device publishes to the host: a system-scope release
  // on coarse-grained memory would not order the count stores before their sequence word
  CHIP(hipHostMalloc(reinterpret_cast<void**>(&C->h_cnt), 32 * sizeof(uint64_t),
                     hipHostMallocCoherent | hipHostMallocMapped));
  CHIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&C->dm_cnt), C->h_cnt, 0));
  if (const char* to = getenv("TGSIM_COMM_TIMEOUT_MS")) C->timeout_ms = std::max<uint64_t>(1, strtoull(to, nullptr, 10));
  CHIP(C->d_cnt.ensure(32 * sizeof(uint64_t)));
  ncclUniqueId uid;
  memcpy(&uid, id, TGSIM_COMM_ID_BYTES);
  CNCCL(C->R->CommInitRank(&C->nc, nranks, uid, C->rank));
  // gather every rank's shard and check that they tile [0, n_peers) in rank order
  uint32_t b0 = 0, b1 = 0;
  engine_shard(e, &b0, &b1);
  C->h_cnt[0] = b0;
  C->h_cnt[1] = b1;
  CHIP(hipMemcpyAsync(C->d_cnt.p, C->h_cnt, 2 * sizeof(uint64_t), hipMemcpyHostToDevice, C->xs));
  CNCCL(C->R->AllGather(C->d_cnt.p, C->d_cnt.p + 2 * sizeof(uint64_t), 2, ncclUint64, C->nc, C->xs));
  CHIP(hipMemcpyAsync(C->h_cnt + 2, C->d_cnt.p + 2 * sizeof(uint64_t), 2 * nranks * sizeof(uint64_t),
                      hipMemcpyDeviceToHost, C->xs));
  CHIP(hipStreamSynchronize(C->xs));
  for (int r = 0; r < nranks; ++r) {
    const uint64_t lo_r = C->h_cnt[2 + 2 * r], hi_r = C->h_cnt[3 + 2 * r];
    const uint64_t want = r ? C->bounds[r] : 0;
    if (lo_r != want || hi_r <= lo_r)
      return fail(C, -EINVAL, "comm_init: rank %d owns [%llu, %llu), expected a shard starting at %llu", r,
                  static_cast<unsigned long long>(lo_r), static_cast<unsigned long long>(hi_r),
                  static_cast<unsigned long long>(want));
    C->bounds[r] = static_cast<uint32_t>(lo_r);
    C->bounds[r + 1] = static_cast<uint32_t>(hi_r);
  }
  if (C->bounds[nranks] != engine_peers(e))
    return fail(C, -EINVAL, "comm_init: the shards end at %u, not at n_peers %u", C->bounds[nranks], engine_peers(e));
  memset(C->h_cnt, 0, 32 * sizeof(uint64_t));  // no stale word may read as a published sequence
  const char* r1 = getenv("TGSIM_COMM_ROUTE1");
  C->local = nranks == 1 && !(r1 && atoi(r1));
  return 0;
}

}  // namespace

extern "C" {

int tgsim_comm_init(void* e, const void* id, int rank, int nranks) {
  CommSlot* slot = engine_comm_slot(e);
  if (!slot || !id || nranks < 1 || nranks > 8 || rank < 0 || rank >= nranks) return -EINVAL;
  if (slot->state) return engine_fail(e, -EBUSY, "comm_init: the engine already has a communicator");
  std::string why;
  const Rccl* R = rccl(&why);
  if (!R) return engine_fail(e, -ENOSYS, why.c_str());
  Comm* C = new Comm();
  C->eng = e;
  C->R = R;
  C->rank = rank;
  C->nranks = nranks;
  C->dev = engine_device(e);
  const int rc = comm_build(C, id);
  if (rc) {
    comm_free(C);
    return rc;
  }
  slot->state = C;
  slot->free_fn = comm_free;
  // at one rank no RCCL kernel competes with the simulation for CU slots, so fused groups keep
  // their whole persistent grid; with more ranks it holds kRoutedGridPct of the resident workgroups,
  // the rest left free for RCCL's kernels and the group delivery
  engine_persist_routed(e, nranks == 1 ? 100u : kRoutedGridPct);
  return 0;
}

int tgsim_comm_launch(void* e, uint32_t n_ticks) {
  Comm* C = comm_of(e);
  if (!C) return e ? engine_fail(e, -EINVAL, "comm_launch: no communicator (tgsim_comm_init)") : -EINVAL;
  if (C->timed_out) return -ETIMEDOUT;  // a collective never completed (tgsim_last_error says which)
  if (n_ticks == 0) return -EINVAL;
  if (C->launched) return engine_fail(e, -EBUSY, "comm_launch: the launched window is not finished (tgsim_comm_finish)");
  CHIP(hipSetDevice(C->dev));
  if (C->local) {  // one rank owns every destination: nothing to route or move, so the window
                         // is the single-shard step with its asynchronous local delivery (the count
                         // of routed records is never read back: no host round trip)
    CRC(tgsim_step(e, n_ticks));
    C->k++;
    C->launched = true;
    return 0;
  }
  const uint32_t j = C->k % 3;
  const int64_t cap = tgsim_sim_capacity(e);
  if (cap < 0) return static_cast<int>(cap);
  if (C->nranks == 1) {  // TGSIM_COMM_ROUTE1: one chunk of the step's whole capacity, delivered in place
                         // from its count header, so the host never waits for the routing
    CRC(grow(C, C->out[j], C->ev_out[j], C->out_busy[j], (static_cast<size_t>(cap) + 1) * kRec));
    if (C->out_busy[j]) CRC(tgsim_wait_event(e, C->ev_out[j]));
    CRC(tgsim_step_sim_launch_slotted(e, n_ticks, 1, C->bounds, C->out[j].p, static_cast<uint64_t>(cap),
                                      C->ev_routed[j]));
    C->route1_cap[j] = static_cast<uint64_t>(cap);
    C->launched = true;
    return 0;
  }
  CRC(grow(C, C->out[j], C->ev_out[j], C->out_busy[j], static_cast<size_t>(cap) * kRec));
  if (C->out_busy[j]) CRC(tgsim_wait_event(e, C->ev_out[j]));  // an earlier reader of out[j]
  CRC(tgsim_step_sim_launch(e, n_ticks, C->nranks, C->bounds, C->out[j].p, static_cast<size_t>(cap)));
  CRC(engine_record_routed(e, C->ev_routed[j]));  // the exchange of out[j] waits for it on the device
  C->launched = true;
  return 0;
}

int tgsim_comm_finish(void* e) {
  Comm* C = comm_of(e);
  if (!C) return e ? engine_fail(e, -EINVAL, "comm_finish: no communicator (tgsim_comm_init)") : -EINVAL;
  if (C->timed_out) return -ETIMEDOUT;  // a collective never completed (tgsim_last_error says which)
  if (!C->launched) return engine_fail(e, -EINVAL, "comm_finish: no launched window (tgsim_comm_launch)");
  CHIP(hipSetDevice(C->dev));
  C->launched = false;
  const int nr = C->nranks;
  if (C->local) return 0;  // tgsim_comm_launch ran the whole window
  const uint32_t j = C->k % 3, i = C->k % 2;
  uint64_t send[8] = {}, recv[8] = {}, soff[9] = {}, roff[9] = {};
  if (nr == 1) {  // TGSIM_COMM_ROUTE1: nothing to exchange; retired without a wait, delivered in place
    CRC(tgsim_step_sim_release(e));
    C->k++;
    C->exchanged += C->route1_cap[j] + 1;  // record slots, as in the slotted run
    CRC(tgsim_deliver_slotted_async(e, C->out[j].p, 1, C->route1_cap[j], C->ev_routed[j]));
    CRC(tgsim_delivery_event(e, C->ev_out[j]));
    C->out_busy[j] = true;
    return 0;
  }
  // the count all-to-all runs on the device right behind the routing (its per-rank counts never
  // cross to the host first); the host waits once, for the received counts it publishes
  const uint64_t* dsend = engine_route_counts_dev(e);
  if (!dsend) return fail(C, -EIO, "comm_finish: no routed counts on the device");
  CHIP(hipStreamWaitEvent(C->xs, C->ev_routed[j], 0));
  CNCCL(C->R->AllToAll(dsend, C->d_cnt.p + 8 * sizeof(uint64_t), 1, ncclUint64, C->nc, C->xs));
  launch_publish_words(reinterpret_cast<const uint64_t*>(C->d_cnt.p + 8 * sizeof(uint64_t)), static_cast<uint32_t>(nr),
                       C->dm_cnt + 8, ++C->cnt_seq, C->xs);
  CHIP(hipGetLastError());
  CHIP(hipEventRecord(C->ev_cnt, C->xs));
  CRC(tgsim_step_sim_counts(e, send));  // the routing's own published edges (bookkeeping, overflow check)
  C->k++;
  for (int r = 0; r < nr; ++r) {
    soff[r + 1] = soff[r] + send[r];
    C->max_count = std::max(C->max_count, send[r]);
  }
  C->exchanged += soff[nr];
  CRC(wait_counts(C));
  for (int r = 0; r < nr; ++r) {
    recv[r] = C->h_cnt[8 + r];
    roff[r + 1] = roff[r] + recv[r];
  }
  CRC(grow(C, C->in[i], C->ev_in[i], C->in_busy[i], std::max<uint64_t>(roff[nr], 1) * kRec));
  if (C->in_busy[i]) CHIP(hipStreamWaitEvent(C->xs, C->ev_in[i], 0));  // the delivery of window k - 2
  CHIP(hipStreamWaitEvent(C->xs, C->ev_routed[j], 0));  // the routing that wrote out[j]
  CRC(exchange(C, C->out[j].p, C->in[i].p, send, soff, recv, roff));
  CHIP(hipEventRecord(C->ev_out[j], C->xs));
  C->out_busy[j] = true;
  CRC(tgsim_deliver_async(e, C->in[i].p, roff[nr], C->ev_out[j]));
  CRC(tgsim_delivery_event(e, C->ev_in[i]));
  C->in_busy[i] = true;
  return 0;
}

int tgsim_comm_step(void* e, uint32_t n_ticks) {
  int rc = tgsim_comm_launch(e, n_ticks);
  return rc ? rc : tgsim_comm_finish(e);
}

int tgsim_comm_run(void* e, uint32_t n_ticks, uint32_t n_steps, uint32_t fuse, uint64_t slot_cap) {
  Comm* C = comm_of(e);
  if (!C) return e ? engine_fail(e, -EINVAL, "comm_run: no communicator (tgsim_comm_init)") : -EINVAL;
  if (C->timed_out) return -ETIMEDOUT;  // a collective never completed (tgsim_last_error says which)
  if (n_ticks == 0 || fuse == 0 || fuse > kFuseMax) return -EINVAL;
  if (C->launched) return engine_fail(e, -EBUSY, "comm_run: a launched window is not finished (tgsim_comm_finish)");
  if (!n_steps) return 0;
  CHIP(hipSetDevice(C->dev));
  const int nr = C->nranks;
  if (C->local) {  // one rank: nothing to route or move; the single-shard fused groups
    CRC(tgsim_step_n(e, n_ticks, n_steps));
    C->k += n_steps;
    return 0;
  }
  if (!slot_cap) {  // from the exact windows so far, max over ranks (a collective every rank makes)
    uint64_t mx = 0;
    if (nr == 1) CRC(engine_route_max(e, &C->max_count));  // TGSIM_COMM_ROUTE1: counts never came to the host
    C->h_cnt[0] = C->max_count;
    CHIP(hipMemcpyAsync(C->d_cnt.p, C->h_cnt, sizeof(uint64_t), hipMemcpyHostToDevice, C->xs));
    CRC(allreduce_u64(C, C->d_cnt.p, &mx, ncclMax));
    slot_cap = mx + mx / 4 + 4096;
    if (!mx) {  // no exact window seen yet: the bound of what one window can emit (never overflows)
      const int64_t cap = tgsim_sim_capacity(e);
      if (cap < 0) return static_cast<int>(cap);
      C->h_cnt[0] = static_cast<uint64_t>(cap);
      CHIP(hipMemcpyAsync(C->d_cnt.p, C->h_cnt, sizeof(uint64_t), hipMemcpyHostToDevice, C->xs));
      CRC(allreduce_u64(C, C->d_cnt.p, &slot_cap, ncclMax));
    }
  }
  C->slot_cap = slot_cap;
  std::vector<uint32_t> groups;
  for (uint32_t left = n_steps; left;) {
    const uint32_t g = std::min(left, fuse);
    groups.push_back(g);
    left -= g;
  }
  struct Launched {
    uint32_t j, w;
    uint64_t kk;  // launch index (in[kk % 2] receives it)
  };
  std::vector<Launched> pend;
  auto launch = [&](uint32_t w) -> int {
    const uint32_t j = C->k % 3;
    const size_t bytes = static_cast<size_t>(nr) * w * (slot_cap + 1) * kRec;
    CRC(grow(C, C->out[j], C->ev_out[j], C->out_busy[j], bytes));
    if (C->out_busy[j]) CRC(tgsim_wait_event(e, C->ev_out[j]));
    CRC(tgsim_step_sim_launch_slotted_n(e, n_ticks, w, nr, C->bounds, C->out[j].p, slot_cap, C->ev_routed[j]));
    pend.push_back({j, w, C->k});
    C->k++;
    return 0;
  };
  for (size_t s = 0; s < std::min<size_t>(2, groups.size()); ++s) CRC(launch(groups[s]));
  for (size_t s = 0; s < groups.size(); ++s) {
    const Launched L = pend.front();
    pend.erase(pend.begin());
    CRC(tgsim_step_sim_release(e));  // retires the oldest launch without waiting (overflow -> -ENOSPC)
    if (s + 2 < groups.size()) CRC(launch(groups[s + 2]));
    const uint64_t chunk = static_cast<uint64_t>(L.w) * (slot_cap + 1);  // records per rank
    C->exchanged += nr * chunk;
    if (nr == 1) {  // TGSIM_COMM_ROUTE1: the routed chunk is this rank's own, delivered in place
      CRC(tgsim_deliver_slotted_n_async(e, C->out[L.j].p, 1, L.w, slot_cap, C->ev_routed[L.j]));
      CRC(tgsim_delivery_event(e, C->ev_out[L.j]));
      C->out_busy[L.j] = true;
      continue;
    }
    const uint32_t i = static_cast<uint32_t>(L.kk % 2);
    CRC(grow(C, C->in[i], C->ev_in[i], C->in_busy[i], static_cast<size_t>(nr) * chunk * kRec));
    CHIP(hipStreamWaitEvent(C->xs, C->ev_routed[L.j], 0));
    if (C->in_busy[i]) CHIP(hipStreamWaitEvent(C->xs, C->ev_in[i], 0));
    uint64_t cnt[8], off[9];
    for (int r = 0; r <= nr; ++r) off[r] = r * chunk;
    for (int r = 0; r < nr; ++r) cnt[r] = chunk;
    CRC(exchange(C, C->out[L.j].p, C->in[i].p, cnt, off, cnt, off));
    CHIP(hipEventRecord(C->ev_out[L.j], C->xs));
    C->out_busy[L.j] = true;
    CRC(tgsim_deliver_slotted_n_async(e, C->in[i].p, nr, L.w, slot_cap, C->ev_out[L.j]));
    CRC(tgsim_delivery_event(e, C->ev_in[i]));
    C->in_busy[i] = true;
  }
  return 0;
}

int tgsim_comm_barrier(void* e, uint32_t state, uint64_t target) {
  Comm* C = comm_of(e);
  if (!C) return e ? engine_fail(e, -EINVAL, "comm_barrier: no communicator (tgsim_comm_init)") : -EINVAL;
  if (C->timed_out) return -ETIMEDOUT;  // a collective never completed (tgsim_last_error says which)
  if (state >= TGSIM_SYNC_STATES) return -EINVAL;
  CHIP(hipSetDevice(C->dev));
  void* table = nullptr;
  uint32_t n = 0;
  CRC(tgsim_sync_counters(e, &table, &n, C->ev_sig));  // ev_sig: after every signal issued so far
  CHIP(hipStreamWaitEvent(C->xs, C->ev_sig, 0));
  uint64_t sum = 0;
  CRC(allreduce_u64(C, static_cast<const uint64_t*>(table) + state, &sum, ncclSum));
  return sum >= target ? 1 : 0;
}

int tgsim_comm_info(void* e, tgsim_comm_info_t* out) {
  Comm* C = comm_of(e);
  if (!out) return -EINVAL;
  if (!C) return e ? engine_fail(e, -EINVAL, "comm_info: no communicator (tgsim_comm_init)") : -EINVAL;
  memset(out, 0, sizeof *out);
  out->rank = C->rank;
  out->nranks = C->nranks;
  out->exchanged_records = C->exchanged;
  out->max_rank_count = C->max_count;
  out->slot_cap = C->slot_cap;
  for (int r = 0; r <= C->nranks; ++r) out->bounds[r] = C->bounds[r];
  return 0;
}

}  // extern "C"
