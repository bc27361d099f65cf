// Test double for librccl.so.1 (TEST INFRASTRUCTURE, never the product): the ncclXxx entry points
// tgsim_comm.cpp uses, for a world whose ranks are THREADS of one process driving
// engines on ONE GPU.  RCCL itself refuses two ranks on one device ("Duplicate GPU detected"), and
// the GPU pool hands out one-GPU boxes, so without this the engine's N > 1 exchange (routing, count
// all-to-all, grouped send/recv, slotted chunks, barrier all-reduce) would first run in the driver's
// 8-GPU scaling job.  Its entry points are the nccl ones prefixed mockrccl_ (no symbol of the real
// library is shadowed); tgsim_comm.cpp compiled with -DTGSIM_COMM_TEST_TRANSPORT binds them, and the
// two link into tests/mockrccl/libtgsim_mockcomm.so, the engine build tests/test_gpu_multirank.py
// loads.  The product libtgsim.so contains neither.
//
// Semantics kept from NCCL: operations between two ranks match in issue order; a group's sends and
// receives complete together; everything is stream-ordered (a receive copies on the receiver's
// stream after an event recorded on the sender's; the sender's stream waits for that copy, so its
// buffer may be reused after the call exactly as with RCCL).  Host waits are bounded (60 s): a rank
// whose partner never posts gets ncclSystemError instead of a hang.
//
// A partner that stopped (MOCKRCCL_ABANDON_MS, tests only): RCCL's collectives are asynchronous, so
// a rank whose peer never joins returns from the call and its stream stops where RCCL's kernel would
// wait.  With MOCKRCCL_ABANDON_MS set, a wait for a partner that exceeds it does the same: the call
// returns success without the data and leaves a gate kernel on the caller's stream, which spins until
// the communicator is aborted or destroyed (ncclCommAbort / ncclCommDestroy of any rank), bounded at
// 120 s.  The engine's own bounded host waits (TGSIM_COMM_TIMEOUT_MS) are then what ends the rank.
// Only an abandoned collective spins on the device: a spinning kernel can hold up other streams
// that share its hardware queue, so the tests that use it keep every other rank idle meanwhile.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace {

constexpr auto kWait = std::chrono::seconds(60);

struct Msg {
  const void* buf = nullptr;
  size_t bytes = 0;
  hipEvent_t sent = nullptr, done = nullptr;
  bool copied = false;
};

struct World {
  int n = 0, joined = 0, destroyed = 0;
  bool aborted = false;
  std::vector<uint32_t*> gates;  // pinned words of abandoned collectives' gate kernels (1: open)
  std::mutex m;
  std::condition_variable cv;
  std::map<std::pair<int, int>, std::deque<std::shared_ptr<Msg>>> box;  // (src, dst) -> messages
  std::vector<hipEvent_t> events;  // destroyed with the world
  // host all-gather (reductions and the init-time gather)
  int ag_arrived = 0;
  uint64_t ag_gen = 0;
  std::vector<std::vector<uint8_t>> ag_in, ag_out;
};

std::mutex g_m;
std::map<uint64_t, World*> g_worlds;
uint64_t g_next = 1;

struct Op {
  bool send;
  void* buf;
  size_t bytes;
  int peer;
  ncclComm* comm;
  hipStream_t s;
};
thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;
thread_local ncclResult_t t_err = ncclSuccess;

}  // namespace

struct ncclComm {
  World* w;
  int rank;
};

namespace {

size_t type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

// MOCKRCCL_ABANDON_MS (0: never): how long a collective waits for a stopped partner before it is
// abandoned to a gate kernel.
std::chrono::milliseconds abandon_after() {
  const char* v = getenv("MOCKRCCL_ABANDON_MS");
  const long ms = v ? atol(v) : 0;
  return ms > 0 ? std::chrono::milliseconds(ms) : std::chrono::milliseconds(0);
}

// Holds the caller's stream until the world is aborted or destroyed (bounded: 120 s of
// s_memrealtime at 100 MHz, so no wave outlives a test that forgot to).
__global__ void k_gate(const uint32_t* gate) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > 12000000000ull) break;
    __builtin_amdgcn_s_sleep(100);
  }
}

// The collective the caller waits for will never complete: its stream stops at a gate (as RCCL's
// kernel would); the call itself returns success.  Called with w->m held.
ncclResult_t abandon(World* w, hipStream_t s) {
  uint32_t* gate = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&gate), sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped) !=
      hipSuccess)
    return ncclUnhandledCudaError;
  *gate = w->aborted ? 1u : 0u;
  w->gates.push_back(gate);
  hipLaunchKernelGGL(k_gate, dim3(1), dim3(1), 0, s, gate);
  return hipGetLastError() == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

// A rank left (destroy or abort): no abandoned collective can complete any more.
void open_gates(World* w) {
  std::lock_guard<std::mutex> l(w->m);
  w->aborted = true;
  for (uint32_t* g : w->gates) __atomic_store_n(g, 1u, __ATOMIC_RELEASE);
}

hipEvent_t new_event(World* w) {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> l(w->m);
  w->events.push_back(e);
  return e;
}

// One group: post every send, serve every receive, then make each send's stream wait for its copy.
ncclResult_t run(std::vector<Op>& ops) {
  std::vector<std::pair<std::shared_ptr<Msg>, const Op*>> posted;
  for (const Op& o : ops) {
    if (!o.send) continue;
    World* w = o.comm->w;
    auto msg = std::make_shared<Msg>();
    msg->buf = o.buf;
    msg->bytes = o.bytes;
    if (!(msg->sent = new_event(w)) || hipEventRecord(msg->sent, o.s) != hipSuccess) return ncclUnhandledCudaError;
    {
      std::lock_guard<std::mutex> l(w->m);
      w->box[{o.comm->rank, o.peer}].push_back(msg);
    }
    w->cv.notify_all();
    posted.emplace_back(msg, &o);
  }
  for (const Op& o : ops) {
    if (o.send) continue;
    World* w = o.comm->w;
    std::shared_ptr<Msg> msg;
    {
      std::unique_lock<std::mutex> l(w->m);
      auto& q = w->box[{o.peer, o.comm->rank}];
      const auto ab = abandon_after();
      if (ab.count() && !w->cv.wait_for(l, ab, [&] { return !q.empty(); })) return abandon(w, o.s);
      if (!w->cv.wait_for(l, kWait, [&] { return !q.empty(); })) return ncclSystemError;
      msg = q.front();
      q.pop_front();
    }
    if (msg->bytes != o.bytes) return ncclInvalidUsage;
    if (hipStreamWaitEvent(o.s, msg->sent, 0) != hipSuccess) return ncclUnhandledCudaError;
    if (o.bytes && hipMemcpyAsync(o.buf, msg->buf, o.bytes, hipMemcpyDeviceToDevice, o.s) != hipSuccess)
      return ncclUnhandledCudaError;
    hipEvent_t done = new_event(w);
    if (!done || hipEventRecord(done, o.s) != hipSuccess) return ncclUnhandledCudaError;
    {
      std::lock_guard<std::mutex> l(w->m);
      msg->done = done;
      msg->copied = true;
    }
    w->cv.notify_all();
  }
  for (auto& p : posted) {
    const std::shared_ptr<Msg>& msg = p.first;
    const Op* o = p.second;
    World* w = o->comm->w;
    {
      std::unique_lock<std::mutex> l(w->m);
      if (!w->cv.wait_for(l, kWait, [&] { return msg->copied; })) return ncclSystemError;
    }
    if (hipStreamWaitEvent(o->s, msg->done, 0) != hipSuccess) return ncclUnhandledCudaError;
  }
  return ncclSuccess;
}

ncclResult_t enqueue(Op o) {
  if (!o.comm || o.peer < 0 || o.peer >= o.comm->w->n) return ncclInvalidArgument;
  if (t_depth) {
    t_ops.push_back(o);
    return ncclSuccess;
  }
  std::vector<Op> one{o};
  return run(one);
}

// Every rank's bytes, in rank order, after the caller's stream has drained (host copy).
ncclResult_t host_allgather(ncclComm* c, const void* dev, size_t bytes, hipStream_t s, std::vector<uint8_t>* all) {
  std::vector<uint8_t> mine(bytes);
  if (hipStreamSynchronize(s) != hipSuccess) return ncclUnhandledCudaError;
  if (bytes && hipMemcpy(mine.data(), dev, bytes, hipMemcpyDeviceToHost) != hipSuccess) return ncclUnhandledCudaError;
  World* w = c->w;
  std::unique_lock<std::mutex> l(w->m);
  if (w->ag_arrived == 0) w->ag_in.assign(w->n, {});
  w->ag_in[c->rank] = std::move(mine);
  const uint64_t gen = w->ag_gen;
  if (++w->ag_arrived == w->n) {
    w->ag_out = w->ag_in;
    w->ag_arrived = 0;
    w->ag_gen++;
    w->cv.notify_all();
  } else {
    const auto ab = abandon_after();
    if (ab.count() && !w->cv.wait_for(l, ab, [&] { return w->ag_gen != gen; })) {
      w->ag_arrived--;  // this rank's contribution is withdrawn: the gather never completes
      all->clear();
      return abandon(w, s) == ncclSuccess ? ncclInProgress : ncclUnhandledCudaError;
    }
    if (!w->cv.wait_for(l, kWait, [&] { return w->ag_gen != gen; })) return ncclSystemError;
  }
  all->clear();
  for (auto& v : w->ag_out) all->insert(all->end(), v.begin(), v.end());
  return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t mockrccl_GetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  std::lock_guard<std::mutex> l(g_m);
  memset(id, 0, sizeof *id);
  const uint64_t key = g_next++;
  memcpy(id->internal, &key, sizeof key);
  return ncclSuccess;
}

ncclResult_t mockrccl_CommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  uint64_t key;
  memcpy(&key, id.internal, sizeof key);
  World* w;
  {
    std::lock_guard<std::mutex> l(g_m);
    World*& slot = g_worlds[key];
    if (!slot) {
      slot = new World();
      slot->n = nranks;
    }
    w = slot;
  }
  if (w->n != nranks) return ncclInvalidUsage;
  std::unique_lock<std::mutex> l(w->m);
  w->joined++;
  w->cv.notify_all();
  if (!w->cv.wait_for(l, kWait, [&] { return w->joined == w->n; })) return ncclSystemError;
  *comm = new ncclComm{w, rank};
  return ncclSuccess;
}

ncclResult_t mockrccl_CommDestroy(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  World* w = comm->w;
  delete comm;
  open_gates(w);  // a rank that leaves never posts again
  bool last;
  {
    std::lock_guard<std::mutex> l(w->m);
    last = ++w->destroyed == w->n;
  }
  if (last) {
    (void)hipDeviceSynchronize();
    for (hipEvent_t e : w->events) (void)hipEventDestroy(e);
    for (uint32_t* g : w->gates) (void)hipHostFree(g);
    std::lock_guard<std::mutex> l(g_m);
    for (auto it = g_worlds.begin(); it != g_worlds.end(); ++it)
      if (it->second == w) {
        g_worlds.erase(it);
        break;
      }
    delete w;
  }
  return ncclSuccess;
}

ncclResult_t mockrccl_CommAbort(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  open_gates(comm->w);
  return mockrccl_CommDestroy(comm);
}

const char* mockrccl_GetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "mock rccl: success";
    case ncclSystemError: return "mock rccl: a partner rank did not post within 60 s";
    case ncclInvalidUsage: return "mock rccl: send and receive sizes differ";
    case ncclInvalidArgument: return "mock rccl: invalid argument";
    default: return "mock rccl: HIP call failed";
  }
}

ncclResult_t mockrccl_GroupStart() {
  t_depth++;
  return ncclSuccess;
}

ncclResult_t mockrccl_GroupEnd() {
  if (t_depth <= 0) return ncclInvalidUsage;
  if (--t_depth) return ncclSuccess;
  std::vector<Op> ops;
  ops.swap(t_ops);
  ncclResult_t r = t_err != ncclSuccess ? t_err : run(ops);
  t_err = ncclSuccess;
  return r;
}

ncclResult_t mockrccl_Send(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s) {
  const size_t es = type_size(t);
  if (!es) return ncclInvalidArgument;
  return enqueue({true, const_cast<void*>(buf), count * es, peer, comm, s});
}

ncclResult_t mockrccl_Recv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s) {
  const size_t es = type_size(t);
  if (!es) return ncclInvalidArgument;
  return enqueue({false, buf, count * es, peer, comm, s});
}

ncclResult_t mockrccl_AllToAll(const void* send, void* recv, size_t count, ncclDataType_t t, ncclComm_t comm,
                          hipStream_t s) {
  const size_t es = type_size(t);
  if (!es || !comm) return ncclInvalidArgument;
  const size_t b = count * es;
  std::vector<Op> ops;
  for (int r = 0; r < comm->w->n; ++r) {
    ops.push_back({true, const_cast<uint8_t*>(static_cast<const uint8_t*>(send)) + r * b, b, r, comm, s});
    ops.push_back({false, static_cast<uint8_t*>(recv) + r * b, b, r, comm, s});
  }
  return run(ops);
}

ncclResult_t mockrccl_AllGather(const void* send, void* recv, size_t count, ncclDataType_t t, ncclComm_t comm,
                           hipStream_t s) {
  const size_t es = type_size(t);
  if (!es || !comm) return ncclInvalidArgument;
  std::vector<uint8_t> all;
  ncclResult_t r = host_allgather(comm, send, count * es, s, &all);
  if (r == ncclInProgress) return ncclSuccess;  // abandoned: the stream waits at its gate
  if (r != ncclSuccess) return r;
  return hipMemcpy(recv, all.data(), all.size(), hipMemcpyHostToDevice) == hipSuccess ? ncclSuccess
                                                                                     : ncclUnhandledCudaError;
}

ncclResult_t mockrccl_AllReduce(const void* send, void* recv, size_t count, ncclDataType_t t, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t s) {
  if (!comm || (t != ncclUint64 && t != ncclInt64) || (op != ncclSum && op != ncclMax && op != ncclMin))
    return ncclInvalidArgument;
  std::vector<uint8_t> all;
  ncclResult_t r = host_allgather(comm, send, count * 8, s, &all);
  if (r == ncclInProgress) return ncclSuccess;  // abandoned: the stream waits at its gate
  if (r != ncclSuccess) return r;
  std::vector<uint64_t> v(all.size() / 8), out(count);
  memcpy(v.data(), all.data(), all.size());
  for (size_t i = 0; i < count; ++i) {
    uint64_t acc = v[i];
    for (int k = 1; k < comm->w->n; ++k) {
      const uint64_t x = v[k * count + i];
      if (op == ncclSum) acc += x;
      else if (t == ncclUint64) acc = op == ncclMax ? std::max(acc, x) : std::min(acc, x);
      else acc = static_cast<uint64_t>(op == ncclMax ? std::max<int64_t>(acc, x) : std::min<int64_t>(acc, x));
    }
    out[i] = acc;
  }
  return hipMemcpy(recv, out.data(), count * 8, hipMemcpyHostToDevice) == hipSuccess ? ncclSuccess
                                                                                   : ncclUnhandledCudaError;
}

}  // extern "C"
