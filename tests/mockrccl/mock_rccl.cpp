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
// The all-to-all and the all-reduce are asynchronous, as RCCL's are: the call records an event and
// enqueues a gate kernel on the caller's stream and returns at once; the rank that posts last moves
// the data (on a service stream, after every rank's event) and opens every gate.  So a rank whose
// peer never posts sees its stream stop at the gate, exactly where RCCL's kernel would wait, and the
// engine's own bounded host waits (TGSIM_COMM_TIMEOUT_MS) are what end it.  ncclCommAbort (and the
// destroy of any rank) opens the gates of every collective that can no longer complete.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <chrono>
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

// One asynchronous collective (all-to-all or all-reduce), matched across ranks by issue order.
struct Coll {
  int kind = 0;  // 0 all-to-all (bytes per peer), 1 all-reduce (count u64 words)
  size_t bytes = 0, count = 0;
  ncclRedOp_t op = ncclSum;
  ncclDataType_t type = ncclUint64;
  int posted = 0;
  struct Part {
    const void* send = nullptr;
    void* recv = nullptr;
    hipEvent_t ready = nullptr;
    uint32_t* gate = nullptr;  // pinned, coherent: 0 closed, 1 data in place, 2 aborted
  };
  std::vector<Part> parts;
};

struct World {
  int n = 0, joined = 0, destroyed = 0;
  bool aborted = false;
  std::vector<uint64_t> next_coll;                  // per rank: collectives issued so far
  std::map<uint64_t, std::shared_ptr<Coll>> colls;  // not yet complete, by issue index
  std::vector<uint32_t*> gates;                     // freed with the world
  hipStream_t svc = nullptr;                        // the completing rank's copies
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
  } else if (!w->cv.wait_for(l, kWait, [&] { return w->ag_gen != gen; })) {
    return ncclSystemError;
  }
  all->clear();
  for (auto& v : w->ag_out) all->insert(all->end(), v.begin(), v.end());
  return ncclSuccess;
}

// Holds the caller's stream until the collective's data is in place (or it was aborted); bounded
// (120 s of s_memrealtime at 100 MHz) so that no wave outlives a test that forgot to abort.
__global__ void k_gate(const uint32_t* gate) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > 12000000000ull) break;
    __builtin_amdgcn_s_sleep(100);
  }
}

void open_gates(Coll& c, uint32_t v) {
  for (auto& p : c.parts)
    if (p.gate) __atomic_store_n(p.gate, v, __ATOMIC_RELEASE);
}

// The last rank to post moves the data once every rank's stream has reached the collective.
ncclResult_t complete(World* w, Coll& c) {
  for (auto& p : c.parts)
    if (hipEventSynchronize(p.ready) != hipSuccess) return ncclUnhandledCudaError;
  const int n = w->n;
  if (c.kind == 0) {
    for (int q = 0; q < n; ++q)
      for (int r = 0; r < n; ++r)
        if (c.bytes && hipMemcpyAsync(static_cast<uint8_t*>(c.parts[q].recv) + r * c.bytes,
                                      static_cast<const uint8_t*>(c.parts[r].send) + q * c.bytes, c.bytes,
                                      hipMemcpyDeviceToDevice, w->svc) != hipSuccess)
          return ncclUnhandledCudaError;
  } else {
    std::vector<uint64_t> v(n * c.count), out(c.count);
    for (int r = 0; r < n; ++r)
      if (hipMemcpyAsync(v.data() + r * c.count, c.parts[r].send, c.count * 8, hipMemcpyDeviceToHost, w->svc) != hipSuccess)
        return ncclUnhandledCudaError;
    if (hipStreamSynchronize(w->svc) != hipSuccess) return ncclUnhandledCudaError;
    for (size_t i = 0; i < c.count; ++i) {
      uint64_t acc = v[i];
      for (int k = 1; k < n; ++k) {
        const uint64_t x = v[k * c.count + i];
        if (c.op == ncclSum) acc += x;
        else if (c.type == ncclUint64) acc = c.op == ncclMax ? std::max(acc, x) : std::min(acc, x);
        else acc = static_cast<uint64_t>(c.op == ncclMax ? std::max<int64_t>(acc, x) : std::min<int64_t>(acc, x));
      }
      out[i] = acc;
    }
    for (int r = 0; r < n; ++r)
      if (hipMemcpyAsync(c.parts[r].recv, out.data(), c.count * 8, hipMemcpyHostToDevice, w->svc) != hipSuccess)
        return ncclUnhandledCudaError;
  }
  if (hipStreamSynchronize(w->svc) != hipSuccess) return ncclUnhandledCudaError;
  open_gates(c, 1u);
  return ncclSuccess;
}

ncclResult_t post(ncclComm* comm, const Coll& shape, const void* send, void* recv, hipStream_t s) {
  World* w = comm->w;
  uint32_t* gate = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&gate), sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped) !=
      hipSuccess)
    return ncclUnhandledCudaError;
  *gate = 0;
  hipEvent_t ready = new_event(w);
  if (!ready || hipEventRecord(ready, s) != hipSuccess) return ncclUnhandledCudaError;
  hipLaunchKernelGGL(k_gate, dim3(1), dim3(1), 0, s, gate);
  if (hipGetLastError() != hipSuccess) return ncclUnhandledCudaError;
  std::shared_ptr<Coll> done;
  {
    std::lock_guard<std::mutex> l(w->m);
    w->gates.push_back(gate);
    if (w->aborted) {
      *gate = 2u;
      return ncclSystemError;
    }
    const uint64_t k = w->next_coll[comm->rank]++;
    std::shared_ptr<Coll>& c = w->colls[k];
    if (!c) {
      c = std::make_shared<Coll>(shape);
      c->parts.assign(w->n, {});
    } else if (c->kind != shape.kind || c->bytes != shape.bytes || c->count != shape.count) {
      *gate = 2u;
      return ncclInvalidUsage;
    }
    c->parts[comm->rank] = {send, recv, ready, gate};
    if (++c->posted == w->n) {
      done = c;
      w->colls.erase(k);
    }
  }
  return done ? complete(w, *done) : ncclSuccess;
}

// Every collective that has not completed can no longer complete: its gates open as aborted.
void abort_world(World* w) {
  std::lock_guard<std::mutex> l(w->m);
  w->aborted = true;
  for (auto& kv : w->colls) open_gates(*kv.second, 2u);
  w->colls.clear();
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
      slot->next_coll.assign(nranks, 0);
      if (hipStreamCreateWithFlags(&slot->svc, hipStreamNonBlocking) != hipSuccess) return ncclUnhandledCudaError;
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
  abort_world(w);  // a rank that leaves never posts again
  bool last;
  {
    std::lock_guard<std::mutex> l(w->m);
    last = ++w->destroyed == w->n;
  }
  if (last) {
    (void)hipDeviceSynchronize();
    for (hipEvent_t e : w->events) (void)hipEventDestroy(e);
    for (uint32_t* g : w->gates) (void)hipHostFree(g);
    if (w->svc) (void)hipStreamDestroy(w->svc);
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
  abort_world(comm->w);
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
  Coll shape;
  shape.kind = 0;
  shape.bytes = count * es;
  return post(comm, shape, send, recv, s);
}

ncclResult_t mockrccl_AllGather(const void* send, void* recv, size_t count, ncclDataType_t t, ncclComm_t comm,
                           hipStream_t s) {
  const size_t es = type_size(t);
  if (!es || !comm) return ncclInvalidArgument;
  std::vector<uint8_t> all;
  ncclResult_t r = host_allgather(comm, send, count * es, s, &all);
  if (r != ncclSuccess) return r;
  return hipMemcpy(recv, all.data(), all.size(), hipMemcpyHostToDevice) == hipSuccess ? ncclSuccess
                                                                                     : ncclUnhandledCudaError;
}

ncclResult_t mockrccl_AllReduce(const void* send, void* recv, size_t count, ncclDataType_t t, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t s) {
  if (!comm || (t != ncclUint64 && t != ncclInt64) || (op != ncclSum && op != ncclMax && op != ncclMin))
    return ncclInvalidArgument;
  Coll shape;
  shape.kind = 1;
  shape.count = count;
  shape.op = op;
  shape.type = t;
  return post(comm, shape, send, recv, s);
}

}  // extern "C"
