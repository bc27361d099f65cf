// tgsim_kernels.hip — gfx950 kernels of the per-packet network.Config enforcement path.
//
//   k_sim          K1+K2+K3+K4 of SURVEY §2.1: FIB filter, netem enqueue decisions (Philox
//                  keyed by (seed, src, dst, seq)), netem queue limit, eligibility queue and HTB
//                  token bucket.  One lane owns one source for the whole step (the state is a
//                  sequential recurrence per source); a step spans many ticks so one launch
//                  carries millions of packets.
//   k_apply_cfg    K9: scatters compiled LinkShape deltas into the SoA parameter/state arrays.
//   k_gen_*        synthetic storm traffic written straight into the CSR input.
//   k_gossip_*     closed-loop gossip flood traffic (C4): receipts at delivery, forwards per window.
//   k_route_*      groups scheduled records by the destination's shard (input of the RCCL
//                  all-to-all; plain compaction on one GPU).
//   k_dst_*        K5: counting sort of deliveries by destination, then a per-destination sort
//                  by (t, src, seq, clone-first).
#include "tgsim_launch.h"

namespace tgsim {

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 (Random123 constants).
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                       uint32_t k0, uint32_t k1, uint32_t r[4]) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t h0 = __umulhi(0xD2511F53u, c0), l0 = 0xD2511F53u * c0;
    const uint32_t h1 = __umulhi(0xCD9E8D57u, c2), l1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  r[0] = c0; r[1] = c1; r[2] = c2; r[3] = c3;
}

// get_crandom(): correlated uniform, state updated only when rho != 0.
__device__ __forceinline__ uint32_t crand(uint32_t raw, uint32_t rho, uint32_t& last) {
  if (rho == 0) return raw;
  const uint64_t r = (uint64_t)rho + 1;
  const uint32_t a = (uint32_t)(((uint64_t)raw * ((1ull << 32) - r) + (uint64_t)last * r) >> 32);
  last = a;
  return a;
}

// Queued item (16 B): w0 = e | len << 46 | flags << 62, seq, dst.
__device__ __forceinline__ uint64_t w0_of(const uint4& a) {
  return ((uint64_t)a.y << 32) | a.x;
}
__device__ __forceinline__ bool item_lt(const uint4& a, const uint4& b) {
  // (e, seq, clone first), evaluated without branches: a divergent compare in the sift loop costs
  // more than the LDS round trip it guards.
  const uint64_t ea = w0_of(a) & kEMask, eb = w0_of(b) & kEMask;
  const bool dup_first = (a.y >> 30 & 1u) > (b.y >> 30 & 1u);
  const bool seq_lt = (a.z < b.z) | ((a.z == b.z) & dup_first);
  return (ea < eb) | ((ea == eb) & seq_lt);
}

// Per-workgroup LDS: the eligibility heaps and departure rings of kSpw sources, plus the staging
// area where all 64 lanes leave the prefetched record + Philox draws for the sequential lanes.
struct alignas(16) Pre {
  uint4 rec;   // dst, seq, tick, len | filter verdict << 16
  uint4 r0;    // draw 0: dup, loss, corrupt, reorder
  uint4 r2;    // draw 2 (clone): loss, corrupt, reorder, delay
  uint4 r1;    // draw 1: delay word in .x
};
struct SimLds {
  uint4 heap[(kHeapCap + 4) * kSpw];  // slot k of source j at k * kSpw + j (+4: child reads past n)
  uint64_t ring[kHeapCap * kSpw];  // departure times, circular per source
  Pre stage[kWave];
  uint8_t vst[kWave];              // verdicts of the batch, stored back coalesced
};
static_assert(sizeof(SimLds) <= 163840, "simulate workgroup exceeds 160 KiB of LDS");

constexpr uint32_t kFvPass = 0xFFu;

struct Lane {
  uint4* hb;        // LDS heap of this source, stride kSpw
  uint64_t* rb;     // LDS ring of this source, stride kSpw
  tgsim_delivery* emit;
  uint32_t n_emit;
  SrcState st;
  SrcParams p;
  uint32_t src;
  uint32_t scheduled, corrupted;
  uint64_t bytes;
  uint32_t err;
  // register copies of the two values the common (queue-full) path compares against
  uint64_t top_e;   // eligibility time of the heap root, ~0 when the heap is empty
  uint64_t head_d;  // departure time at the ring head, ~0 when the ring is empty
#ifdef TGSIM_PROFILE
  uint64_t pc[6];   // diagnostic build: cycles in admit / heap_pop / heap_push and their counts
#endif
};

// Diagnostic build (-DTGSIM_PROFILE, libtgsim_prof.so): s_memtime cycle accounting of the
// sequential recurrence, reported through the stamp slots.  Compiled out of the product.
#ifdef TGSIM_PROFILE
#define PROF_T0() const uint64_t _pt0 = __builtin_amdgcn_s_memtime()
#define PROF_ADD(L, k) do { (L).pc[2 * (k)] += __builtin_amdgcn_s_memtime() - _pt0; (L).pc[2 * (k) + 1]++; } while (0)
#else
#define PROF_T0() do {} while (0)
#define PROF_ADD(L, k) do {} while (0)
#endif

__device__ __forceinline__ uint4 hget(const Lane& L, uint32_t k) { return L.hb[k * kSpw]; }
__device__ __forceinline__ void hset(Lane& L, uint32_t k, const uint4& v) { L.hb[k * kSpw] = v; }

// 4-ary min-heap on (e, seq, clone first) in LDS: the four children of a node are read together,
// so a sift-down level costs one LDS round trip and the depth is log4(1024) = 5.
__device__ __forceinline__ void heap_push(Lane& L, uint4 it) {
  PROF_T0();
  const uint64_t e = w0_of(it) & kEMask;
  if (e < L.top_e) L.top_e = e;  // ties keep the root's e: only the time is cached
  uint32_t i = L.st.heap_n++;
  while (i > 0) {
    const uint32_t par = (i - 1) >> 2;
    const uint4 pv = hget(L, par);
    if (!item_lt(it, pv)) break;
    hset(L, i, pv);
    i = par;
  }
  hset(L, i, it);
  PROF_ADD(L, 2);
}

__device__ __forceinline__ void heap_pop(Lane& L) {
  PROF_T0();
  const uint32_t n = --L.st.heap_n;
  const uint4 last = hget(L, n);
  uint32_t i = 0;
  for (;;) {
    const uint32_t c = 4 * i + 1;
    if (c >= n) break;
    const uint4 v0 = hget(L, c), v1 = hget(L, c + 1), v2 = hget(L, c + 2), v3 = hget(L, c + 3);
    uint4 best = v0;
    uint32_t bi = c;
    if (c + 1 < n && item_lt(v1, best)) { best = v1; bi = c + 1; }
    if (c + 2 < n && item_lt(v2, best)) { best = v2; bi = c + 2; }
    if (c + 3 < n && item_lt(v3, best)) { best = v3; bi = c + 3; }
    if (!item_lt(best, last)) break;
    hset(L, i, best);
    i = bi;
  }
  if (n) hset(L, i, last);
  L.top_e = n ? (w0_of(hget(L, 0)) & kEMask) : ~0ull;
  PROF_ADD(L, 1);
}

// HTB class serving the netem queue in eligibility order: d = max(e, TAT),
// TAT' = max(TAT, e - B) + len * mult >> shift.
__device__ __forceinline__ void htb_until(Lane& L, uint64_t horizon) {
  while (L.top_e < horizon) {
    const uint4 top = hget(L, 0);
    const uint64_t w0 = w0_of(top);
    const uint64_t e = w0 & kEMask;
    if (e >= horizon) break;
    heap_pop(L);
    const uint32_t len = (uint32_t)(w0 >> 46) & 0xFFFFu;
    const uint32_t flags = (uint32_t)(w0 >> 62);
    const uint64_t d = e > L.st.tat ? e : L.st.tat;
    const uint64_t fl = e > L.p.burst_ns ? e - L.p.burst_ns : 0;
    const uint64_t base = L.st.tat > fl ? L.st.tat : fl;
    L.st.tat = base + (((uint64_t)len * L.p.mult) >> (L.p.shift_ext & 0xFFu));
    L.rb[((L.st.ring_head + L.st.ring_n) & (kHeapCap - 1)) * kSpw] = d;
    if (L.st.ring_n++ == 0) L.head_d = d;
    uint64_t* rw = reinterpret_cast<uint64_t*>(L.emit + L.n_emit++);
    rw[0] = d;
    rw[1] = ((uint64_t)top.w << 32) | L.src;
    rw[2] = ((uint64_t)flags << 48) | ((uint64_t)len << 32) | top.z;
    L.scheduled++;
    L.bytes += len;
    L.corrupted += (flags >> 1) & 1u;
  }
}

// Queue-limit check and insertion of one netem item whose eligibility time e is already known.
__device__ __forceinline__ uint32_t admit(Lane& L, uint32_t limit, uint64_t T, uint64_t e, uint32_t dst,
                                          uint32_t seq, uint32_t len, uint32_t flags) {
  PROF_T0();
  htb_until(L, T);
  while (L.head_d < T) {  // departures before T leave the netem queue
    L.st.ring_head = (L.st.ring_head + 1) & (kHeapCap - 1);
    L.head_d = --L.st.ring_n ? L.rb[L.st.ring_head * kSpw] : ~0ull;
  }
  if (L.st.heap_n + L.st.ring_n >= limit) {
    PROF_ADD(L, 0);
    return TGSIM_V_QUEUE_FULL;
  }
  const uint64_t w0 = e | ((uint64_t)(len & 0xFFFFu) << 46) | ((uint64_t)flags << 62);
  heap_push(L, make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), seq, dst));
  PROF_ADD(L, 0);
  return TGSIM_V_SCHEDULED;
}

// tabledist() uniform branch: e = T + max(0, L - sigma + raw mod 2 sigma), or T + L when sigma = 0.
__device__ __forceinline__ uint64_t delayed(const SrcParams& p, uint64_t T, uint32_t raw) {
  if (p.sigma == 0) return T + p.lat_ns;
  const uint32_t m = 2u * (uint32_t)p.sigma;
  const int64_t delay = (int64_t)(raw % m) + (int64_t)p.lat_ns - (int64_t)p.sigma;
  return delay > 0 ? T + (uint64_t)delay : T;
}

// netem_enqueue from the queue-limit check on, for sources with correlated draws: the reorder
// decision consumes correlated state only when the packet passes the limit check.
__device__ __forceinline__ uint32_t enqueue(Lane& L, uint32_t limit, uint64_t T, uint32_t dst,
                                            uint32_t seq, uint32_t len, uint32_t reo_raw,
                                            uint32_t delay_raw, uint32_t flags) {
  htb_until(L, T);
  while (L.head_d < T) {
    L.st.ring_head = (L.st.ring_head + 1) & (kHeapCap - 1);
    L.head_d = --L.st.ring_n ? L.rb[L.st.ring_head * kSpw] : ~0ull;
  }
  if (L.st.heap_n + L.st.ring_n >= limit) return TGSIM_V_QUEUE_FULL;
  bool reordered = false;
  if (L.p.thr_reo) reordered = !(L.p.thr_reo < crand(reo_raw, L.p.rho_reo, L.st.last_reo));
  uint64_t e = reordered ? T : delayed(L.p, T, delay_raw);
  if (e > kEMask) {
    L.err |= kErrTimeOverflow;
    e = kEMask;
  }
  const uint64_t w0 = e | ((uint64_t)(len & 0xFFFFu) << 46) | ((uint64_t)flags << 62);
  heap_push(L, make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), seq, dst));
  return TGSIM_V_SCHEDULED;
}

__device__ __forceinline__ uint32_t fib_lookup(const Interval* iv, uint32_t n, uint32_t ip) {
  uint32_t lo = 0, hi = n;  // binary search over sorted disjoint intervals
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (iv[mid].hi < ip) lo = mid + 1;
    else hi = mid;
  }
  if (lo < n && iv[lo].lo <= ip) return iv[lo].act;
  return TGSIM_ACCEPT;
}

// Connectivity, routing policy and FIB rules (no queue state involved).  Returns kFvPass or the
// verdict.
__device__ __forceinline__ uint32_t filter(const SimArgs& a, const SrcParams& p, bool src_on, uint32_t dst) {
  if (dst == TGSIM_EXTERNAL) {
    if (!src_on) return TGSIM_V_DISCONNECTED;
    return (p.shift_ext >> 8 & 1u) ? TGSIM_V_EXTERNAL : TGSIM_V_NO_ROUTE;
  }
  if (!src_on || (a.any_disabled && !a.enabled[dst])) return TGSIM_V_DISCONNECTED;
  if (p.rule_n) {
    const uint32_t act = fib_lookup(a.rules + p.rule_off, p.rule_n, a.ip[dst]);
    if (act == TGSIM_DROP) return TGSIM_V_BLACKHOLE;
    if (act == TGSIM_REJECT) return TGSIM_V_PROHIBIT;
  }
  return kFvPass;
}

// Sequential netem_enqueue for one offered packet of a correlated source (raw draws staged).
__device__ __forceinline__ uint32_t process_corr(Lane& L, uint32_t limit, uint64_t T, const Pre& pre) {
  const uint32_t dst = pre.rec.x, seq = pre.rec.y, len = pre.rec.w & 0xFFFFu;
  const uint32_t fv = pre.rec.w >> 16;
  if (fv != kFvPass) return 0xF0u | fv;
  int count = 1;
  if (L.p.thr_dup && L.p.thr_dup >= crand(pre.r0.x, L.p.rho_dup, L.st.last_dup)) ++count;
  if (L.p.thr_loss && L.p.thr_loss >= pre.r0.y) --count;
  if (count == 0) return 0xF0u | TGSIM_V_LOSS;
  uint32_t cv = TGSIM_V_NONE;
  if (count == 2) {  // the clone re-enters the root qdisc with duplicate = 0
    if (L.p.thr_loss && L.p.thr_loss >= pre.r2.x) {
      cv = TGSIM_V_LOSS;
    } else {
      uint32_t fl = TGSIM_FLAG_DUP;
      if (L.p.thr_cor && L.p.thr_cor >= crand(pre.r2.y, L.p.rho_cor, L.st.last_cor)) fl |= TGSIM_FLAG_CORRUPT;
      cv = enqueue(L, limit, T, dst, seq, len, pre.r2.z, pre.r2.w, fl);
    }
  }
  uint32_t fl = 0;
  if (L.p.thr_cor && L.p.thr_cor >= crand(pre.r0.z, L.p.rho_cor, L.st.last_cor)) fl |= TGSIM_FLAG_CORRUPT;
  const uint32_t ov = enqueue(L, limit, T, dst, seq, len, pre.r0.w, pre.r1.x, fl);
  return (cv << 4) | ov;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, o, 64);
    const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor(v, o, 64));
  return v;
}

// Staged candidate of an uncorrelated source (48 B of a Pre slot): everything netem decides
// without queue state is resolved by the lane that loaded the packet.
//   rec = {T lo, T hi, e_orig lo, e_orig hi}, r0 = {e_clone lo, e_clone hi, dst, seq},
//   r2.x = len | orig flags << 16 | clone flags << 18 | clone state << 20 | batch slot << 24
// clone state: 0 none, 1 lost, 2 queue candidate.

// One wavefront per workgroup owns kSpw sources (kSpw = 1: one netem queue per wavefront, so the
// sequential recurrences of different sources are independent waves the SIMDs interleave).  Per
// batch every lane (j, r) = (lane % kSpw, lane / kSpw) loads record r of source j's next kAhead
// records and resolves the filter and all Philox-driven decisions; lane j then replays the queue
// candidates (compacted with a ballot) through the netem-limit / eligibility-heap / HTB
// recurrence held in LDS.  Sources with correlated draws (get_crandom, rho != 0) replay the raw
// draws sequentially instead.  The next batch's records are in flight during the sequential phase.
// The simulate workgroup is a single wavefront: cross-lane LDS hand-offs only need this wave's
// LDS operations to have landed (lgkmcnt(0)), not the vmcnt(0) drain of outstanding global stores
// and prefetch loads that __syncthreads() implies.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt(63) expcnt(7) lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  __asm__ volatile("" ::: "memory");
}

__device__ __forceinline__ void stamp(const SimArgs& a, uint32_t lane, uint32_t k, uint64_t v) {
  if (a.stamps && lane == 0) a.stamps[(size_t)blockIdx.x * kStampSlots + k] = v;
}

__global__ __launch_bounds__(kWave) void k_sim(SimArgs a) {
  __shared__ SimLds lds;
  const uint32_t lane = threadIdx.x;
  // heavy-first dispatch order (previous step's HTB work per source), identity when absent
  const uint32_t s0 = (kSpw == 1 && a.order) ? a.order[blockIdx.x] : blockIdx.x * kSpw;
  stamp(a, lane, 0, __builtin_amdgcn_s_memrealtime());
  // ---- load heaps and rings of the workgroup's sources into LDS
  for (uint32_t j = 0; j < kSpw; ++j) {
    const uint32_t s = s0 + j;
    if (s >= a.n_src) break;
    const uint32_t hn = a.state[s].heap_n, rn = a.state[s].ring_n;
    const uint4* gh = a.heap + (size_t)s * kHeapCap;
    const uint64_t* gr = a.ring + (size_t)s * kHeapCap;
    for (uint32_t k0 = 0; k0 < hn; k0 += 4 * kWave) {  // four loads in flight per lane
      const uint32_t k = k0 + lane;
      const uint4 v0 = gh[min(k, hn - 1)], v1 = gh[min(k + kWave, hn - 1)];
      const uint4 v2 = gh[min(k + 2 * kWave, hn - 1)], v3 = gh[min(k + 3 * kWave, hn - 1)];
      if (k < hn) lds.heap[k * kSpw + j] = v0;
      if (k + kWave < hn) lds.heap[(k + kWave) * kSpw + j] = v1;
      if (k + 2 * kWave < hn) lds.heap[(k + 2 * kWave) * kSpw + j] = v2;
      if (k + 3 * kWave < hn) lds.heap[(k + 3 * kWave) * kSpw + j] = v3;
    }
    for (uint32_t k0 = 0; k0 < rn; k0 += 4 * kWave) {
      const uint32_t k = k0 + lane;
      const uint64_t v0 = gr[min(k, rn - 1)], v1 = gr[min(k + kWave, rn - 1)];
      const uint64_t v2 = gr[min(k + 2 * kWave, rn - 1)], v3 = gr[min(k + 3 * kWave, rn - 1)];
      if (k < rn) lds.ring[k * kSpw + j] = v0;
      if (k + kWave < rn) lds.ring[(k + kWave) * kSpw + j] = v1;
      if (k + 2 * kWave < rn) lds.ring[(k + 2 * kWave) * kSpw + j] = v2;
      if (k + 3 * kWave < rn) lds.ring[(k + 3 * kWave) * kSpw + j] = v3;
    }
  }
  // ---- per-lane roles
  const uint32_t pj = lane % kSpw, pr = lane / kSpw;
  const bool prefetcher = pr < kAhead && s0 + pj < a.n_src;
  SrcParams pp;
  uint64_t pbeg = 0, pend = 0;
  bool src_on = false;
  uint32_t psrc = 0;
  if (prefetcher) {
    pp = a.params[s0 + pj];
    pbeg = a.off[s0 + pj];
    pend = a.off[s0 + pj + 1];
    psrc = a.shard_begin + s0 + pj;
    src_on = a.enabled[psrc] != 0;
  }
  // correlated sources replay raw draws; with kSpw = 1 this is uniform across the wavefront
  const bool corr = kSpw != 1 || (prefetcher && (pp.rho_dup | pp.rho_cor | pp.rho_reo) != 0);
  const bool any_corr = __any(corr);
  const bool seq_lane = lane < kSpw && s0 + lane < a.n_src;
  Lane L;
#ifdef TGSIM_PROFILE
  for (int k = 0; k < 6; ++k) L.pc[k] = 0;
  uint64_t prof_par = 0, prof_rep = 0, prof_runs = 0;
#endif
  L.scheduled = L.corrupted = 0;
  L.bytes = 0;
  L.err = 0;
  L.n_emit = 0;
  uint64_t sbeg = 0, send = 0;
  uint32_t nb = 0;
  if (seq_lane) {
    const uint32_t s = s0 + lane;
    L.p = a.params[s];
    L.st = a.state[s];
    L.st.ring_head = 0;  // rings are stored compacted
    L.src = a.shard_begin + s;
    L.hb = lds.heap + lane;
    L.rb = lds.ring + lane;
    sbeg = a.off[s];
    send = a.off[s + 1];
    L.emit = a.emit + 2 * sbeg + (uint64_t)kHeapCap * s;
    nb = (uint32_t)((send - sbeg + kAhead - 1) / kAhead);
  }
  const uint32_t n_batches = wave_max(nb);
  const uint64_t qbytes_in = seq_lane ? 16ull * L.st.heap_n + 8ull * L.st.ring_n : 0;
  uint64_t c_off = 0, c_clone = 0, c_v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t perr = 0;
  wave_lds_sync();
  if (seq_lane) {
    L.top_e = L.st.heap_n ? (w0_of(lds.heap[lane]) & kEMask) : ~0ull;
    L.head_d = L.st.ring_n ? lds.ring[lane] : ~0ull;
  }
  stamp(a, lane, 1, __builtin_amdgcn_s_memrealtime());
  // ---- batch loop
  uint64_t idx = pbeg + pr;
  InRec rec = {}, rec2 = {};  // records of batches b and b + 1 (two batches in flight)
  if (prefetcher && idx < pend) rec = a.in[idx];
  if (prefetcher && idx + kAhead < pend) rec2 = a.in[idx + kAhead];
  for (uint32_t b = 0; b < n_batches; ++b) {
#ifdef TGSIM_PROFILE
    const uint64_t pb0 = __builtin_amdgcn_s_memtime();
#endif
    const uint64_t my_idx = idx;  // the record this lane stages in this batch
    const bool staged = prefetcher && my_idx < pend;
    uint32_t n_cand = 0;
    if (any_corr) {
      // ---------- correlated path: stage raw draws, replay every packet in order
      if (staged) {
        Pre pre;
        const uint32_t fv = filter(a, pp, src_on, rec.dst);
        pre.rec = make_uint4(rec.dst, rec.seq, rec.tick, (rec.len & 0xFFFFu) | (fv << 16));
        pre.r0 = pre.r1 = pre.r2 = make_uint4(0, 0, 0, 0);
        if (fv == kFvPass) {
          uint32_t r[4];
          philox(psrc, rec.dst, rec.seq, 0, a.key0, a.key1, r);
          pre.r0 = make_uint4(r[0], r[1], r[2], r[3]);
          if (pp.thr_dup) {
            philox(psrc, rec.dst, rec.seq, 2, a.key0, a.key1, r);
            pre.r2 = make_uint4(r[0], r[1], r[2], r[3]);
          }
          if (pp.sigma) {
            philox(psrc, rec.dst, rec.seq, 1, a.key0, a.key1, r);
            pre.r1.x = r[0];
          }
        }
        lds.stage[lane] = pre;
      }
    } else {
      // ---------- uncorrelated path: resolve everything but the queue in parallel
      uint32_t fin = 0;  // final verdict when no queue decision is needed
      bool cand = false;
      Pre pre;
      if (staged) {
        const uint64_t T = a.t0_ns + (uint64_t)rec.tick * a.tick_ns;
        const uint32_t fv = filter(a, pp, src_on, rec.dst);
        if (fv != kFvPass) {
          fin = 0xF0u | fv;
        } else {
          uint32_t r0[4];
          philox(psrc, rec.dst, rec.seq, 0, a.key0, a.key1, r0);
          const int count = 1 + (pp.thr_dup && pp.thr_dup >= r0[0]) - (pp.thr_loss && pp.thr_loss >= r0[1]);
          if (count == 0) {
            fin = 0xF0u | TGSIM_V_LOSS;
          } else {
            uint32_t cstate = 0, flc = TGSIM_FLAG_DUP;
            uint64_t ec = ~0ull;
            if (count == 2) {
              uint32_t r2[4];
              philox(psrc, rec.dst, rec.seq, 2, a.key0, a.key1, r2);
              if (pp.thr_loss && pp.thr_loss >= r2[0]) {
                cstate = 1;
              } else {
                cstate = 2;
                if (pp.thr_cor && pp.thr_cor >= r2[1]) flc |= TGSIM_FLAG_CORRUPT;
                ec = (pp.thr_reo && pp.thr_reo >= r2[2]) ? T : delayed(pp, T, r2[3]);
              }
            }
            const uint32_t flo = (pp.thr_cor && pp.thr_cor >= r0[2]) ? TGSIM_FLAG_CORRUPT : 0u;
            uint64_t eo;
            if (pp.thr_reo && pp.thr_reo >= r0[3]) {
              eo = T;
            } else if (pp.sigma) {
              uint32_t r1[4];
              philox(psrc, rec.dst, rec.seq, 1, a.key0, a.key1, r1);
              eo = delayed(pp, T, r1[0]);
            } else {
              eo = T + pp.lat_ns;
            }
            if (eo > kEMask || (cstate == 2 && ec > kEMask)) perr = 1;
            pre.rec = make_uint4((uint32_t)T, (uint32_t)(T >> 32), (uint32_t)eo, (uint32_t)(eo >> 32));
            pre.r0 = make_uint4((uint32_t)ec, (uint32_t)(ec >> 32), rec.dst, rec.seq);
            pre.r2 = make_uint4((rec.len & 0xFFFFu) | (flo << 16) | (flc << 18) | (cstate << 20) | (pr << 24),
                                0, 0, 0);
            cand = true;
          }
        }
      }
      const uint64_t m = __ballot(cand);
      n_cand = __popcll(m);
      if (cand) {
        const Pre p2 = pre;
        const uint32_t slot = __popcll(m & ((1ull << lane) - 1));
        lds.stage[slot].rec = p2.rec;
        lds.stage[slot].r0 = p2.r0;
        lds.stage[slot].r2 = p2.r2;
      } else if (staged) {
        lds.vst[lane] = (uint8_t)fin;
      }
    }
    wave_lds_sync();
#ifdef TGSIM_PROFILE
    const uint64_t pb1 = __builtin_amdgcn_s_memtime();
    prof_par += pb1 - pb0;
#endif
    idx += kAhead;
    rec = rec2;
    if (prefetcher && idx + kAhead < pend) rec2 = a.in[idx + kAhead];  // in flight two batches ahead
    if (seq_lane) {
      if (any_corr) {
        const uint64_t first = sbeg + (uint64_t)b * kAhead;
        const uint32_t nr = first < send ? (uint32_t)min((uint64_t)kAhead, send - first) : 0u;
        for (uint32_t r = 0; r < nr; ++r) {
          const Pre pre = lds.stage[r * kSpw + lane];
          const uint64_t T = a.t0_ns + (uint64_t)pre.rec.z * a.tick_ns;
          lds.vst[r * kSpw + lane] = (uint8_t)process_corr(L, a.queue_limit, T, pre);
        }
      }
    }
    if (!any_corr) {
      // Uniform replay of the compacted candidates.  While the netem queue is full its state
      // cannot change before min(next departure, next eligibility), so every candidate offered
      // up to that instant is a QUEUE_FULL drop: the whole run is resolved with one ballot
      // (T is non-decreasing over the candidates); the remaining candidates go through the
      // sequential lane one by one.
      uint64_t Tc = ~0ull;
      uint32_t cinfo = 0;
      if (lane < n_cand) {
        const uint4 r = lds.stage[lane].rec;
        Tc = ((uint64_t)r.y << 32) | r.x;
        cinfo = lds.stage[lane].r2.x;
      }
      uint32_t c = 0;
      while (c < n_cand) {
        uint64_t thr = 0;
        uint32_t full = 0;
        if (lane == 0) {
          thr = L.top_e < L.head_d ? L.top_e : L.head_d;
          full = L.st.heap_n + L.st.ring_n >= a.queue_limit;
        }
        full = __builtin_amdgcn_readfirstlane(full);
        if (full) {
          thr = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(thr >> 32)) << 32) |
                __builtin_amdgcn_readfirstlane((uint32_t)thr);
          const bool drop = lane >= c && lane < n_cand && Tc <= thr;
          const uint64_t m = __ballot(drop);
          if (drop) {
            const uint32_t cst = (cinfo >> 20) & 3u;
            const uint32_t cv = cst == 0 ? TGSIM_V_NONE : (cst == 1 ? TGSIM_V_LOSS : TGSIM_V_QUEUE_FULL);
            lds.vst[cinfo >> 24] = (uint8_t)((cv << 4) | TGSIM_V_QUEUE_FULL);
          }
          c += __popcll(m);
#ifdef TGSIM_PROFILE
          prof_runs++;
#endif
          if (c >= n_cand) break;
        }
        if (lane == 0) {
          const uint4 crec = lds.stage[c].rec, cr0 = lds.stage[c].r0, cr2 = lds.stage[c].r2;
          const uint64_t T = ((uint64_t)crec.y << 32) | crec.x;
          const uint64_t eo = ((uint64_t)crec.w << 32) | crec.z;
          const uint32_t info = cr2.x, len = info & 0xFFFFu, cstate = (info >> 20) & 3u;
          uint32_t cv = cstate == 0 ? TGSIM_V_NONE : TGSIM_V_LOSS;
          if (cstate == 2) {
            const uint64_t ec = ((uint64_t)cr0.y << 32) | cr0.x;
            cv = admit(L, a.queue_limit, T, ec, cr0.z, cr0.w, len, (info >> 18) & 3u);
          }
          const uint32_t ov = admit(L, a.queue_limit, T, eo, cr0.z, cr0.w, len, (info >> 16) & 3u);
          lds.vst[info >> 24] = (uint8_t)((cv << 4) | ov);
        }
        ++c;
      }
    }
    wave_lds_sync();
#ifdef TGSIM_PROFILE
    prof_rep += __builtin_amdgcn_s_memtime() - pb1;
#endif
    if (staged) {
      const uint32_t v = lds.vst[lane];
      a.verdict[my_idx] = (uint8_t)v;
    }
    // statistics from the verdict bytes (wave-uniform ballot counts)
    const uint32_t v = staged ? lds.vst[lane] : 0xFFu;
    c_off += __popcll(__ballot(staged));
    c_clone += __popcll(__ballot(staged && (v >> 4) != TGSIM_V_NONE));
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k)
      c_v[k] += __popcll(__ballot(staged && (v & 15u) == k)) + __popcll(__ballot(staged && (v >> 4) == k));
  }
  stamp(a, lane, 2, __builtin_amdgcn_s_memrealtime());
  if (seq_lane) {
    htb_until(L, a.horizon_ns);
    a.emit_n[s0 + lane] = L.n_emit;
  }
  wave_lds_sync();
  stamp(a, lane, 3, __builtin_amdgcn_s_memrealtime());
  // ---- write back state, heaps and (compacted) rings
  for (uint32_t j = 0; j < kSpw; ++j) {
    const uint32_t s = s0 + j;
    if (s >= a.n_src) break;
    const uint32_t hn = __shfl(L.st.heap_n, j, 64);
    const uint32_t rn = __shfl(L.st.ring_n, j, 64);
    const uint32_t rh = __shfl(L.st.ring_head, j, 64);
    for (uint32_t k = lane; k < hn; k += kWave) a.heap[(size_t)s * kHeapCap + k] = lds.heap[k * kSpw + j];
    for (uint32_t k = lane; k < rn; k += kWave)
      a.ring[(size_t)s * kHeapCap + k] = lds.ring[((rh + k) & (kHeapCap - 1)) * kSpw + j];
  }
  if (seq_lane) {
    L.st.ring_head = 0;
    a.state[s0 + lane] = L.st;
  }
  stamp(a, lane, 4, __builtin_amdgcn_s_memrealtime());
  stamp(a, lane, 5, ((uint64_t)s0 << 32) | n_batches);
  stamp(a, lane, 6, __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)));  // HW_ID
  stamp(a, lane, 7, seq_lane ? ((uint64_t)L.st.heap_n << 32 | L.st.ring_n) : 0);
#ifdef TGSIM_PROFILE
  for (int k = 0; k < 6; ++k) stamp(a, lane, 8 + k, L.pc[k]);
  stamp(a, lane, 14, prof_par);
  stamp(a, lane, 15, (prof_rep << 20) | (prof_runs & 0xFFFFF));
#endif
  const uint64_t sched = wave_sum(seq_lane ? L.scheduled : 0u);
  const uint64_t corrupted = wave_sum(seq_lane ? L.corrupted : 0u);
  const uint64_t bytes = wave_sum(seq_lane ? L.bytes : 0ull);
  const uint64_t qbytes = wave_sum(seq_lane ? qbytes_in + 16ull * L.st.heap_n + 8ull * L.st.ring_n : 0ull);
  const uint64_t err = wave_sum((seq_lane && L.err) || perr ? 1u : 0u);
  if (lane == 0) {
    atomicAdd(&a.stats[kStOffered], (unsigned long long)c_off);
    if (sched) atomicAdd(&a.stats[kStScheduled], (unsigned long long)sched);
    if (c_clone) atomicAdd(&a.stats[kStCloned], (unsigned long long)c_clone);
    if (corrupted) atomicAdd(&a.stats[kStCorrupted], (unsigned long long)corrupted);
    for (int k = 0; k < 8; ++k)
      if (c_v[k]) atomicAdd(&a.stats[kStVerdict0 + k], (unsigned long long)c_v[k]);
    if (bytes) atomicAdd(&a.stats[kStBytes], (unsigned long long)bytes);
    if (qbytes) atomicAdd(&a.stats[kStQueue], (unsigned long long)qbytes);
    if (err) atomicOr(&a.stats[kStErr], (unsigned long long)kErrTimeOverflow);
  }
}

// ---------------------------------------------------------------------------------------------
// Longest-processing-time-first dispatch order for the next k_sim: sources bucketed by
// log2(HTB records emitted this step), heaviest bucket first (one workgroup, LDS counting sort).
// Only the dispatch order changes; every source's result is independent of it.
__global__ __launch_bounds__(1024) void k_order(const uint32_t* emit_n, uint32_t n, uint32_t* order) {
  __shared__ uint32_t cnt[33], base[33];
  for (uint32_t i = threadIdx.x; i < 33; i += blockDim.x) cnt[i] = 0;
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < n; s += blockDim.x) atomicAdd(&cnt[__clz(emit_n[s])], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int b = 0; b < 33; ++b) {
      base[b] = acc;
      acc += cnt[b];
    }
  }
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < n; s += blockDim.x) {
    const uint32_t b = __clz(emit_n[s]);
    order[atomicAdd(&base[b], 1u)] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// K9: configuration apply.
__global__ void k_apply_cfg(const CfgPatch* __restrict__ patches, uint32_t n, SrcParams* params,
                            SrcState* state) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const CfgPatch c = patches[i];
  params[c.s] = c.p;
  SrcState st = state[c.s];
  if (c.mask & 1u) st.last_dup = c.last_dup;
  if (c.mask & 2u) st.last_cor = c.last_cor;
  if (c.mask & 4u) st.last_reo = c.last_reo;
  if (c.mask & 8u) st.tat = 0;
  state[c.s] = st;
}

// ---------------------------------------------------------------------------------------------
// Storm traffic generator.
struct GenArgs {
  uint32_t tab[16];
  uint32_t k0, k1, n_src, shard_begin, n_peers, n_ticks;
  uint64_t now_tick;
};

__device__ __forceinline__ uint32_t poisson_count(const GenArgs& g, uint32_t u) {
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) c += (u >= g.tab[k]) && (c == (uint32_t)k);
  return c;
}

__global__ void k_gen_count(GenArgs g, uint64_t* counts) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.n_src) return;
  const uint32_t src = g.shard_begin + s;
  uint64_t total = 0;
  if (g.n_peers >= 2) {
    for (uint32_t t = 0; t < g.n_ticks; ++t) {
      uint32_t r[4];
      philox(src, (uint32_t)(g.now_tick + t), 0x53544F52u, 0, g.k0, g.k1, r);
      total += poisson_count(g, r[0]);
    }
  }
  counts[s] = total;
}

__global__ void k_gen_write(GenArgs g, const uint64_t* off, uint32_t* gen_seq, InRec* out) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.n_src || g.n_peers < 2) return;
  const uint32_t src = g.shard_begin + s;
  uint64_t o = off[s];
  uint32_t seq = gen_seq[s];
  for (uint32_t t = 0; t < g.n_ticks; ++t) {
    const uint32_t at = (uint32_t)(g.now_tick + t);
    uint32_t r[4];
    philox(src, at, 0x53544F52u, 0, g.k0, g.k1, r);
    const uint32_t cnt = poisson_count(g, r[0]);
    for (uint32_t j = 0; j < cnt; ++j) {
      uint32_t q[4];
      philox(src, at, 0x53544F52u, j + 1, g.k0, g.k1, q);
      uint32_t d = q[0] % (g.n_peers - 1);
      d += d >= src;
      InRec rec;
      rec.dst = d;
      rec.seq = seq++;
      rec.tick = t;
      rec.len = 64u + q[1] % 1437u;
      out[o++] = rec;
    }
  }
  gen_seq[s] = seq;
}

// ---------------------------------------------------------------------------------------------
// Gossip flood workload (C4): receipts are folded into a per-(peer, flood) earliest-receipt tick
// at delivery; each window emits, per peer, the floods first received in it, earliest first.
__device__ __forceinline__ uint32_t gossip_neighbour(const GossipArgs& g, uint32_t peer, uint32_t k) {
  uint32_t r[4];
  philox(peer, k, 0x474F5350u, 0, g.k0, g.k1, r);
  const uint32_t d = r[0] % (g.n_peers - 1);
  return d + (d >= peer);
}

__global__ void k_gossip_recv(GossipArgs g, const tgsim_delivery* in, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const tgsim_delivery r = in[i];
  const uint32_t f = r.seq / g.degree;
  if (f >= g.n_floods || (r.flags & TGSIM_FLAG_CORRUPT)) return;
  const uint32_t s = r.dst - g.shard_begin;
  if (g.fwd[s] >> f & 1ull) return;
  uint64_t t = r.t_ns / g.tick_ns + 1;
  if (t > 0xFFFFFFFEull) t = 0xFFFFFFFEull;
  atomicMin(&g.first[(uint64_t)s * 64 + f], (uint32_t)t);
}

// Floods due in [win0, win0 + n_ticks) for local peer s, as a bitmask; flags late receipts.
__device__ __forceinline__ uint64_t gossip_due(const GossipArgs& g, uint32_t s) {
  const uint64_t done = g.fwd[s];
  const uint32_t* fs = g.first + (uint64_t)s * 64;
  uint64_t due = 0;
  for (uint32_t f = 0; f < g.n_floods; ++f) {
    const uint32_t t = fs[f];
    if ((done >> f & 1ull) || t == 0xFFFFFFFFu || (uint64_t)t >= g.win0 + g.n_ticks) continue;
    if ((uint64_t)t < g.win0) atomicOr(g.err, 1u);
    due |= 1ull << f;
  }
  return due;
}

__global__ void k_gossip_count(GossipArgs g, uint64_t* counts) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.n_src) return;
  counts[s] = (uint64_t)__popcll(gossip_due(g, s)) * g.degree;
}

__global__ void k_gossip_write(GossipArgs g, const uint64_t* off, InRec* out) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= g.n_src) return;
  uint64_t due = gossip_due(g, s);
  if (!due) return;
  g.fwd[s] |= due;
  const uint32_t src = g.shard_begin + s;
  const uint32_t* fs = g.first + (uint64_t)s * 64;
  uint64_t o = off[s];
  while (due) {  // earliest receipt first, ties by flood id (seq order within a tick)
    uint32_t best = __ffsll((unsigned long long)due) - 1, bt = fs[best];
    for (uint64_t m = due & (due - 1); m; m &= m - 1) {
      const uint32_t f = __ffsll((unsigned long long)m) - 1;
      if (fs[f] < bt) { best = f; bt = fs[f]; }
    }
    due &= ~(1ull << best);
    for (uint32_t k = 0; k < g.degree; ++k) {
      InRec rec;
      rec.dst = gossip_neighbour(g, src, k);
      rec.seq = best * g.degree + k;
      rec.tick = (uint32_t)(bt - g.win0);
      rec.len = g.msg_len;
      out[o++] = rec;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Exclusive scan (u64), three phases, 1024 elements per block.
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* sh, uint64_t& total) {
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  uint64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t lo = __shfl_up((uint32_t)x, o, 64), hi = __shfl_up((uint32_t)(x >> 32), o, 64);
    if (lane >= (uint32_t)o) x += ((uint64_t)hi << 32) | lo;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  if (t == 0) {
    uint64_t acc = 0;
    for (uint32_t i = 0; i < blockDim.x / 64; ++i) {
      const uint64_t s = sh[i];
      sh[i] = acc;
      acc += s;
    }
    sh[15] = acc;
  }
  __syncthreads();
  total = sh[15];
  const uint64_t r = x - v + sh[w];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void k_scan_local(const uint64_t* in, uint64_t* out, uint64_t n,
                                                    uint64_t* block_sums) {
  __shared__ uint64_t sh[16];
  const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
  uint64_t v[4], s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = base + i < n ? in[base + i] : 0;
    s += v[i];
  }
  uint64_t total;
  uint64_t pre = block_excl_scan(s, sh, total);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (base + i < n) out[base + i] = pre;
    pre += v[i];
  }
  if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_scan_sums(uint64_t* sums, uint64_t nb, uint64_t* total_out) {
  __shared__ uint64_t sh[16];
  uint64_t carry = 0;
  for (uint64_t base = 0; base < nb; base += 256) {
    const uint64_t i = base + threadIdx.x;
    const uint64_t v = i < nb ? sums[i] : 0;
    uint64_t total;
    const uint64_t pre = block_excl_scan(v, sh, total);
    if (i < nb) sums[i] = carry + pre;
    carry += total;
  }
  if (threadIdx.x == 0) *total_out = carry;
}

__global__ __launch_bounds__(256) void k_scan_add(uint64_t* out, uint64_t n, const uint64_t* sums) {
  const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
  const uint64_t add = sums[blockIdx.x];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (base + i < n) out[base + i] += add;
}

// ---------------------------------------------------------------------------------------------
// Route: group the emitted records by the destination shard, deterministically and without
// contended atomics: per (rank, source) counts -> one exclusive scan over [rank][source] -> every
// source writes its records of rank r at off[r * S + s] in emission order.
struct RouteArgs {
  const tgsim_delivery* emit;
  const uint32_t* emit_n;
  const uint64_t* off;           // CSR offsets of the step input: region base 2*off[s] + kHeapCap*s
  uint32_t n_src;
  uint32_t n_ranks;
  uint32_t bounds[9];
  uint64_t* cnt;                 // [n_ranks][n_src] records per (rank, source)
  const uint64_t* pos;           // exclusive scan of cnt
  tgsim_delivery* out;
};

__device__ __forceinline__ uint32_t rank_of(const RouteArgs& a, uint32_t dst) {
  uint32_t r = 0;
  for (uint32_t i = 1; i < a.n_ranks; ++i) r += dst >= a.bounds[i];
  return r;
}

__global__ __launch_bounds__(256) void k_route_count(RouteArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nw = gridDim.x * 4;
  for (uint32_t s = blockIdx.x * 4 + (threadIdx.x >> 6); s < a.n_src; s += nw) {
    const uint32_t n = a.emit_n[s];
    if (a.n_ranks == 1) {
      if (lane == 0) a.cnt[s] = n;
      continue;
    }
    const tgsim_delivery* base = a.emit + 2 * a.off[s] + (uint64_t)kHeapCap * s;
    uint32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
      const uint32_t i = i0 + lane;
      const uint32_t rk = i < n ? rank_of(a, base[i].dst) : 0xFFFFFFFFu;
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q) c[q] += __popcll(__ballot(rk == q));
    }
    if (lane < a.n_ranks) {
      uint32_t v = 0;
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q) v = lane == q ? c[q] : v;
      a.cnt[(size_t)lane * a.n_src + s] = v;
    }
  }
}

__global__ __launch_bounds__(256) void k_route_scatter(RouteArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nw = gridDim.x * 4;
  for (uint32_t s = blockIdx.x * 4 + (threadIdx.x >> 6); s < a.n_src; s += nw) {
    const uint32_t n = a.emit_n[s];
    const tgsim_delivery* base = a.emit + 2 * a.off[s] + (uint64_t)kHeapCap * s;
    uint64_t run[8];
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) run[q] = q < a.n_ranks ? a.pos[(size_t)q * a.n_src + s] : 0;
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
      const uint32_t i = i0 + lane;
      tgsim_delivery r;
      uint32_t rk = 0xFFFFFFFFu;
      if (i < n) {
        r = base[i];
        rk = rank_of(a, r.dst);
      }
      const uint64_t below = (1ull << lane) - 1;
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q) {
        const uint64_t m = __ballot(rk == q);
        if (rk == q) a.out[run[q] + __popcll(m & below)] = r;
        run[q] += __popcll(m);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Delivery: counting sort by destination, then per-destination ordering.
__global__ void k_dst_hist(const tgsim_delivery* in, uint64_t n, uint32_t dst_begin, uint64_t* cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  atomicAdd(reinterpret_cast<unsigned long long*>(&cnt[in[i].dst - dst_begin]), 1ull);
}

__global__ void k_dst_scatter(const tgsim_delivery* in, uint64_t n, uint32_t dst_begin,
                              const uint64_t* off, uint64_t* cursor, tgsim_delivery* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const tgsim_delivery r = in[i];
  const uint32_t d = r.dst - dst_begin;
  const uint64_t p = atomicAdd(reinterpret_cast<unsigned long long*>(&cursor[d]), 1ull);
  out[off[d] + p] = r;
}

struct SortKey {
  uint64_t t;
  uint64_t sq;   // src << 32 | seq
  uint32_t idx;  // (clone ? 0 : 1) << 31 | position in the segment
};

__device__ __forceinline__ bool key_lt(const SortKey& a, const SortKey& b) {
  if (a.t != b.t) return a.t < b.t;
  if (a.sq != b.sq) return a.sq < b.sq;
  return a.idx < b.idx;
}

__device__ __forceinline__ SortKey make_key(const tgsim_delivery& r, uint32_t i) {
  SortKey k;
  k.t = r.t_ns;
  k.sq = ((uint64_t)r.src << 32) | r.seq;
  k.idx = ((r.flags & TGSIM_FLAG_DUP) ? 0u : 0x80000000u) | i;
  return k;
}

constexpr uint32_t kSegLds = 2048;

// One workgroup per destination segment: bitonic sort of (t, src, seq, clone-first) keys in LDS
// (global scratch for segments longer than kSegLds), then a gather into delivery order.
__global__ __launch_bounds__(256) void k_dst_sort(const tgsim_delivery* in, const uint64_t* off,
                                                  const uint64_t* cnt, tgsim_delivery* out,
                                                  SortKey* scratch) {
  __shared__ SortKey sk[kSegLds];
  const uint32_t d = blockIdx.x;
  const uint64_t b = off[d];
  const uint32_t n = (uint32_t)cnt[d];
  if (n == 0) return;
  if (n == 1) {
    if (threadIdx.x == 0) out[b] = in[b];
    return;
  }
  uint32_t P = 1;
  while (P < n) P <<= 1;
  SortKey* k = P <= kSegLds ? sk : scratch + 2 * b;  // P < 2n: disjoint per segment
  for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
    if (i < n) {
      k[i] = make_key(in[b + i], i);
    } else {
      k[i].t = ~0ull;
      k[i].sq = ~0ull;
      k[i].idx = 0xFFFFFFFFu;
    }
  }
  __syncthreads();
  for (uint32_t size = 2; size <= P; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
        const uint32_t j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const SortKey x = k[i], y = k[j];
          if (key_lt(y, x) == up) {
            k[i] = y;
            k[j] = x;
          }
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) out[b + i] = in[b + (k[i].idx & 0x7FFFFFFFu)];
}

// ---------------------------------------------------------------------------------------------
// Host-side launchers.
void launch_sim(const SimArgs& a, uint32_t n_wg, hipStream_t st) {
  hipLaunchKernelGGL(k_sim, dim3(n_wg), dim3(kWave), 0, st, a);  // n_wg = ceil(n_src / kSpw)
}

void launch_order(const uint32_t* emit_n, uint32_t n, uint32_t* order, hipStream_t st) {
  hipLaunchKernelGGL(k_order, dim3(1), dim3(1024), 0, st, emit_n, n, order);
}

void launch_apply_cfg(const CfgPatch* p, uint32_t n, SrcParams* params, SrcState* state, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_apply_cfg, dim3((n + 255) / 256), dim3(256), 0, st, p, n, params, state);
}

void launch_gen(const GenArgsHost& h, uint64_t* counts, const uint64_t* off, uint32_t* gen_seq,
                InRec* out, int phase, hipStream_t st) {
  GenArgs g;
  for (int i = 0; i < 16; ++i) g.tab[i] = h.tab[i];
  g.k0 = h.k0; g.k1 = h.k1; g.n_src = h.n_src; g.shard_begin = h.shard_begin;
  g.n_peers = h.n_peers; g.n_ticks = h.n_ticks; g.now_tick = h.now_tick;
  const dim3 grid((h.n_src + 63) / 64), blk(64);
  if (phase == 0) hipLaunchKernelGGL(k_gen_count, grid, blk, 0, st, g, counts);
  else hipLaunchKernelGGL(k_gen_write, grid, blk, 0, st, g, off, gen_seq, out);
}

void launch_gossip(const GossipArgs& g, const tgsim_delivery* recs, uint64_t n, uint64_t* counts,
                   const uint64_t* off, InRec* out, int phase, hipStream_t st) {
  if (phase == 0) {
    if (n) hipLaunchKernelGGL(k_gossip_recv, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, g, recs, n);
    return;
  }
  const dim3 grid((g.n_src + 255) / 256), blk(256);
  if (phase == 1) hipLaunchKernelGGL(k_gossip_count, grid, blk, 0, st, g, counts);
  else hipLaunchKernelGGL(k_gossip_write, grid, blk, 0, st, g, off, out);
}

void launch_scan(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* block_sums,
                 uint64_t* total, hipStream_t st) {
  const uint64_t nb = (n + 1023) / 1024;
  if (nb == 0) {
    (void)hipMemsetAsync(total, 0, sizeof(uint64_t), st);
    return;
  }
  hipLaunchKernelGGL(k_scan_local, dim3((uint32_t)nb), dim3(256), 0, st, in, out, n, block_sums);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(256), 0, st, block_sums, nb, total);
  hipLaunchKernelGGL(k_scan_add, dim3((uint32_t)nb), dim3(256), 0, st, out, n, block_sums);
}

void launch_route(const RouteArgsHost& h, int phase, hipStream_t st) {
  RouteArgs a;
  a.emit = h.emit;
  a.emit_n = h.emit_n;
  a.off = h.off;
  a.n_src = h.n_src;
  a.n_ranks = h.n_ranks;
  for (int i = 0; i < 9; ++i) a.bounds[i] = h.bounds[i];
  a.cnt = h.cnt;
  a.pos = h.pos;
  a.out = h.out;
  uint32_t grid = (h.n_src + 3) / 4;
  if (grid > 4096) grid = 4096;
  if (grid == 0) grid = 1;
  if (phase == 0) hipLaunchKernelGGL(k_route_count, dim3(grid), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(k_route_scatter, dim3(grid), dim3(256), 0, st, a);
}

void launch_dst_hist(const tgsim_delivery* in, uint64_t n, uint32_t dst_begin, uint64_t* cnt, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_dst_hist, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, in, n, dst_begin, cnt);
}

void launch_dst_scatter(const tgsim_delivery* in, uint64_t n, uint32_t dst_begin, const uint64_t* off,
                        uint64_t* cursor, tgsim_delivery* out, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_dst_scatter, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, in, n,
                     dst_begin, off, cursor, out);
}

void launch_dst_sort(const tgsim_delivery* in, const uint64_t* off, const uint64_t* cnt, uint32_t n_dst,
                     tgsim_delivery* out, void* scratch, hipStream_t st) {
  if (!n_dst) return;
  hipLaunchKernelGGL(k_dst_sort, dim3(n_dst), dim3(256), 0, st, in, off, cnt, out,
                     reinterpret_cast<SortKey*>(scratch));
}

size_t sort_key_bytes() { return sizeof(SortKey); }

}  // namespace tgsim
