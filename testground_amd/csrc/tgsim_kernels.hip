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
#include <errno.h>
#include <stdlib.h>
#include "tgsim_launch.h"

namespace tgsim {

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 (Random123 constants).
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                       uint32_t k0, uint32_t k1, uint32_t r[4]) {
  // the round keys are derived from the key at every call (2 SALU per round): hoisted out of the
  // simulate loop they held 20 SGPRs and came back as spill reloads (v_readlane) at every draw
  __asm__ volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    // one v_mad_u64_u32 per product instead of a v_mul_hi_u32 + v_mul_lo_u32 pair
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
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

// ---------------------------------------------------------------------------------------------
// k_sim: one wavefront owns one source's netem queue for the whole step.
//
// The queue lives in LDS as ONE circular buffer of kHeapCap 16-B slots: the departure ring (items
// already given a departure time by HTB, d in .x/.y, oldest first), immediately followed by the
// eligibility queue (items waiting for their netem time e) in two regions: the NEAR region, kept
// SORTED by (e, seq, clone first), holds every item with e < B; the POOL behind it holds the items
// with e >= B in no order.  HTB serves the near region from its head, so serving an item turns the
// slot at the boundary into the ring's newest entry in place; the netem limit bounds
// ring + near + pool <= 1024.  A new item whose e >= B is appended to the pool (no search, no
// shift: with jitter or a long latency most items are far in the future); before anything needs
// the items eligible before h, `refill` raises B past h, moving the pool items below the new B
// into the near region (chosen so that at most 64 move at a time).
//
// The sequential recurrence of netem_enqueue (limit check) + HTB is resolved a WINDOW of offered
// packets at a time, wave-parallel:
//   1. the queue-head items that may become eligible before the batch's last packet are served
//      optimistically with a max-plus scan (TAT' = max(TAT + c, e - B + c));
//   2. every candidate counts the departures before its offer time (binary search over the ring
//      ++ the newly served items, both sorted by d);
//   3. the netem limit is a saturating counter x -> min(x + a, limit), whose prefix composition is
//      closed-form (prefix sum + prefix max), so all admission decisions come from two scans;
//   4. the window ends before the first packet whose offer time is after the eligibility time of
//      an item admitted earlier in the window (only then could the optimistic HTB service be
//      wrong): reordered (e = T) and near-zero-delay admissions split windows, nothing else does;
//   5. admitted items are merged into the sorted queue (binary search + tail shift).
// Sources with correlated draws (get_crandom, rho != 0) consume state in admission order and take
// the per-packet path built from the same wave-wide primitives.
template <uint32_t kCap>
struct SimLdsT {
  uint4 slot[kCap];         // circular: departure ring, then the eligibility queue (near, pool)
  uint32_t wcnt[kWheelB];   // the timing wheel's bucket counts while far items are parked
  uint32_t whdr[4];         // and its base id, control word, due items loaded (kept here, not in
                            // registers, from the window's start to its end)
};
static_assert(sizeof(SimLdsT<kHeapCap>) <= 65536, "simulate workgroup LDS");

constexpr uint32_t kFvPass = 0xFFu;

// Cross-lane guards (TGSIM_CHECK builds only): a readlane must name an active
// lane, and the DPP scans, wave shuffles and the sorted-count search read every lane, so they need
// the whole wave active.  Round 4's fault was exactly such a read inside a lane-divergent branch.
// A violation is counted in tg_exec_faults (read by tgsim_debug_exec_faults) and the first few are
// printed by the first active lane of the offending wave.
#ifdef TGSIM_CHECK
__device__ unsigned int tg_exec_faults;
__device__ unsigned int tg_exec_lines[8192];  // violations per source line (the first one printed)
__device__ __noinline__ void tg_exec_fault(const char* what, uint64_t exec, uint32_t l, int line) {
  const uint32_t me = __lane_id();
  if (me == (uint32_t)__builtin_ctzll(exec)) {
    atomicAdd(&tg_exec_faults, 1u);
    const unsigned int k = atomicAdd(&tg_exec_lines[(uint32_t)line & 8191u], 1u);
    if (k == 0u)
      printf("EXEC CHECK %s at line %d: exec %016llx lane %u (block %u)\n", what, line, (unsigned long long)exec, l,
             blockIdx.x);
    else if ((k & (k + 1u)) == 0u && k >= 0xFFFFu)  // 2^16, 2^17, ... violations at this line
      printf("EXEC CHECK line %d: %u violations\n", line, k + 1u);
  }
}
__device__ __forceinline__ void tg_full_exec(const char* what, int line) {
  const uint64_t x = __builtin_amdgcn_read_exec();
  if (x != ~0ull) tg_exec_fault(what, x, 64u, line);
}
__device__ __forceinline__ void tg_lane_live(const char* what, uint32_t l, int line) {
  const uint64_t x = __builtin_amdgcn_read_exec();
  if (l >= 64u || !(x >> l & 1ull)) tg_exec_fault(what, x, l, line);
}
#define TG_FULL_EXEC(what) tg_full_exec(what, __LINE__)
#define TG_FULL_EXEC_AT(what, line) tg_full_exec(what, line)
#define TG_LANE_LIVE_AT(what, l, line) tg_lane_live(what, l, line)
#else
#define TG_FULL_EXEC(what) ((void)0)
#define TG_FULL_EXEC_AT(what, line) ((void)(line))
#define TG_LANE_LIVE_AT(what, l, line) ((void)(line))
#endif
// (line: the caller's source line, for the check build's report)
__device__ __forceinline__ uint32_t readlane32(uint32_t v, uint32_t l, int line = __builtin_LINE()) {
  TG_LANE_LIVE_AT("readlane", l, line);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l, int line = __builtin_LINE()) {
  return ((uint64_t)readlane32((uint32_t)(v >> 32), l, line) << 32) | readlane32((uint32_t)v, l, line);
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src, int line = __builtin_LINE()) {
  TG_FULL_EXEC_AT("shfl64", line);
  const uint32_t lo = __shfl((uint32_t)v, (int)src, 64), hi = __shfl((uint32_t)(v >> 32), (int)src, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t ballot_count(bool p) { return (uint32_t)__popcll(__ballot(p)); }

// Inclusive wave scans (lane order = packet / queue order) on DPP: row_shr 1/2/4/8 inside each
// row of 16 lanes, then row_bcast:15 and row_bcast:31 carry the row totals (GFX9 wave64 pattern).
// Lanes without a source lane read the identity.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp(uint32_t id, uint32_t v, int line = __builtin_LINE()) {
  TG_FULL_EXEC_AT("dpp", line);
  return (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, CTRL, ROWS, 0xF, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp64(uint64_t id, uint64_t v, int line = __builtin_LINE()) {
  return ((uint64_t)dpp<CTRL, ROWS>((uint32_t)(id >> 32), (uint32_t)(v >> 32), line) << 32) |
         dpp<CTRL, ROWS>((uint32_t)id, (uint32_t)v, line);
}
#define TG_SCAN_STEPS(STEP) STEP(0x111, 0xF) STEP(0x112, 0xF) STEP(0x114, 0xF) STEP(0x118, 0xF) \
                            STEP(0x142, 0xA) STEP(0x143, 0xC)
constexpr int kDppWaveShr1 = 0x138;  // wave_shr:1 (lane i reads lane i - 1; lane 0 the identity)

// wave_shr:1 must stay a plain v_mov_b32_dpp: folded into a VOP2 ALU op (v_sub_u32_dpp ...
// wave_shr:1) it gave wrong results on gfx950, so the asm barrier keeps the DPP combiner off it.
__device__ __forceinline__ uint32_t shr1_u32(uint32_t v, uint32_t id, int line = __builtin_LINE()) {
  uint32_t r = dpp<kDppWaveShr1, 0xF>(id, v, line);
  __asm__ volatile("" : "+v"(r));
  return r;
}
__device__ __forceinline__ uint64_t shr1_u64(uint64_t v, uint64_t id, int line = __builtin_LINE()) {
  return ((uint64_t)shr1_u32((uint32_t)(v >> 32), (uint32_t)(id >> 32), line) << 32) |
         shr1_u32((uint32_t)v, (uint32_t)id, line);
}

__device__ __forceinline__ void scan_maxplus(uint64_t& a, uint64_t& b, int line = __builtin_LINE()) {
  // maps x -> max(x + a, b); earlier (pa, pb) then later (a, b) = (pa + a, max(pb + a, b))
#define STEP(C, R) { const uint64_t pa = dpp64<C, R>(0, a, line), pb = dpp64<C, R>(0, b, line); \
                     const uint64_t nb = pb + a; b = nb > b ? nb : b; a = pa + a; }
  TG_SCAN_STEPS(STEP)
#undef STEP
}
__device__ __forceinline__ int32_t scan_sum_i32(int32_t v, int line = __builtin_LINE()) {
#define STEP(C, R) v += (int32_t)dpp<C, R>(0u, (uint32_t)v, line);
  TG_SCAN_STEPS(STEP)
#undef STEP
  return v;
}
__device__ __forceinline__ int32_t scan_max_i32(int32_t v, int line = __builtin_LINE()) {
#define STEP(C, R) v = max(v, (int32_t)dpp<C, R>(0x80000000u, (uint32_t)v, line));
  TG_SCAN_STEPS(STEP)
#undef STEP
  return v;
}
__device__ __forceinline__ uint32_t scan_max_u32(uint32_t v, int line = __builtin_LINE()) {
#define STEP(C, R) v = max(v, dpp<C, R>(0u, v, line));
  TG_SCAN_STEPS(STEP)
#undef STEP
  return v;
}
__device__ __forceinline__ uint64_t scan_max_u64(uint64_t v, int line = __builtin_LINE()) {
#define STEP(C, R) { const uint64_t p = dpp64<C, R>(0ull, v, line); v = p > v ? p : v; }
  TG_SCAN_STEPS(STEP)
#undef STEP
  return v;
}
__device__ __forceinline__ uint64_t scan_min_u64(uint64_t v, int line = __builtin_LINE()) {
#define STEP(C, R) { const uint64_t p = dpp64<C, R>(~0ull, v, line); v = p < v ? p : v; }
  TG_SCAN_STEPS(STEP)
#undef STEP
  return v;
}

// Count of the 64 lane values v (sorted ascending over lanes) that are <= t, for every lane's t.
__device__ __forceinline__ uint32_t count_le_sorted_u32(uint32_t v, uint32_t t, int line = __builtin_LINE()) {
  TG_FULL_EXEC_AT("count_le_sorted", line);
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t s = 32; s; s >>= 1)
    if ((uint32_t)__shfl(v, (int)(lo + s - 1), 64) <= t) lo += s;
  return lo + ((uint32_t)__shfl(v, (int)lo, 64) <= t ? 1u : 0u);
}

// tabledist() uniform branch: e = T + max(0, L - sigma + raw mod 2 sigma), or T + L when sigma = 0.
__device__ __forceinline__ uint64_t delayed(const SrcParams& p, uint64_t T, uint32_t raw) {
  if (p.sigma == 0) return T + p.lat_ns;
  const uint32_t m = 2u * (uint32_t)p.sigma;
  const int64_t delay = (int64_t)(raw % m) + (int64_t)p.lat_ns - (int64_t)p.sigma;
  return delay > 0 ? T + (uint64_t)delay : T;
}

// Gossip receipt of one emitted record (single shard; what k_gossip_recv does at delivery): the
// earliest receipt tick of flood seq / degree at the destination, which becomes pending unless it
// has forwarded the flood already (fw: the destination's forwarded mask).  Receipts are order-free
// (the earliest tick wins), so folding them in at emission changes no result.  Only destinations
// of this shard are folded in; the others' receipts are taken where their records are delivered
// (k_gossip_recv_in).
struct RecvFold {
  uint32_t* first;
  uint64_t* pend;
  const uint64_t* fwd;
  uint32_t floods, degree, shard_begin, n_local;
  uint64_t tick_ns;
  double inv_tick;
};
__device__ __forceinline__ RecvFold recv_fold(const SimArgs& a) {
  return RecvFold{a.g_first, a.g_pend,  a.g_fwd,   a.g_floods,
                  a.g_degree, a.shard_begin, a.n_src, a.tick_ns, 1.0 / (double)a.tick_ns};
}
__device__ __forceinline__ void fold_receipt(const RecvFold& g, uint32_t dst, uint32_t seq, uint32_t flags, uint64_t d,
                                             uint64_t fw) {
  const uint32_t f = seq / g.degree, s = dst - g.shard_begin;
  if (s >= g.n_local || f >= g.floods || (flags & TGSIM_FLAG_CORRUPT) || (fw >> f & 1ull)) return;
  // t = d / tick + 1 without a 64-bit division: d < 2^46 is exact in a double, and the estimate is
  // off by at most one
  uint64_t q = (uint64_t)((double)d * g.inv_tick);
  const int64_t r = (int64_t)(d - q * g.tick_ns);
  q = r < 0 ? q - 1 : (uint64_t)r >= g.tick_ns ? q + 1 : q;
  uint64_t t = q + 1;
  if (t > 0xFFFFFFFEull) t = 0xFFFFFFFEull;
  // the first receipt ever (exactly one sees "none") marks the flood pending: one atomic per receipt
  // and one per (peer, flood), not two per receipt (every one a memory-side request)
  if (__hip_atomic_fetch_min(&g.first[(uint64_t)s * 64 + f], (uint32_t)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
      0xFFFFFFFFu)
    __hip_atomic_fetch_or(&g.pend[s], 1ull << f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Emit slots of one source in one window (SimArgs::emit_r): the first cap in its region,
// the rest claimed from the window's pool.  A claim the pool cannot hold raises kErrEmitPool (-ENOSPC
// at the next call) and the records past cap are dropped (over stays null).
struct EmitOut {
  tgsim_delivery* region;
  tgsim_delivery* over;
  uint32_t cap;
  __device__ __forceinline__ bool fits(uint32_t i) const { return i < cap || over != nullptr; }
  __device__ __forceinline__ tgsim_delivery* at(uint32_t i) const { return i < cap ? region + i : over + (i - cap); }
};
__device__ __forceinline__ EmitOut emit_out(const SimArgs& a, uint32_t s, uint64_t sbeg, uint64_t send) {
  EmitOut o;
  o.region = a.emit + 2 * sbeg + (uint64_t)a.emit_r * s;
  o.over = nullptr;
  o.cap = (uint32_t)(2 * (send - sbeg)) + a.emit_r;
  return o;
}
// For up to `total` records: what exceeds the region comes from the pool, one atomic (lane 0; the
// caller is wave-uniform).  The classic layout (emit_r = kHeapCap) never needs it.
__device__ __forceinline__ void emit_claim(const SimArgs& a, uint32_t s, EmitOut& o, uint32_t total, uint32_t lane) {
  if (total <= o.cap) return;
  const uint32_t need = total - o.cap;
  uint32_t at = 0;
  if (lane == 0) at = atomicAdd(a.worklist - 2, need);
  at = (uint32_t)__builtin_amdgcn_readfirstlane((int)at);
  if ((uint64_t)at + need <= a.emit_pool_cap) {
    o.over = a.emit_pool + at;
    if (lane == 0) a.emit_pool_idx[s] = at;
  } else if (lane == 0) {
    atomicOr(&a.stats[kStErr], (unsigned long long)kErrEmitPool);
    if (a.err_host) __hip_atomic_store(a.err_host, (uint64_t)kErrEmitPool, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
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

__device__ __forceinline__ uint64_t wave_sum(uint64_t v, int line = __builtin_LINE()) {
  TG_FULL_EXEC_AT("wave_sum", line);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)v, o, 64);
    const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// Cross-lane LDS hand-off inside the single-wavefront workgroup: this wave's LDS operations have
// landed (lgkmcnt(0)); no vmcnt drain of the outstanding global stores and prefetch loads.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt(63) expcnt(7) lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  __asm__ volatile("" ::: "memory");
}

__device__ __forceinline__ void stamp(const SimArgs& a, uint32_t wg, uint32_t lane, uint32_t k, uint64_t v) {
  if (a.stamps && lane == 0) a.stamps[(size_t)wg * kStampSlots + k] = v;
}

#ifdef TGSIM_PROFILE
#define PROF_T0(n) const uint64_t _pt##n = __builtin_amdgcn_s_memtime()
#define PROF_ADD(k, n) (pf[k] += __builtin_amdgcn_s_memtime() - _pt##n)
#define PROF_CNT(k, v) (pf[k] += (v))
#else
#define PROF_T0(n) do {} while (0)
#define PROF_ADD(k, n) do {} while (0)
#define PROF_CNT(k, v) do {} while (0)
#endif

// Wave-uniform queue state of the source plus the helpers that operate on it.  Every member is
// identical in all 64 lanes; per-lane scratch is passed in and out.
// Bitonic sort of one item per lane across the wave (ascending by item_lt; lanes without an
// item, has = false, sort behind every item): 21 compare-exchange stages.  Partner lane lane ^ J:
// DPP quad_perm for J = 1, 2, ds_swizzle (xor mode, within 32 lanes) for J = 4..16, a
// ds_bpermute for J = 32.
template <uint32_t J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
  TG_FULL_EXEC("xor_lane");
  uint32_t r;
  if constexpr (J == 1) r = dpp<0xB1, 0xF>(0u, v, __LINE__);       // quad_perm [1, 0, 3, 2]
  else if constexpr (J == 2) r = dpp<0x4E, 0xF>(0u, v, __LINE__);  // quad_perm [2, 3, 0, 1]
  else if constexpr (J < 32) r = (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (int)(0x1Fu | (J << 10)));
  else r = (uint32_t)__shfl_xor((int)v, 32, 64);
  __asm__ volatile("" : "+v"(r));  // keep the DPP moves plain (see shr1_u32)
  return r;
}
template <uint32_t K, uint32_t J>
__device__ __forceinline__ void sort_stage(uint4& v, uint32_t& vf, uint32_t lane) {
  const uint4 pv = make_uint4(xor_lane<J>(v.x), xor_lane<J>(v.y), xor_lane<J>(v.z), xor_lane<J>(v.w));
  const uint32_t pf = xor_lane<J>(vf);
  const bool m_lt = vf < pf || (vf == pf && item_lt(v, pv));  // mine < partner's
  const bool keep_min = ((lane & J) == 0) == ((lane & K) == 0);
  if (keep_min != m_lt) {  // take the partner's item
    v = pv;
    vf = pf;
  }
  if constexpr (J > 1) sort_stage<K, J / 2>(v, vf, lane);
}
template <uint32_t K>
__device__ __forceinline__ void sort_merge(uint4& v, uint32_t& vf, uint32_t lane) {
  sort_stage<K, K / 2>(v, vf, lane);
  if constexpr (K < kWave) sort_merge<K * 2>(v, vf, lane);
}
__device__ __forceinline__ void wave_sort_items(uint4& v, bool has, uint32_t lane) {
  uint32_t vf = has ? 0u : 1u;
  sort_merge<2>(v, vf, lane);
}

// kOver: the records may run past the source's region into the emit pool (k_sim_list of a sparse
// window in the compact layout: over/cap set by the caller); otherwise emit + n_emit, classic layout.
template <uint32_t kCap, bool kOver = false>
struct SimQueue {
  static constexpr uint32_t kSlotMask = kCap - 1;
  SimLdsT<kCap>& lds;
  const SrcParams& p;
  uint32_t lane;
  uint32_t rh, rn, qn, pn;  // ring head slot, ring length, near-region length, soon-pool length
  uint32_t fn;              // far-pool length (behind the soon pool)
  uint32_t pk;              // far items parked in the timing wheel (not in LDS; all >= H)
  uint32_t rpush;           // entries appended to the ring this window (the ones written back)
  uint64_t B;               // near/pool boundary: near items have e < B, pool items e >= B
  uint64_t H;               // the step's horizon: every serve is before it; soon items e < H <= far
  uint64_t tat;             // HTB theoretical arrival time
  tgsim_delivery* emit;
  tgsim_delivery* over;      // kOver: records from cap on (null: the pool could not take them, dropped)
  uint32_t cap;              // kOver: records that fit in the source's region
  unsigned long long* dcnt;  // per-destination histogram (single shard) or null
  bool dslot;                // kOver: the records carry their destination slot (SimArgs::dst_slot)
  tgsim_delivery* bkt;       // kOver: the destinations' buckets (SimArgs::dst_bkt), or null
  uint32_t bkt_log;
  RecvFold rf;               // gossip receipts folded in at emission (rf.first null: none)
  uint32_t n_emit, src;
  // per-lane accumulators (summed over the wave at the end)
  uint32_t sched, corrupted, lost;
  uint64_t bytes;
#ifdef TGSIM_PROFILE
  uint64_t pf[24];
#endif

  __device__ __forceinline__ uint4& slot(uint32_t k) { return lds.slot[(rh + k) & kSlotMask]; }
  __device__ __forceinline__ uint64_t ring_d(uint32_t k) {
    const uint2 v = *reinterpret_cast<const uint2*>(&lds.slot[(rh + k) & kSlotMask]);
    return ((uint64_t)v.y << 32) | v.x;
  }

#ifdef TGSIM_CHECK
  // Debug: near < B <= soon < H <= far and B <= far (B may pass H when there are no soon items), near
  // sorted; prints the first violation.
  __device__ void check(int tag) {
    uint32_t bad = 0;
    uint64_t be = 0;
    for (uint32_t k = lane; k < qn; k += kWave) {
      const uint64_t e = w0_of(slot(rn + k)) & kEMask;
      if (e >= B) { bad |= 1; be = e; }
      if (k + 1 < qn && item_lt(slot(rn + k + 1), slot(rn + k))) bad |= 2;
    }
    for (uint32_t k = lane; k < pn; k += kWave) {
      const uint64_t e = w0_of(slot(rn + qn + k)) & kEMask;
      if (e < B || e >= H) { bad |= 4; be = e; }
    }
    for (uint32_t k = lane; k < fn; k += kWave) {
      const uint64_t e = w0_of(slot(rn + qn + pn + k)) & kEMask;
      if (e < H || e < B) { bad |= 8 | (k << 8); be = e; }
    }
    // (B > H is fine without soon items: the sparse FIFO path stores a whole sorted queue as the
    // near region, due prefix served, the rest after H, and every item behind it is >= B)
    if (B > H && pn) bad |= 16;
    const uint64_t m = __ballot(bad != 0);
    if (m) {
      const uint32_t l = (uint32_t)__builtin_ctzll(m);
      const uint32_t bb = readlane32(bad, l);
      const uint64_t ee = readlane64(be, l);
      if (lane == 0)
        printf("CHECK tag %d src %u rn %u qn %u pn %u fn %u B %llu H %llu bad %x e %llu lanes %llx\n", tag, src, rn, qn,
               pn, fn, (unsigned long long)B, (unsigned long long)H, bb, (unsigned long long)ee, (unsigned long long)m);
    }
  }
#define QCHECK(t) Q.check(t)
#else
#define QCHECK(t) do {} while (0)
#endif

  // HTB departure times of the queue-head items held one per lane (in = lane < n, e/len of the
  // lane's item): d = max(e, TAT_before), and the TAT after each item.
  __device__ __forceinline__ void htb_scan(bool in, uint64_t e, uint32_t len, uint64_t& d,
                                           uint64_t& tat_after) const {
    const uint64_t c = ((uint64_t)len * p.mult) >> (p.shift_ext & 0xFFu);
    uint64_t A = in ? c : 0, B = in ? (e > p.burst_ns ? e - p.burst_ns : 0) + c : 0;
    scan_maxplus(A, B);
    const uint64_t ta = tat + A;
    tat_after = ta > B ? ta : B;
    const uint64_t before = shr1_u64(tat_after, tat);
    d = e > before ? e : before;
  }

  // Commits the HTB service of the first n queue items (lanes < n): slot -> ring entry, record.
  // An item whose destination went away while it was queued (kDeadDst, k_purge) still takes its
  // HTB turn and its place in the ring (it leaves the sender) but emits no record.
  __device__ __forceinline__ void commit(bool c, uint32_t n, const uint4& qi, uint64_t d, uint64_t tat_after) {
    if constexpr (kOver) commit_over(c, n, qi, d, tat_after);
    else commit_plain(c, n, qi, d, tat_after);
  }
  // records past the region with no pool space are dropped (kErrEmitPool)
  // (as emit_record: the destination slot first, then the bucket or the emit records)
  __device__ __forceinline__ void commit_over(bool c, uint32_t n, const uint4& qi, uint64_t d, uint64_t tat_after) {
    const bool live = c && qi.w != kDeadDst;
    unsigned long long rank = 0;
    if (live && dcnt) {
      if (dslot) rank = atomicAdd(&dcnt[qi.w], 1ull);
      else atomicAdd(&dcnt[qi.w], 1ull);
    }
    const bool inb = live && bkt != nullptr && rank < (1ull << bkt_log);
    bool ov = live && !inb;
    const uint32_t ri = n_emit + (uint32_t)__popcll(__ballot(ov) & ((1ull << lane) - 1));
    ov = ov && (ri < cap || over != nullptr);
    const uint64_t lm = __ballot(ov);
    if (c) {
      *reinterpret_cast<uint2*>(&slot(rn + lane)) = make_uint2((uint32_t)d, (uint32_t)(d >> 32));
      if (inb || ov) {
        const uint32_t len = qi.y >> 14 & 0xFFFFu, flags = qi.y >> 30;
        uint64_t* rw = reinterpret_cast<uint64_t*>(inb ? bkt + ((uint64_t)qi.w << bkt_log) + rank
                                                       : ri >= cap ? over + (ri - cap) : emit + ri);
        rw[1] = ((uint64_t)qi.w << 32) | src;
        rw[2] = ((uint64_t)flags << 48) | ((uint64_t)len << 32) | qi.z;
        rw[0] = inb || !dslot ? d : d | slot_bits(rank);
        if (rf.first && qi.w - rf.shard_begin < rf.n_local)
          fold_receipt(rf, qi.w, qi.z, flags, d, rf.fwd[qi.w - rf.shard_begin]);
        sched++;
        bytes += len;
        corrupted += (flags >> 1) & 1u;
      } else {
        lost++;
      }
    }
    tat = readlane64(tat_after, n - 1);
    rn += n;
    rpush += n;
    qn -= n;
    n_emit += (uint32_t)__popcll(lm);
    wave_lds_sync();
  }
  __device__ __forceinline__ void commit_plain(bool c, uint32_t n, const uint4& qi, uint64_t d, uint64_t tat_after) {
    const bool live = c && qi.w != kDeadDst;
    const uint64_t lm = __ballot(live);
    if (c) {
      *reinterpret_cast<uint2*>(&slot(rn + lane)) = make_uint2((uint32_t)d, (uint32_t)(d >> 32));
      if (live) {
        const uint32_t len = qi.y >> 14 & 0xFFFFu, flags = qi.y >> 30;
        uint64_t* rw = reinterpret_cast<uint64_t*>(emit + n_emit + __popcll(lm & ((1ull << lane) - 1)));
        rw[0] = d;
        rw[1] = ((uint64_t)qi.w << 32) | src;
        rw[2] = ((uint64_t)flags << 48) | ((uint64_t)len << 32) | qi.z;
        if (dcnt) atomicAdd(&dcnt[qi.w], 1ull);
        if (rf.first && qi.w - rf.shard_begin < rf.n_local)
          fold_receipt(rf, qi.w, qi.z, flags, d, rf.fwd[qi.w - rf.shard_begin]);
        sched++;
        bytes += len;
        corrupted += (flags >> 1) & 1u;
      } else {
        lost++;
      }
    }
    tat = readlane64(tat_after, n - 1);
    rn += n;
    rpush += n;
    qn -= n;
    n_emit += (uint32_t)__popcll(lm);
    wave_lds_sync();
  }

  // HTB serves every queued item eligible before h (e < h), in (e, seq, clone first) order.
  __device__ __forceinline__ void serve_until(uint64_t h) {
    refill(h);
    for (;;) {
      const bool hq = lane < qn;
      const uint4 qi = hq ? slot(rn + lane) : make_uint4(0, 0, 0, 0);
      const uint64_t qe = hq ? (w0_of(qi) & kEMask) : ~0ull;
      const bool in = qe < h;
      const uint32_t n = ballot_count(in);
      if (!n) break;
      uint64_t d, ta;
      htb_scan(in, qe, qi.y >> 14 & 0xFFFFu, d, ta);
      commit(in, n, qi, d, ta);
      if (n < kWave) break;
    }
  }

  // Items whose departure time is before T leave the netem queue.
  __device__ __forceinline__ void depart_before(uint64_t T) {
    for (;;) {
      const uint64_t dep = lane < rn ? ring_d(lane) : ~0ull;
      const uint64_t stop = __ballot(dep >= T);  // released from the head while head < T
      const uint32_t k = stop ? (uint32_t)__builtin_ctzll(stop) : kWave;
      rh = (rh + k) & kSlotMask;
      rn -= k;
      if (k < kWave) break;
    }
  }

  // New items of the lanes (has): into the near region when eligible before B, else appended to
  // the pool: the SOON part when eligible before the step's horizon H (refill may need them), the
  // FAR part behind it otherwise (never needed in this step, so refill never scans them).
  __device__ __forceinline__ void insert(bool has, const uint4& it) {
    const uint64_t e = w0_of(it) & kEMask;
    const bool pool = has && e >= B;
    insert_near(has && !pool, it, true);
    append_pool(pool, it);
  }
  // Pool items of the lanes (pool: every one >= B) appended to the soon or the far part.
  __device__ __forceinline__ void append_pool(bool pool, const uint4& it) {
    const uint64_t e = w0_of(it) & kEMask;
    const bool vfar = pool && e >= H;
    const uint64_t ms = __ballot(pool && !vfar), mf = __ballot(vfar);
    if (!(ms | mf)) return;
    const uint64_t below = (1ull << lane) - 1;
    const uint32_t ks = (uint32_t)__popcll(ms);
    relocate_far(ks);  // ks free slots behind the soon part
    if (pool && !vfar) slot(rn + qn + pn + (uint32_t)__popcll(ms & below)) = it;
    pn += ks;
    if (vfar) slot(rn + qn + pn + fn + (uint32_t)__popcll(mf & below)) = it;
    fn += (uint32_t)__popcll(mf);
    PROF_CNT(19, (uint32_t)__popcll(ms | mf));
    wave_lds_sync();
  }

  // k free slots right behind the soon pool: the first min(k, fn) far items move behind the far
  // pool (it has no order).
  __device__ __forceinline__ void relocate_far(uint32_t k) {
    const uint32_t mv = k < fn ? k : fn, off = k > fn ? k : fn;
    if (!mv) return;
    const uint32_t b = rn + qn + pn;
    const bool l = lane < mv;
    const uint4 v = l ? slot(b + lane) : make_uint4(0, 0, 0, 0);
    __asm__ volatile("" ::: "memory");
    if (l) slot(b + off + lane) = v;
    __asm__ volatile("" ::: "memory");
  }

  // The near region grows by k at its end: k slots open behind the soon pool (relocate_far), then
  // the first min(k, pn) soon items move into them (no order either), so the near suffix can
  // shift up into their slots.
  __device__ __forceinline__ void relocate_pool(uint32_t k) {
    relocate_far(k);
    const uint32_t mv = k < pn ? k : pn, off = k > pn ? k : pn;
    if (!mv) return;
    const bool l = lane < mv;
    const uint4 v = l ? slot(rn + qn + lane) : make_uint4(0, 0, 0, 0);
    __asm__ volatile("" ::: "memory");
    if (l) slot(rn + qn + off + lane) = v;
    __asm__ volatile("" ::: "memory");
  }

  // Raises B to at least h: every pool item eligible before h joins the near region.  The new B
  // is the largest candidate h + d_c whose pool items number at most 64 (one count pass, eleven
  // thresholds); those are taken out of the pool (the pool's first slots refill the holes they
  // leave, so the pool then starts right behind them) and merged into the near region, where they
  // land at its end: every pool item is >= B > every near item.  More than 64 pool items below h
  // itself take several rounds.
  __device__ __forceinline__ void refill(uint64_t h) {
    if (!(pn && B < h)) return;
    PROF_T0(rf);
    while (pn && B < h) {
      PROF_CNT(17, 1);
      constexpr int kCand = 11;
      uint32_t cnt[kCand];
#pragma unroll
      for (int c = 0; c < kCand; ++c) cnt[c] = 0;
      PROF_T0(rc);
      for (uint32_t base = 0; base < pn; base += kWave) {
        const uint32_t k = base + lane;
        const uint64_t e = k < pn ? (ring_d(rn + qn + k) & kEMask) : ~0ull;
#pragma unroll
        for (int c = 0; c < kCand; ++c) cnt[c] += ballot_count(e < h + (c ? (4096ull << c) : 0ull));
      }
      PROF_ADD(20, rc);
      uint64_t Bp = h;
      uint32_t total = cnt[0];
#pragma unroll
      for (int c = 1; c < kCand; ++c)
        if (cnt[c] <= kWave) {  // counts grow with c: the last that fits
          Bp = h + (4096ull << c);
          total = cnt[c];
        }
      if (Bp > H) Bp = H;  // far items are >= H; the soon items (all < H) counted below Bp stay the same
      if (!total) {
        B = Bp;
        break;
      }
      const uint32_t nx = total < kWave ? total : kWave;
      const uint64_t below = (1ull << lane) - 1;
      uint4 xv = make_uint4(0, 0, 0, 0), av = make_uint4(0, 0, 0, 0);
      uint32_t gx = 0, gh = 0;  // items taken so far, holes refilled so far
      PROF_T0(rt);
      for (uint32_t base = 0; gx < nx; base += kWave) {
        const uint32_t k = base + lane;
        const bool in = k < pn;
        const uint4 v = in ? slot(rn + qn + k) : make_uint4(0, 0, 0, 0);
        const bool ex0 = in && (w0_of(v) & kEMask) < Bp;
        const uint32_t rx = gx + (uint32_t)__popcll(__ballot(ex0) & below);
        const bool ex = ex0 && rx < nx;  // the first nx by position
        const uint64_t mex = __ballot(ex);
        const uint32_t cx = (uint32_t)__popcll(mex);
        {  // taken items to lanes [gx, gx + cx) (forward permute; the others fill the rest)
          const uint32_t to = (ex ? rx : gx + cx + (uint32_t)__popcll(~mex & below)) & (kWave - 1);
          TG_FULL_EXEC("ds_permute");
          const uint4 pv = make_uint4((uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.x),
                                      (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.y),
                                      (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.z),
                                      (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.w));
          if (lane >= gx && lane < gx + cx) xv = pv;
        }
        if (base == 0) {  // the items that stay but sit in the first nx slots, ranked, to lanes
          const bool st = in && k < nx && !ex;
          const uint64_t ma = __ballot(st);
          const uint32_t to = (st ? (uint32_t)__popcll(ma & below)
                                  : (uint32_t)__popcll(ma) + (uint32_t)__popcll(~ma & below)) & (kWave - 1);
          TG_FULL_EXEC("ds_permute");
          av = make_uint4((uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.x),
                          (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.y),
                          (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.z),
                          (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.w));
        }
        // slots the taken items leave behind the first nx receive those items, in rank order
        const bool hole = ex && k >= nx;
        const uint64_t mh = __ballot(hole);
        const uint32_t src = (gh + (uint32_t)__popcll(mh & below)) & (kWave - 1);
        TG_FULL_EXEC("ds_permute");
        const uint4 fill = make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)av.x),
                                      (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)av.y),
                                      (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)av.z),
                                      (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)av.w));
        if (hole) slot(rn + qn + k) = fill;
        gh += (uint32_t)__popcll(mh);
        gx += cx;
      }
      wave_lds_sync();
      PROF_ADD(21, rt);
      pn -= nx;  // the pool now starts nx slots further; those slots are free
      PROF_CNT(18, nx);
      // every pool item is >= B > every near item, so the taken items, sorted, extend the near
      // region into the nx free slots behind it; only when more than 64 pool items are below h
      // (B not raised) can a later round take items below those taken before: merged then
      PROF_T0(ri);
      wave_sort_items(xv, lane < nx, lane);
      const uint4 first = make_uint4(readlane32(xv.x, 0), readlane32(xv.y, 0), readlane32(xv.z, 0), 0u);
      if (qn == 0 || item_lt(slot(rn + qn - 1), first)) {
        if (lane < nx) slot(rn + qn + lane) = xv;
        qn += nx;
        wave_lds_sync();
        PROF_CNT(5, nx);
      } else {
        insert_near(lane < nx, xv, false);
      }
      PROF_ADD(22, ri);
      if (total <= kWave) B = Bp;
    }
    PROF_ADD(16, rf);
  }

  // Merges the lanes' new items (has) into the sorted near region: each item's position among
  // the queued items (lower bound of its key), its rank among the new items, then the queued items
  // from the first position on move up by the number of new items before them (after the pool
  // has made room behind the near region, when reloc; without it the slots behind the near region
  // are free).
  __device__ __forceinline__ void insert_near(bool has, const uint4& it, bool reloc) {
    const uint64_t m = __ballot(has);
    if (!m) return;
    PROF_T0(i);
    const uint32_t nm = (uint32_t)__popcll(m);
    uint32_t pos = 0;
    PROF_T0(q1);
    if (nm <= 8) {
      if (qn) {
        // two-level search, one item at a time: a sample every 16th queued key (one read per
        // lane), then the 15 keys between the two samples that bracket the item
        const uint4 last = slot(rn + qn - 1);
        const bool hs = 16 * lane < qn;
        const uint4 smp = hs ? slot(rn + 16 * lane) : make_uint4(0, 0, 0, 0);
        for (uint64_t mm = m; mm; mm &= mm - 1) {
          const uint32_t b = (uint32_t)__builtin_ctzll(mm);
          const uint4 k = make_uint4(readlane32(it.x, b), readlane32(it.y, b), readlane32(it.z, b), 0u);
          uint32_t p = qn;  // appended: the common case (e grows with the offer time)
          if (!item_lt(last, k)) {
            const uint32_t c = ballot_count(hs && item_lt(smp, k));
            p = 0;
            if (c) {
              const uint32_t base = 16 * (c - 1);
              const bool hb = lane >= 1 && lane < 16 && base + lane < qn;
              const uint4 blk = hb ? slot(rn + base + lane) : make_uint4(0, 0, 0, 0);
              p = base + 1 + ballot_count(hb && item_lt(blk, k));
            }
          }
          if (lane == b) pos = p;
        }
      }
    } else {
      if (has && qn) {
        if (item_lt(slot(rn + qn - 1), it)) {
          pos = qn;
        } else {
          uint32_t lo = 0, hi = qn - 1;
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (item_lt(slot(rn + mid), it)) lo = mid + 1;
            else hi = mid;
          }
          pos = lo;
        }
      }
    }
    PROF_ADD(14, q1);
    // rank among the new items (equal keys: lane order)
    uint32_t rank = 0;
    bool ranked = nm <= 1;
    if (nm > 2) {
      // common case (no jitter or reorder: e grows with the offer time): the items are already in
      // key order across the lanes, checked against each item's predecessor in one pass
      const uint64_t below = m & ((1ull << lane) - 1);
      const uint32_t prev = below ? 63u - (uint32_t)__builtin_clzll(below) : lane;
      TG_FULL_EXEC("ds_permute");
      const uint4 pk = make_uint4((uint32_t)__shfl(it.x, (int)prev, 64), (uint32_t)__shfl(it.y, (int)prev, 64),
                                  (uint32_t)__shfl(it.z, (int)prev, 64), 0u);
      if (!__ballot(has && below && !item_lt(pk, it))) {
        rank = (uint32_t)__popcll(below);
        ranked = true;
      }
    }
    if (!ranked) {
      for (uint64_t mm = m; mm; mm &= mm - 1) {
        const uint32_t b = (uint32_t)__builtin_ctzll(mm);
        const uint4 o = make_uint4(readlane32(it.x, b), readlane32(it.y, b), readlane32(it.z, b), 0u);
        rank += (has && (item_lt(o, it) || (!item_lt(it, o) && b < lane))) ? 1u : 0u;
      }
    }
    PROF_T0(q2);
    // lane r receives the position of the rank-r item through a forward permute (the LDS
    // crossbar, no LDS allocation); lanes without an item take ranks nm.., so every lane gets one
    const uint32_t to = has ? rank : nm + (uint32_t)__popcll(~m & ((1ull << lane) - 1));
    TG_FULL_EXEC("ds_permute");
    const uint32_t sp_all = (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)(has ? pos : 0xFFFFFFFFu));
    uint32_t kL = 0;  // new items placed by moving the ring and the queue prefix down
    if (nm <= 8) {
      const uint32_t sp = lane < nm ? sp_all : 0u;  // lane r: position of the rank-r item
      // Two-sided merge.  The first kL items (by key) go in by moving the departure ring and the
      // queue prefix [0, maxL) down into the free slots before the ring head, the others by
      // moving the suffix [minR, qn) up; kL minimizes the slots moved.  Items eligible at once
      // (delay 0, reorder) land at the head and cost only the ring.
      const uint32_t spm1 = shr1_u32(sp, 0u);
      const uint32_t pmv = reloc ? (nm - lane < pn ? nm - lane : pn) + (nm - lane < fn ? nm - lane : fn) : 0u;  // pool items moved aside
      const uint32_t cost = lane <= nm ? (lane > 0 ? rn + spm1 : 0u) + (lane < nm ? qn - sp + pmv : 0u) : 0xFFFFFFFFu;
      // without reloc (refill) the pool already starts nm slots behind the near region: the new
      // items must fill exactly those slots, so nothing moves down (kL = 0)
      uint32_t best = readlane32(cost, 0);
      for (uint32_t k = 1; reloc && k <= nm; ++k) {
        const uint32_t c = readlane32(cost, k);
        if (c < best) {
          best = c;
          kL = k;
        }
      }
      const int32_t maxL = kL ? (int32_t)readlane32(sp, kL - 1) : 0;
      const int32_t minR = kL < nm ? (int32_t)readlane32(sp, kL) : (int32_t)qn;
      if (reloc) relocate_pool(nm - kL);
      // suffix up: queue item j >= minR moves by #{rank >= kL with pos <= j}; passes of four
      // chunks from the tail down, all reads of a pass before its writes
      for (int32_t hi = (int32_t)qn; hi > minR; hi -= 4 * (int32_t)kWave) {
        uint4 v[4];
        int32_t r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          r[u] = hi - (u + 1) * (int32_t)kWave + (int32_t)lane;
          v[u] = r[u] >= minR ? slot(rn + (uint32_t)r[u]) : make_uint4(0, 0, 0, 0);
        }
        uint32_t sh[4] = {0, 0, 0, 0};
        for (uint32_t k = kL; k < nm; ++k) {
          const int32_t pb = (int32_t)readlane32(sp, k);
#pragma unroll
          for (int u = 0; u < 4; ++u) sh[u] += pb <= r[u] ? 1u : 0u;
        }
        __asm__ volatile("" ::: "memory");
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (r[u] >= minR) slot(rn + (uint32_t)r[u] + sh[u]) = v[u];
        PROF_CNT(6, 1);
      }
      // ring and prefix down: combined index c < rn + maxL moves by -kL (+ #{rank < kL with
      // pos <= j} for queue item j = c - rn); passes from the ring head up
      for (int32_t lo = 0; kL && lo < (int32_t)rn + maxL; lo += 4 * (int32_t)kWave) {
        uint4 v[4];
        int32_t c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          c[u] = lo + u * (int32_t)kWave + (int32_t)lane;
          v[u] = c[u] < (int32_t)rn + maxL ? slot((uint32_t)c[u]) : make_uint4(0, 0, 0, 0);
        }
        uint32_t sh[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < kL; ++k) {
          const int32_t pb = (int32_t)readlane32(sp, k) + (int32_t)rn;
#pragma unroll
          for (int u = 0; u < 4; ++u) sh[u] += (c[u] >= (int32_t)rn && pb <= c[u]) ? 1u : 0u;
        }
        __asm__ volatile("" ::: "memory");
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (c[u] < (int32_t)rn + maxL) slot((uint32_t)(c[u] - (int32_t)kL) + sh[u]) = v[u];
        PROF_CNT(6, 1);
      }
    } else {
      const uint32_t sp = sp_all;  // ascending, 0xFFFFFFFF beyond nm
      const int32_t mp = (int32_t)readlane32(sp, 0);
      const bool mine = lane < nm;
      if (reloc) relocate_pool(nm);
      // queue item p >= mp moves up by #{new items at or before p}: passes of four chunks from the
      // tail down, all reads of a pass before its writes
      for (int32_t hi = (int32_t)qn; hi > mp; hi -= 4 * (int32_t)kWave) {
        uint4 v[4];
        int32_t r[4];
        uint32_t sh[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          r[u] = hi - (u + 1) * (int32_t)kWave + (int32_t)lane;
          v[u] = r[u] >= mp ? slot(rn + (uint32_t)r[u]) : make_uint4(0, 0, 0, 0);
        }
        // the items before the chunk, plus those inside it at or before the lane
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int32_t b = hi - (u + 1) * (int32_t)kWave;
          uint32_t c = ballot_count(mine && (int32_t)sp < b);
          for (uint64_t mk = __ballot(mine && (int32_t)sp >= b && (int32_t)sp < b + (int32_t)kWave); mk; mk &= mk - 1)
            c += (int32_t)lane >= (int32_t)readlane32(sp, (uint32_t)__builtin_ctzll(mk)) - b ? 1u : 0u;
          sh[u] = c;
        }
        __asm__ volatile("" ::: "memory");
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (r[u] >= mp) slot(rn + (uint32_t)r[u] + sh[u]) = v[u];
        PROF_CNT(6, 1);
      }
    }
    PROF_ADD(15, q2);
    __asm__ volatile("" ::: "memory");
    if (has) slot(rn - kL + pos + rank) = it;
    rh = (rh - kL) & kSlotMask;
    qn += nm;
    wave_lds_sync();
    PROF_ADD(4, i);
    PROF_CNT(5, nm);
  }
};

__device__ __forceinline__ uint4 make_item(uint64_t e, uint32_t len, uint32_t flags, uint32_t seq, uint32_t dst) {
  const uint64_t w0 = e | ((uint64_t)(len & 0xFFFFu) << 46) | ((uint64_t)flags << 62);
  return make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), seq, dst);
}

// ---------------------------------------------------------------------------------------------
// The carried netem queue and departure ring move between HBM and LDS with bounded buffer loads
// and stores: the resource covers exactly the live entries, so a lane past the end reads 0 without
// touching memory (one load instruction per 64 slots, no per-lane bounds branch).
//
// Hand-off of a source's carried state between the windows of one window-major fused launch
// (k_sim_fused): window k+1 of a source may run on another CU or XCD than window k, inside the same
// kernel, where neither the L1s nor the per-XCD L2s are coherent.  The producer writes every
// handed-off byte with write-through (sc1) stores, drains them (vmcnt(0)), then one lane stores the
// source's completion word; the consumer polls that word and reads every handed-off byte with
// L1-bypassing sc1 buffer loads (MI355X_MICROARCH.md, "Valid forms", first row of the hand-off table).
using v4u = unsigned int __attribute__((ext_vector_type(4)));
using v2u = unsigned int __attribute__((ext_vector_type(2)));
constexpr int kSc1 = 16;  // buffer cache-policy bit SC1 (gfx940+)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t region(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
template <int kPol>
__device__ __forceinline__ uint4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kPol));
}
template <int kPol>
__device__ __forceinline__ uint64_t ld8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, kPol));
}
template <int kPol>
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), r, (int)off, 0, kPol);
}
template <int kPol>
__device__ __forceinline__ uint32_t ld2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return (uint32_t)__builtin_bit_cast(uint16_t, __builtin_amdgcn_raw_buffer_load_b16(r, (int)off, 0, kPol));
}
template <int kPol>
__device__ __forceinline__ void st2(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (uint16_t)v), r, (int)off, 0, kPol);
}
template <int kPol>
__device__ __forceinline__ void st8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint64_t v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), r, (int)off, 0, kPol);
}
struct StatePair {
  uint4 lo, hi;
};

// Bucket width of an empty timing wheel (2^g ns): the narrowest for which the source's whole delay
// range (latency + jitter: every far item is eligible less than that past the horizon) spans at most
// kWheelB - 2 buckets, so the wheel holds every far item as its base slides up.  At the netem limit
// that is 16-32 items a bucket when they are spread evenly; bursts of admissions crowd some buckets,
// hence room for kWheelCB = 64.  Only the cost depends on it: a far item that does not fit (a full
// bucket, or a reshaped link's longer delay) stays in the heap array.
__device__ __forceinline__ uint32_t wheel_width(uint64_t span) {
  uint32_t g = kWheelGMin;
  while (g < kWheelGMax && (span >> g) > kWheelB - 2) ++g;
  return g;
}
constexpr uint32_t kWheelRebuildKeep = 32;  // far items left out of the wheel that ask for a rebuild
constexpr uint32_t kWheelCooldown = 16;     // windows before the next rebuild may be asked for
static_assert(sizeof(StatePair) == sizeof(SrcState), "SrcState hand-off");

// One source's step (K1-K4), run by one wavefront.  kOpen: the caller has checked that the step
// is an open queue without correlated draws, so only the open path is compiled in (fewer
// registers, a kCap-slot LDS queue).  wg: the slot of the stamps and the statistics copy.
// The queue, ring and SrcState come from HBM and go back there at the end.  *claim (when given) is
// the workgroup's next ticket, claimed before the write-back so that the atomic's round trip overlaps
// the stores; returned minus claim_base.  kMode: 0 plain loads and stores (k_sim, k_sim_list); 1 the
// HBM state is handed off inside a fused launch (bounded sc1 loads and stores).
constexpr int kModePlain = 0, kModeHandoff = 1;
// Departure-ring entries read with the queue (more, 64 at a time, only while none of them departs at
// or after the horizon): a window releases at most the entries before the first one >= an offer
// time < H, about a dozen per source in the C3 storm and three in C5
constexpr uint32_t kRingFirst = 16;
template <bool kOpen, uint32_t kCap, int kMode = kModePlain, bool kRecv = false, bool kList = false>
__device__ __forceinline__ uint32_t sim_source(const SimArgs& a, const uint32_t s, const uint32_t wg, SimLdsT<kCap>& lds,
                                               uint32_t* claim = nullptr, uint32_t claim_base = 0) {
  const uint32_t lane = threadIdx.x;
  constexpr uint32_t kSlotMask = kCap - 1;
  stamp(a, wg, lane, 0, __builtin_amdgcn_s_memrealtime());
  const SrcParams pp = a.params[s];
  constexpr bool kH = kMode == kModeHandoff, kBounded = kMode != kModePlain;
  constexpr int kPol = kH ? kSc1 : 0;
  SrcState st;  // dead after the set-up: the end writes a fresh state
  if constexpr (kH) {
    const auto rs = region(a.state + s, sizeof(SrcState));
    st = __builtin_bit_cast(SrcState, (StatePair{ld16<kSc1>(rs, 0), ld16<kSc1>(rs, 16)}));
  } else {
    st = a.state[s];
  }
  // the timing wheel's counts (lane j: bucket j) and header, loaded beside the state (used only when
  // the state says items are parked; an engine without a wheel reads nothing: offsets past a buffer
  // resource return 0 without a memory access)
  const auto rm = region(a.wmeta + s, sizeof(WheelMeta));
  const auto rw = region(a.wheel + (size_t)s * kWheelB * kWheelCB, kWheelB * kWheelCB * 16u);
  constexpr uint32_t kOff = 0xFFFFFFF0u;
  uint32_t wcnt = ld2<kPol>(rm, a.wmeta ? 2u * lane : kOff);
  const uint4 whd = ld16<kPol>(rm, a.wmeta ? 2u * kWheelB : kOff);
  // the offered packets' range and the source's link state with them (the records themselves are
  // loaded with the queue: one HBM round trip less before the first batch)
  const uint64_t sbeg = a.off[s], send = a.off[s + 1];
  const bool src_on = a.enabled[a.shard_begin + s] != 0;
  SimQueue<kCap, kList> Q{lds, pp, lane};
  Q.rh = 0;
  Q.rn = r_len(st);
  Q.rpush = 0;
  Q.qn = q_near(st);
  Q.pn = q_len(st) - q_near(st);  // the whole pool until it is split
  Q.fn = 0;
  Q.H = a.horizon_ns;
  Q.tat = st.tat;
  Q.src = a.shard_begin + s;
  // dense steps and fused windows: the classic layout; k_sim_list: the window's (EmitRead, emit_claim below)
  Q.emit = a.emit + 2 * sbeg + (uint64_t)(kList ? a.emit_r : kHeapCap) * s;
  Q.n_emit = 0;
  Q.dcnt = a.dst_cnt;
  Q.dslot = kList && a.dst_slot;
  Q.bkt = kList ? a.dst_bkt : nullptr;
  Q.bkt_log = a.bkt_log;
  Q.rf = kRecv ? recv_fold(a) : RecvFold{};
  Q.sched = Q.corrupted = Q.lost = 0;
  Q.bytes = 0;
#ifdef TGSIM_PROFILE
  for (int k = 0; k < 24; ++k) Q.pf[k] = 0;
  uint64_t* pf = Q.pf;
#endif
  // ---- load the head of the departure ring and the eligibility queue into LDS
  // The ring is circular in HBM (r_head): entry k of the ring is at slot (rh0 + k) of the source's
  // array.  Only a prefix is loaded, up to (and including) the first entry departing at or after the
  // horizon: every release this window stops at an entry >= an offer time < horizon, so the entries
  // behind it are never read; their LDS slots keep whatever they held (moved, never read) and they
  // stay in HBM untouched.  The ring moves in LDS only as a whole (release, append, the two-sided
  // merge), so the loaded entries stay the prefix.
  const uint32_t rh0 = r_head(st), rn0 = Q.rn;
  uint32_t rl = 0;  // ring entries loaded (a prefix)
  uint64_t idx = sbeg + lane;  // the lane's next offered record
  const uint64_t last_in = send > sbeg ? send - 1 : sbeg;
  InRec rec = {}, rec2 = {};   // records of batches b and b + 1
  uint32_t wbase = 0, wctl = 0, wdue = 0, nd = 0;  // wheel: base id, control word, lane j: bucket j's due count
  uint64_t wlast = 0;                              // the last bucket id due before H
  // due item c + lane: its bucket (from the base) is the first whose running sum exceeds it (the
  // running sums are re-derived at each call: nothing but wdue stays live across the queue's loads)
  auto wheel_item = [&](uint32_t c, bool& in) -> uint4 {
    TG_FULL_EXEC("ds_bpermute");
    const uint32_t rot = (uint32_t)__shfl((int)wdue, (int)((wbase + lane) & (kWheelB - 1)), 64);
    const uint32_t wincl = (uint32_t)scan_sum_i32((int32_t)rot), wexcl = wincl - rot;
    const uint32_t k = c + lane;
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t sb = kWave / 2; sb; sb >>= 1)
      if ((uint32_t)__shfl((int)wincl, (int)(lo + sb - 1), 64) <= k) lo += sb;
    const uint32_t j = lo & (kWheelB - 1);
    const uint32_t idx = k - (uint32_t)__shfl((int)wexcl, (int)j, 64);
    in = k < nd;
    return ld16<kPol>(rw, in ? 16u * (((wbase + j) & (kWheelB - 1)) * kWheelCB + idx) : kOff);
  };
  uint64_t moved = 0;  // queue-state bytes this source actually moves through HBM (carry accounting)
  {
    const uint64_t* gr = a.ring + (size_t)s * kHeapCap;
    const uint4* gh = a.heap + (size_t)s * kHeapCap;
    const uint32_t rn = Q.rn, qn = Q.qn + Q.pn;
    // every load of the ring's first chunk and the queue in flight before the first LDS write (one
    // HBM latency instead of one per 256 slots); a queue region of exactly qn entries, so the loads
    // past it return 0 with no memory access (branch-free: a conditional load made the compiler
    // wait for each chunk inside its branch)
    uint64_t rv0;
    uint4 qv[kCap / kWave];
    if constexpr (kBounded) {
      const auto rr = region(gr, 8u * kHeapCap), rq = region(gh, 16u * qn);
      rv0 = ld8<kPol>(rr, lane < kRingFirst ? 8u * ((rh0 + (lane < rn ? lane : 0u)) & (kHeapCap - 1)) : kOff);
#pragma unroll
      for (uint32_t u = 0; u < kCap / kWave; ++u) qv[u] = ld16<kPol>(rq, 16u * (u * kWave + lane));
    } else {  // a lane past the end re-reads the last entry (the same line as its neighbours)
      const uint32_t ql = qn ? qn - 1 : 0, qh = q_head(st);
      rv0 = gr[(rh0 + (lane < rn && lane < kRingFirst ? lane : 0u)) & (kHeapCap - 1)];
#pragma unroll
      for (uint32_t u = 0; u < kCap / kWave; ++u) {
        const uint32_t k = u * kWave + lane;
        qv[u] = gh[(qh + (k < qn ? k : ql)) & (kHeapCap - 1)];
      }
    }
    // the records of the first two batches (two batches in flight from here on); branch-free loads, a
    // lane past the end re-reads the last record (never used): a conditional load left a wait inside
    // its branch
    if (send > sbeg) {
      rec = a.in[idx < send ? idx : last_in];
      rec2 = a.in[idx + kWave < send ? idx + kWave : last_in];
    }
    // the timing wheel's due buckets (every bucket for k_sim_list or a rebuild): lane j holds the
    // running sum of the due counts of the buckets from the base up to the j-th; their items are
    // loaded with the queue (the first 64 here, the rest after the partition)
    if (q_parked(st)) {
      wbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)whd.x);
      wctl = (uint32_t)__builtin_amdgcn_readfirstlane((int)whd.y);
      const bool all = kList || (wctl >> 8 & 1u);
      wlast = (Q.H - 1) >> (wctl & 0xFFu);
      const bool due = all || (uint64_t)wbase + ((lane - wbase) & (kWheelB - 1)) <= wlast;
      wdue = due ? wcnt : 0u;
      nd = readlane32((uint32_t)scan_sum_i32((int32_t)wdue), kWave - 1);
      wcnt = due ? 0u : wcnt;
    } else {
      wcnt = 0;
    }
    bool win0;
    const uint4 wv0 = wheel_item(0, win0);
    // every load issued before the partition's ballots, which the scheduler would otherwise
    // interleave with them (one HBM round trip per chunk)
    __builtin_amdgcn_sched_barrier(0);
    rl = rn < kRingFirst ? rn : kRingFirst;
    if (lane < rl) *reinterpret_cast<uint2*>(&lds.slot[lane]) = make_uint2((uint32_t)rv0, (uint32_t)(rv0 >> 32));
    // more of the ring only while no loaded entry departs at or after the horizon (rare: a fast link
    // releasing more than 64 entries in one window)
    for (bool stop = __ballot(lane < rl && rv0 >= Q.H) != 0; !stop && rl < rn; rl = rl + kWave < rn ? rl + kWave : rn) {
      const uint32_t k = rl + lane;
      uint64_t v = ~0ull;
      if constexpr (kBounded) v = ld8<kPol>(region(gr, 8u * kHeapCap), 8u * ((rh0 + k) & (kHeapCap - 1)));
      else if (k < rn) v = gr[(rh0 + k) & (kHeapCap - 1)];
      if (k < rn) *reinterpret_cast<uint2*>(&lds.slot[k]) = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
      stop = __ballot(k < rn && v >= Q.H) != 0;
    }
    moved = 8ull * rl + 16ull * qn;
    // the pool (queue items near_n .. qn) splits into the soon part (e < H), placed from the pool's
    // front, and the far part, placed from its back (no order in either): one pass
    const uint32_t nq = Q.qn;
    const uint64_t below = (1ull << lane) - 1;
    uint32_t cs = 0, cf = 0;
#pragma unroll
    for (uint32_t u = 0; u < kCap / kWave; ++u) {
      const uint32_t k = u * kWave + lane;
      const bool pool = k >= nq && k < qn;
      const bool soon = pool && (w0_of(qv[u]) & kEMask) < Q.H;
      const uint64_t msn = __ballot(soon), mfr = __ballot(pool && !soon);
      uint32_t d = k;  // near items keep their place
      if (soon) d = nq + cs + (uint32_t)__popcll(msn & below);
      else if (pool) d = qn - 1 - cf - (uint32_t)__popcll(mfr & below);
      if (k < qn) lds.slot[(rn + d) & kSlotMask] = qv[u];
      cs += (uint32_t)__popcll(msn);
      cf += (uint32_t)__popcll(mfr);
    }
    Q.pn = cs;
    Q.fn = cf;
    // ---- the timing wheel: the due buckets' items join the pool (every parked item is >= the B of
    // any window since it was parked); the other buckets stay parked, only counted (Q.pk)
    Q.append_pool(win0, wv0);
  }
  for (uint32_t c = kWave; c < nd; c += kWave) {
    bool in;
    const uint4 v = wheel_item(c, in);
    Q.append_pool(in, v);
  }
  Q.pk = readlane32((uint32_t)scan_sum_i32((int32_t)wcnt), kWave - 1);
  if (Q.pk && wlast > wbase) wbase = (uint32_t)wlast;  // its items >= H are parked again
  if constexpr (kList) {
    // records past the source's region come from the emit pool: at most the queued items eligible
    // before the horizon (the near region and the soon pool; far items are >= H and cannot be
    // served) plus two per offered packet
    EmitOut eo = emit_out(a, s, sbeg, send);
    emit_claim(a, s, eo, Q.qn + Q.pn + (uint32_t)(2 * (send - sbeg)), lane);
    Q.over = eo.over;
    Q.cap = eo.cap;
  }
  if (q_parked(st)) moved += sizeof(WheelMeta) + 16ull * nd;
  lds.wcnt[lane] = wcnt;
  if (lane == 0) {
    lds.whdr[0] = wbase;
    lds.whdr[1] = wctl;
    lds.whdr[2] = nd;
    lds.whdr[3] = rh0 + rn0;  // the ring's head slot after the window = this - its length + appends
  }
#ifndef TGSIM_PROFILE
  stamp(a, wg, lane, 11, rl | (uint64_t)rn0 << 16);
#endif
#ifndef TGSIM_PROFILE
  stamp(a, wg, lane, 10, __builtin_amdgcn_s_memrealtime());  // (diagnostics: the wheel's phase)
#endif
  // no rules and every peer connected (the storm and gossip runs): the filter reduces to the
  // external-destination check, and the FIB/peer tables stay out of the loop's registers
  const bool plain = src_on && !a.any_disabled && pp.rule_n == 0;
  const uint32_t ext_v = (pp.shift_ext >> 8 & 1u) ? TGSIM_V_EXTERNAL : TGSIM_V_NO_ROUTE;
  const bool corr = (pp.rho_dup | pp.rho_cor | pp.rho_reo) != 0;
  const uint32_t lim = a.queue_limit;
  uint32_t last_dup = st.last_dup, last_cor = st.last_cor, last_reo = st.last_reo;
  // per-lane verdict counts, reduced over the wave once at the end (no wave-uniform counters held
  // in SGPRs through the loop): 16-bit fields, verdicts 0..3 in vc_lo and 4..7 in vc_hi, emptied
  // into the statistics every 2^14 batches (at most 2 counts per lane and batch), before a field
  // can overflow
  unsigned long long* const sc = a.stats + (size_t)(wg % kStatCopies) * kStSlots;
  // the per-window model of the queue state (a load of all of it here and a store at the end;
  // bit-exact with the oracle): the carry accounting subtracts what the window really moved
  // (the start's part of both here, the end's at the end: nothing of it held through the window)
  {
    const uint64_t b0 = 16ull * (Q.qn + Q.pn + Q.fn + Q.pk) + 8ull * Q.rn;
    if (lane == 0 && b0) atomicAdd(&sc[kStQueue], (unsigned long long)b0);
    if (lane == 0 && b0 != moved) atomicAdd(&sc[kStCarrySkip], (unsigned long long)(b0 - moved));
  }
  uint64_t vc_lo = 0, vc_hi = 0;
  uint32_t n_clone = 0;
  auto flush_verdicts = [&]() {
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      const uint32_t f = (uint32_t)(((k < 4 ? vc_lo : vc_hi) >> (16u * (k & 3u))) & 0xFFFFu);
      const uint32_t tot = readlane32((uint32_t)scan_sum_i32((int32_t)f), kWave - 1);
      if (lane == 0 && tot) atomicAdd(&sc[kStVerdict0 + k], (unsigned long long)tot);
    }
    vc_lo = vc_hi = 0;
  };
  uint32_t perr = 0;
  wave_lds_sync();
  // every pool item is >= the B of the previous step > every near item, so both of these are
  // valid boundaries; with an empty near region every new item starts in the pool
  Q.B = Q.qn ? (w0_of(Q.slot(Q.rn + Q.qn - 1)) & kEMask) + 1 : a.t0_ns;
  QCHECK(1);
  stamp(a, wg, lane, 1, __builtin_amdgcn_s_memrealtime());

  const uint32_t n_batches = (uint32_t)((send - sbeg + kWave - 1) / kWave);
  // open queue: even if every offered packet and its clone were admitted the queue would stay
  // below the netem limit (sparse sources: gossip, ping-pong, splitbrain)
  const bool open_q = kOpen || (!corr && (uint64_t)Q.rn + Q.qn + Q.pn + Q.fn + Q.pk + 2 * (send - sbeg) < lim);
  uint64_t T_enq = 0;  // open queue: offer time of the last packet that reached the netem enqueue
  // the verdict bytes of batch b are stored during batch b + 1: stored last in their own batch,
  // their write latency sat in front of the loop's back edge (vmcnt counts stores)
  uint64_t v_idx = 0;
  uint32_t v_out = 0;
  bool v_pend = false;
  for (uint32_t b = 0; b < n_batches; ++b) {
    PROF_T0(b);
    const uint64_t my_idx = idx;
    const bool staged = my_idx < send;
    const InRec r = rec;
    idx += kWave;
    rec = rec2;
    // in flight two batches ahead (three: no gain, A/B round 2)
    rec2 = a.in[idx + kWave < send ? idx + kWave : last_in];
    if (v_pend) a.verdict[v_idx] = (uint8_t)v_out;
    const uint64_t T = a.t0_ns + (uint64_t)r.tick * a.tick_ns;
    const uint32_t len = r.len & 0xFFFFu;
    uint32_t fv = 0u;
    if (plain) fv = r.dst == TGSIM_EXTERNAL ? ext_v : kFvPass;
    else if (staged) fv = filter(a, pp, src_on, r.dst);
    if (!staged) fv = 0u;
    uint32_t vout = 0xF0u | fv;  // verdict byte (final for filtered packets)
    if (kOpen || !corr) {
      // ---------- parallel phase: every decision that does not depend on queue state
      bool cand = false, reo_o = false;
      uint32_t cst = 0, flo = 0, flc = TGSIM_FLAG_DUP;
      uint64_t ec = ~0ull;
      if (staged && fv == kFvPass) {
        uint32_t r0[4];
        philox(Q.src, r.dst, r.seq, 0, a.key0, a.key1, r0);
        const int count = 1 + (pp.thr_dup && pp.thr_dup >= r0[0]) - (pp.thr_loss && pp.thr_loss >= r0[1]);
        if (count == 0) {
          vout = 0xF0u | TGSIM_V_LOSS;
        } else {
          cand = true;
          if (count == 2) {  // the clone re-enters the root qdisc with duplicate = 0
            uint32_t r2[4];
            philox(Q.src, r.dst, r.seq, 2, a.key0, a.key1, r2);
            if (pp.thr_loss && pp.thr_loss >= r2[0]) {
              cst = 1;
            } else {
              cst = 2;
              if (pp.thr_cor && pp.thr_cor >= r2[1]) flc |= TGSIM_FLAG_CORRUPT;
              ec = (pp.thr_reo && pp.thr_reo >= r2[2]) ? T : delayed(pp, T, r2[3]);
              if (ec > kEMask) { perr = 1; ec = kEMask; }
            }
          }
          flo = (pp.thr_cor && pp.thr_cor >= r0[2]) ? TGSIM_FLAG_CORRUPT : 0u;
          reo_o = pp.thr_reo && pp.thr_reo >= r0[3];
        }
      }
      PROF_ADD(0, b);
      PROF_T0(w);
      if (open_q) {
        // ---------- the netem limit cannot be reached in this step: every candidate is admitted,
        // and HTB serves in key order whatever the interleaving, so the items are merged now and
        // served once the batches are done
        uint64_t eo = reo_o ? T : T + pp.lat_ns;
        const bool need1 = cand && !reo_o && pp.sigma != 0;
        if (__ballot(need1)) {
          if (need1) {
            uint32_t r1[4];
            philox(Q.src, r.dst, r.seq, 1, a.key0, a.key1, r1);
            eo = delayed(pp, T, r1[0]);
          }
        }
        if (cand && eo > kEMask) { perr = 1; eo = kEMask; }
        if (cand) {
          const uint32_t cv = cst == 0 ? TGSIM_V_NONE : cst == 1 ? TGSIM_V_LOSS : TGSIM_V_SCHEDULED;
          vout = (cv << 4) | TGSIM_V_SCHEDULED;
        }
        Q.insert(cand, make_item(eo, len, flo, r.seq, r.dst));
        Q.insert(cand && cst == 2, make_item(ec, len, flc, r.seq, r.dst));
        const uint64_t mc = __ballot(cand);
        if (mc) T_enq = readlane64(T, 63u - (uint32_t)__builtin_clzll(mc));
      }
      // ---------- windows
      uint64_t pend = (kOpen || open_q) ? 0ull : __ballot(cand);
      if constexpr (!kOpen) while (pend) {
        PROF_CNT(3, 1);
        if (Q.rn + Q.qn + Q.pn + Q.fn + Q.pk >= lim) {
          // full queue: nothing changes before the next eligibility or departure time, so every
          // packet offered up to then is a QUEUE_FULL drop (B bounds the soon pool's earliest e,
          // H the far pool's and the parked items')
          const uint64_t qh = Q.qn ? (w0_of(Q.slot(Q.rn)) & kEMask) : Q.pn ? Q.B : (Q.fn | Q.pk) ? Q.H : ~0ull;
          const uint64_t dh = Q.rn ? Q.ring_d(0) : ~0ull;
          const uint64_t t_ev = qh < dh ? qh : dh;
          const uint64_t mf = __ballot(((pend >> lane) & 1ull) && T <= t_ev);
          if (mf) {
            if ((mf >> lane) & 1ull) {
              const uint32_t cv = cst == 0 ? TGSIM_V_NONE : cst == 1 ? TGSIM_V_LOSS : TGSIM_V_QUEUE_FULL;
              vout = (cv << 4) | TGSIM_V_QUEUE_FULL;
            }
            pend &= ~mf;
            PROF_CNT(2, 1);
            continue;
          }
        }
        const uint32_t w0 = (uint32_t)__builtin_ctzll(pend);
        const uint32_t wl = 63u - (uint32_t)__builtin_clzll(pend);
        const uint64_t T_last = readlane64(T, wl);
        QCHECK(10);
        Q.refill(T_last);  // every item eligible before the window's last packet in the near region
        QCHECK(8);
        PROF_T0(s1);
        // (1) queue-head items eligible before the last pending packet, served optimistically
        const bool hq = lane < Q.qn;
        const uint4 qi = hq ? Q.slot(Q.rn + lane) : make_uint4(0, 0, 0, 0);
        const uint64_t qe = hq ? (w0_of(qi) & kEMask) : ~0ull;
        const bool inS = qe < T_last;
        const uint32_t nS = ballot_count(inS);
        uint64_t T_cut = ~0ull;  // packets offered after the 65th queued item's e wait for the next window
        if (nS == kWave && Q.qn > kWave) {
          const uint64_t e64 = w0_of(Q.slot(Q.rn + kWave)) & kEMask;
          if (e64 < T_last) T_cut = e64;
        }
        uint64_t dS = 0, tatS = 0;
        if (nS) Q.htb_scan(inS, qe, qi.y >> 14 & 0xFFFFu, dS, tatS);
        PROF_ADD(7, s1);
        PROF_T0(s2);
        // (2) departures before each candidate's offer time: ring ++ newly served, sorted by d;
        //     only the prefix with d < the window's last offer time matters
        const bool inw = cand && ((pend >> lane) & 1ull) && T <= T_cut;
        const uint64_t mw = __ballot(inw);
        uint32_t D = 0;
        const uint64_t T_mx = mw ? readlane64(T, 63u - (uint32_t)__builtin_clzll(mw)) : 0ull;
        if (mw) {
          const uint64_t T_max = T_mx;
          for (uint32_t base = 0;; base += kWave) {
            const uint32_t k = base + lane;
            const uint32_t ks = k - Q.rn;  // index among the newly served items when k >= rn
            uint64_t dep = ~0ull;
            if (base + kWave > Q.rn && nS) {  // the chunk reaches past the ring (wave-uniform)
              const uint64_t dfs = shfl64(dS, (k >= Q.rn && ks < kWave) ? ks : 0u);
              if (k >= Q.rn && ks < nS) dep = dfs;
            }
            if (k < Q.rn) dep = Q.ring_d(k);
            // the netem queue releases departures from the ring head while head < T (a prefix:
            // with a lookahead the ring need not be sorted across a step boundary)
            const uint64_t stop = __ballot(dep >= T_max);
            const uint32_t nd = stop ? (uint32_t)__builtin_ctzll(stop) : kWave;
            // a lane keeps counting into this chunk only if every earlier entry was before its T
            const bool carry = D == base;
            if (nd > 16) {
              // prefix maxima of the chunk's first nd entries ascend: the lane's departures are
              // the entries before the first prefix maximum >= T (binary search over the lanes)
              const uint64_t pm = scan_max_u64(lane < nd ? dep : ~0ull);
              uint32_t lo = 0;
#pragma unroll
              for (uint32_t sb = 32; sb; sb >>= 1)
                if (shfl64(pm, lo + sb - 1) < T) lo += sb;
              lo += shfl64(pm, lo) < T ? 1u : 0u;
              if (carry) D += lo;
            } else {
              bool alive = carry;
              for (uint32_t l = 0; l < nd; ++l) {
                const uint64_t dl = readlane64(dep, l);  // (every lane: alive diverges)
                alive = alive && dl < T;
                D += alive ? 1u : 0u;
              }
            }
            if (nd < kWave) break;
          }
        }
        PROF_ADD(8, s2);
        PROF_T0(s3);
        // (3) netem limit: saturating occupancy counter, prefix-composed
        const uint32_t Dm = scan_max_u32(inw ? D : 0u);
        const int32_t delta = (int32_t)(Dm - shr1_u32(Dm, 0u));
        const int32_t cnt = inw ? 1 + (cst == 2) : 0;
        const int32_t P = scan_sum_i32(cnt - delta);
        const int32_t M = scan_max_i32(P);
        const int32_t x0 = (int32_t)(Q.rn + Q.qn + Q.pn + Q.fn + Q.pk), ilim = (int32_t)lim;
        const int32_t Pex = (int32_t)shr1_u32((uint32_t)P, 0u);
        const int32_t Mex = (int32_t)shr1_u32((uint32_t)M, 0u);  // lane 0: 0 = identity here
        const int32_t xb = Pex + min(x0, ilim - Mex);
        const int32_t y = xb - delta;
        const bool clone_adm = inw && cst == 2 && y < ilim;
        const bool orig_adm = inw && y + (cst == 2 ? 1 : 0) < ilim;
        // delay draw only for admitted originals
        uint64_t eo = reo_o ? T : T + pp.lat_ns;
        const bool need1 = orig_adm && !reo_o && pp.sigma != 0;
        if (__ballot(need1)) {
          if (need1) {
            uint32_t r1[4];
            philox(Q.src, r.dst, r.seq, 1, a.key0, a.key1, r1);
            eo = delayed(pp, T, r1[0]);
          }
        }
        if (orig_adm && eo > kEMask) { perr = 1; eo = kEMask; }
        PROF_ADD(9, s3);
        PROF_T0(s4);
        // (4) window end.  An admitted item i can change a later packet j's departure count only
        //     if its own departure, or that of a queued item it is served before, precedes T_j.
        //     Lower bound of both (HTB's TAT only grows when items are added):
        //       beta_i = min(d of the first queued item with e >= e_i, max(e_i, TAT before it)).
        //     The window ends before the first packet j with beta_i < T_j for an earlier i.
        uint64_t ea = clone_adm ? ec : ~0ull;
        if (orig_adm && eo < ea) ea = eo;
        // only items eligible before the last packet of the window can end it (beta_i >= e_i)
        const uint64_t madm = __ballot((orig_adm || clone_adm) && ea < T_mx);
        uint32_t wend = kWave;
        if (madm) {
          uint64_t beta = ~0ull;
          for (uint64_t mm = madm; mm; mm &= mm - 1) {
            const uint32_t i = (uint32_t)__builtin_ctzll(mm);
            const uint64_t ei = readlane64(ea, i);
            const uint32_t pe = ballot_count(inS && qe < ei);
            const uint64_t b1 = pe < nS ? readlane64(dS, pe) : ~0ull;
            const uint64_t tb = pe == 0 ? Q.tat : readlane64(tatS, pe - 1);
            const uint64_t b2 = ei > tb ? ei : tb;
            if (lane == i) beta = b1 < b2 ? b1 : b2;
          }
          const uint64_t Bex = shr1_u64(scan_min_u64(beta), ~0ull);
          const uint64_t mv = __ballot(inw && Bex < T);
          if (mv) wend = (uint32_t)__builtin_ctzll(mv);
          PROF_CNT(23, mv ? 1u : 0u);  // a sub-window ended by an admission eligible inside it
        }
        const bool inwin = inw && lane < wend;
        const uint64_t mwin = __ballot(inwin);
        uint64_t T_w, e_new = ~0ull;  // e_new: earliest new item (>= T_w unless madm)
        uint32_t Dw = 0, lw = 0;
        if (mwin) {
          lw = 63u - (uint32_t)__builtin_clzll(mwin);
          T_w = readlane64(T, lw);
          Dw = readlane32(D, lw);
          if (madm) e_new = readlane64(scan_min_u64(inwin ? ea : ~0ull), kWave - 1);
        } else {
          T_w = readlane64(T, w0);
        }
        PROF_ADD(10, s4);
        PROF_T0(s5);
        // commit the optimistic HTB service of the items served before every new item and
        // eligible before the window's last packet (the rest is served after the merge)
        const uint64_t t_c = e_new < T_w ? e_new : T_w;
        const bool inC = inS && qe < t_c;
        const uint32_t nC = ballot_count(inC);
        if (nC) Q.commit(inC, nC, qi, dS, tatS);
        QCHECK(5);
        Q.rh = (Q.rh + Dw) & kSlotMask;
        Q.rn -= Dw;
        PROF_ADD(11, s5);
        if (inwin) {
          const uint32_t cv = cst == 0 ? TGSIM_V_NONE
                            : cst == 1 ? TGSIM_V_LOSS
                                       : (clone_adm ? TGSIM_V_SCHEDULED : TGSIM_V_QUEUE_FULL);
          vout = (cv << 4) | (orig_adm ? TGSIM_V_SCHEDULED : TGSIM_V_QUEUE_FULL);
        }
        // (5) merge the admitted items into the sorted queue
        Q.insert(inwin && orig_adm, make_item(eo, len, flo, r.seq, r.dst));
        QCHECK(6);
        Q.insert(inwin && clone_adm, make_item(ec, len, flc, r.seq, r.dst));
        QCHECK(7);
        if (e_new < T_w) {
          PROF_T0(s6);
          Q.serve_until(T_w);
          PROF_ADD(12, s6);
          QCHECK(9);
        }
        if (mwin) pend &= lw >= 63u ? 0ull : ~((1ull << (lw + 1)) - 1);
        QCHECK(2);
      }
      PROF_ADD(1, w);
    } else if constexpr (!kOpen) {
      // ---------- correlated draws: per-packet netem_enqueue in order, wave-wide queue ops
      uint4 r0 = make_uint4(0, 0, 0, 0), r2 = make_uint4(0, 0, 0, 0);
      uint32_t r1x = 0;
      if (staged && fv == kFvPass) {
        uint32_t t[4];
        philox(Q.src, r.dst, r.seq, 0, a.key0, a.key1, t);
        r0 = make_uint4(t[0], t[1], t[2], t[3]);
        if (pp.thr_dup) {
          philox(Q.src, r.dst, r.seq, 2, a.key0, a.key1, t);
          r2 = make_uint4(t[0], t[1], t[2], t[3]);
        }
        if (pp.sigma) {
          philox(Q.src, r.dst, r.seq, 1, a.key0, a.key1, t);
          r1x = t[0];
        }
      }
      const uint32_t n_st = ballot_count(staged);
      for (uint32_t j = 0; j < n_st; ++j) {
        if (readlane32(fv, j) != kFvPass) continue;
        const uint64_t Tj = readlane64(T, j);
        const uint32_t dj = readlane32(r.dst, j), sj = readlane32(r.seq, j), lj = readlane32(len, j);
        const uint4 a0 = make_uint4(readlane32(r0.x, j), readlane32(r0.y, j), readlane32(r0.z, j), readlane32(r0.w, j));
        int count = 1;
        if (pp.thr_dup && pp.thr_dup >= crand(a0.x, pp.rho_dup, last_dup)) ++count;
        if (pp.thr_loss && pp.thr_loss >= a0.y) --count;
        uint32_t vj;
        if (count == 0) {
          vj = 0xF0u | TGSIM_V_LOSS;
        } else {
          // netem_enqueue from the limit check on; reorder consumes correlated state only when
          // the packet passes the limit
          auto enq = [&](uint32_t reo_raw, uint32_t delay_raw, uint32_t fl) -> uint32_t {
            Q.serve_until(Tj);
            Q.depart_before(Tj);
            if (Q.rn + Q.qn + Q.pn + Q.fn + Q.pk >= lim) return TGSIM_V_QUEUE_FULL;
            bool reordered = false;
            if (pp.thr_reo) reordered = !(pp.thr_reo < crand(reo_raw, pp.rho_reo, last_reo));
            uint64_t e = reordered ? Tj : delayed(pp, Tj, delay_raw);
            if (e > kEMask) { perr = 1; e = kEMask; }
            Q.insert(lane == 0, make_item(e, lj, fl, sj, dj));
            return TGSIM_V_SCHEDULED;
          };
          uint32_t cv = TGSIM_V_NONE;
          if (count == 2) {
            const uint4 a2 = make_uint4(readlane32(r2.x, j), readlane32(r2.y, j), readlane32(r2.z, j), readlane32(r2.w, j));
            if (pp.thr_loss && pp.thr_loss >= a2.x) {
              cv = TGSIM_V_LOSS;
            } else {
              uint32_t fl = TGSIM_FLAG_DUP;
              if (pp.thr_cor && pp.thr_cor >= crand(a2.y, pp.rho_cor, last_cor)) fl |= TGSIM_FLAG_CORRUPT;
              cv = enq(a2.z, a2.w, fl);
            }
          }
          uint32_t fl = 0;
          if (pp.thr_cor && pp.thr_cor >= crand(a0.z, pp.rho_cor, last_cor)) fl |= TGSIM_FLAG_CORRUPT;
          const uint32_t ov = enq(a0.w, readlane32(r1x, j), fl);
          vj = (cv << 4) | ov;
        }
        if (lane == j) vout = vj;
      }
    }
    v_pend = staged;
    v_idx = my_idx;
    v_out = vout;
    if (staged) {
      const uint32_t vo = vout & 15u, vc = vout >> 4;  // original 0..7, clone 0..7 or NONE
      const uint64_t uo = 1ull << (16u * (vo & 3u)), uc = 1ull << (16u * (vc & 3u));
      if (vo < 4) vc_lo += uo;
      else vc_hi += uo;
      if (vc < 4) vc_lo += uc;
      else if (vc < 8) vc_hi += uc;
      n_clone += vc != TGSIM_V_NONE ? 1u : 0u;
    }
    if ((b & 0x3FFFu) == 0x3FFFu) flush_verdicts();
  }
  if (v_pend) a.verdict[v_idx] = (uint8_t)v_out;
  stamp(a, wg, lane, 2, __builtin_amdgcn_s_memrealtime());
  if (open_q && T_enq) {  // what the last enqueue saw: service before its offer time, then departures
    Q.serve_until(T_enq);
    Q.depart_before(T_enq);
  }
  QCHECK(3);
  PROF_T0(e);
  Q.serve_until(a.horizon_ns);
  QCHECK(4);
  PROF_ADD(13, e);
  if (lane == 0) a.emit_n[s] = Q.n_emit;
  stamp(a, wg, lane, 3, __builtin_amdgcn_s_memrealtime());
  uint32_t next_ticket = 0;
  if (claim && lane == 0) next_ticket = atomicAdd(claim, 1u) - claim_base;
  // ---- park the far items in the timing wheel (k_sim_list keeps every item in the heap array: the
  // sparse kernels that run the next windows read only that)
  uint32_t pk_end = Q.pk;
  uint64_t moved_end = 0;  // queue-state bytes the end of the window moves through HBM
  if constexpr (!kList) {
    const uint32_t fn0 = a.wheel ? Q.fn : 0u;  // (no wheel: the engine had no memory for it)
    const auto rm = region(a.wmeta + s, sizeof(WheelMeta));
    const auto rw = region(a.wheel + (size_t)s * kWheelB * kWheelCB, kWheelB * kWheelCB * 16u);
    wbase = lds.whdr[0];
    wctl = lds.whdr[1];
    nd = lds.whdr[2];
    wcnt = lds.wcnt[lane];
    if (fn0) {
      const uint32_t f0 = Q.rn + Q.qn + Q.pn;
      if (!Q.pk) {  // an empty wheel: buckets wide enough for the source's delay range to fit
        wctl = (wctl & 0xFFFF0000u) | wheel_width(pp.lat_ns + (uint64_t)(pp.sigma > 0 ? pp.sigma : 0));
        lds.wcnt[lane] = 0;
        wave_lds_sync();
      }
      const uint32_t g0 = wctl & 0xFFu;
      // the base slides up to the lowest bucket in use (every bucket below it is empty): the far items
      // about to be parked and the buckets still parked
      uint64_t mn = ~0ull;
      for (uint32_t k = lane; k < fn0; k += kWave) {
        const uint64_t e = w0_of(Q.slot(f0 + k)) & kEMask;
        mn = e < mn ? e : mn;
      }
      mn >>= g0;
      if (Q.pk && wcnt) {
        const uint64_t id = (uint64_t)wbase + ((lane - wbase) & (kWheelB - 1));
        mn = id < mn ? id : mn;
      }
      wbase = (uint32_t)readlane64(scan_min_u64(mn), kWave - 1);
      const uint32_t g = g0;
      const uint64_t below = (1ull << lane) - 1;
      uint32_t kept = 0;
      for (uint32_t c = 0; c < fn0; c += kWave) {
        const uint32_t k = c + lane;
        const bool in = k < fn0;
        const uint4 it = in ? Q.slot(f0 + k) : make_uint4(0, 0, 0, 0);
        const uint64_t id = (w0_of(it) & kEMask) >> g;  // >= base: every far item is >= H
        bool ok = in && id - wbase < kWheelB;
        uint32_t pos = kWheelCB;
        if (ok) pos = atomicAdd(&lds.wcnt[(uint32_t)id & (kWheelB - 1)], 1u);
        ok = ok && pos < kWheelCB;
        if (ok) st16<kPol>(rw, 16u * (((uint32_t)id & (kWheelB - 1)) * kWheelCB + pos), it);
        // the others stay in the heap array, compacted behind the near region and the soon pool
        // (every lane has read its item before any lane writes; writes land at or below k)
        const bool kp = in && !ok;
        const uint64_t mk = __ballot(kp);
        if (kp) Q.slot(f0 + kept + (uint32_t)__popcll(mk & below)) = it;
        kept += (uint32_t)__popcll(mk);
      }
      wave_lds_sync();
      wcnt = lds.wcnt[lane];
      wcnt = wcnt < kWheelCB ? wcnt : kWheelCB;
      pk_end = readlane32((uint32_t)scan_sum_i32((int32_t)wcnt), kWave - 1);
      moved_end += 16ull * (fn0 - kept);
      Q.fn = kept;
#ifndef TGSIM_PROFILE
      stamp(a, wg, lane, 8, nd | (uint64_t)Q.pk << 16 | (uint64_t)fn0 << 32 | (uint64_t)kept << 48);
      stamp(a, wg, lane, 9, (uint64_t)g << 32 | (uint64_t)(wctl >> 8 & 1u) << 40);
#endif
    }
    if (pk_end && (nd || fn0 || (wctl >> 16))) {  // the wheel's counts and control word, when they changed
      // a reshaped link whose delay range no longer fits the buckets: every bucket comes back at the
      // next window and the wheel takes the new width
      const uint32_t cool = wctl >> 16;
      if (Q.fn > kWheelRebuildKeep && !cool &&
          wheel_width(pp.lat_ns + (uint64_t)(pp.sigma > 0 ? pp.sigma : 0)) != (wctl & 0xFFu))
        wctl = (wctl & 0xFFu) | 0x100u | kWheelCooldown << 16;
      else wctl = (wctl & 0xFFu) | (cool ? cool - 1 : 0u) << 16;
      st2<kPol>(rm, 2u * lane, wcnt);
      if (lane == 0) st16<kPol>(rm, 2u * kWheelB, make_uint4(wbase, wctl, 0u, 0u));
      moved_end += sizeof(WheelMeta);
    }
  }
  {
    // ---- write back the ring entries appended this window (the others are in HBM already: the
    // head moves past the released ones), the queue (near, then pool) and the state
    uint64_t* gr = a.ring + (size_t)s * kHeapCap;
    uint4* gh = a.heap + (size_t)s * kHeapCap;
    const uint32_t r_new = Q.rpush < Q.rn ? Q.rpush : Q.rn;             // the ring's last r_new entries
    const uint32_t rh1 = (lds.whdr[3] + Q.rpush - Q.rn) & (kHeapCap - 1);  // head after the releases
    moved_end += 8ull * r_new + 16ull * (Q.qn + Q.pn + Q.fn);
    if constexpr (kH) {  // write-through stores
      const auto rr = region(gr, kHeapCap * 8u), rq = region(gh, kHeapCap * 16u);
      for (uint32_t k = Q.rn - r_new + lane; k < Q.rn; k += kWave)
        st8<kSc1>(rr, 8u * ((rh1 + k) & (kHeapCap - 1)), Q.ring_d(k));
      for (uint32_t k = lane; k < Q.qn + Q.pn + Q.fn; k += kWave) st16<kSc1>(rq, 16u * k, Q.slot(Q.rn + k));
    } else {
      for (uint32_t k = Q.rn - r_new + lane; k < Q.rn; k += kWave) gr[(rh1 + k) & (kHeapCap - 1)] = Q.ring_d(k);
      for (uint32_t k = lane; k < Q.qn + Q.pn + Q.fn; k += kWave) gh[k] = Q.slot(Q.rn + k);  // near, then pool
    }
    uint32_t near_out = Q.qn;
    if constexpr (kList) {
      // k_sim_list: a queue whose pool happens to follow its near region in order (FIFO sources: no
      // jitter, reordering or duplication) is stored as one sorted region, so that the next step's
      // k_sim_sparse serves it in place instead of deferring it again
      const uint32_t tot = Q.qn + Q.pn + Q.fn;
      if (Q.pn + Q.fn) {
        bool bad = false;
        for (uint32_t k = lane + 1; k < tot; k += kWave) bad |= item_lt(Q.slot(Q.rn + k), Q.slot(Q.rn + k - 1));
        if (__ballot(bad) == 0) near_out = tot;
      }
    }
    if (lane == 0) {
      SrcState ns;
      ns.tat = Q.tat;
      ns.heap_n = q_pack(Q.qn + Q.pn + Q.fn, pk_end);
      ns.near_n = near_out;
      ns.ring_n = r_pack(Q.rn, rh1);
      ns.last_dup = last_dup;
      ns.last_cor = last_cor;
      ns.last_reo = last_reo;
      if constexpr (kH) {
        const auto rs = region(a.state + s, sizeof(SrcState));
        const StatePair sp = __builtin_bit_cast(StatePair, ns);
        st16<kSc1>(rs, 0, sp.lo);
        st16<kSc1>(rs, 16, sp.hi);
      } else {
        a.state[s] = ns;
      }
    }
  }
  stamp(a, wg, lane, 4, __builtin_amdgcn_s_memrealtime());
  stamp(a, wg, lane, 5, ((uint64_t)s << 32) | n_batches);
  stamp(a, wg, lane, 6, __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)));  // HW_ID
  stamp(a, wg, lane, 7, ((uint64_t)(Q.qn + Q.pn + Q.fn) << 32) | Q.rn);
#ifdef TGSIM_PROFILE
  for (int k = 0; k < 24; ++k) stamp(a, wg, lane, 8 + k, Q.pf[k]);
#endif
  const uint32_t sched = readlane32((uint32_t)scan_sum_i32((int32_t)Q.sched), kWave - 1);
  const uint32_t corrupted = readlane32((uint32_t)scan_sum_i32((int32_t)Q.corrupted), kWave - 1);
  const uint32_t lost = readlane32((uint32_t)scan_sum_i32((int32_t)Q.lost), kWave - 1);
  const uint64_t bytes = wave_sum(Q.bytes);
  const uint64_t qbytes = 16ull * (Q.qn + Q.pn + Q.fn + pk_end) + 8ull * Q.rn;
  const bool err = __ballot(perr != 0) != 0;
  const uint32_t c_clone = readlane32((uint32_t)scan_sum_i32((int32_t)n_clone), kWave - 1);
  flush_verdicts();
  if (lane == 0) {
    if (send > sbeg) atomicAdd(&sc[kStOffered], (unsigned long long)(send - sbeg));
    if (sched) atomicAdd(&sc[kStScheduled], (unsigned long long)sched);
    if (kList && a.dst_bkt && sched > Q.n_emit) atomicAdd(&sc[kStBktRecs], (unsigned long long)(sched - Q.n_emit));
    if (c_clone) atomicAdd(&sc[kStCloned], (unsigned long long)c_clone);
    if (corrupted) atomicAdd(&sc[kStCorrupted], (unsigned long long)corrupted);
    if (lost) atomicAdd(&sc[kStLost], (unsigned long long)lost);
    if (bytes) atomicAdd(&sc[kStBytes], (unsigned long long)bytes);
    if (qbytes) atomicAdd(&sc[kStQueue], (unsigned long long)qbytes);
    // what the model charged and the window did not move (wraps below zero when it moved more: the
    // readers sum modulo 2^64)
    if (qbytes != moved_end) atomicAdd(&sc[kStCarrySkip], (unsigned long long)(qbytes - moved_end));
    if (err) {
      atomicOr(&a.stats[kStErr], (unsigned long long)kErrTimeOverflow);
      if (a.err_host)  // the host's pinned copy (sticky; read at its sync points)
        __hip_atomic_store(a.err_host, (uint64_t)kErrTimeOverflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)next_ticket);
}

__global__ __launch_bounds__(kWave, 3) void k_sim(SimArgs a) {
  __shared__ SimLdsT<kHeapCap> lds;
  // heavy-first dispatch order (previous step's HTB work per source), identity when absent
  const uint32_t s = a.order ? a.order[blockIdx.x] : blockIdx.x;
  if (s >= a.n_src) return;
  sim_source<false, kHeapCap>(a, s, blockIdx.x, lds);
}

// k_sim with the gossip receipts folded in (a dense window of the single-shard gossip loop).
__global__ __launch_bounds__(kWave, 3) void k_sim_recv(SimArgs a) {
  __shared__ SimLdsT<kHeapCap> lds;
  const uint32_t s = a.order ? a.order[blockIdx.x] : blockIdx.x;
  if (s >= a.n_src) return;
  sim_source<false, kHeapCap, kModePlain, true>(a, s, blockIdx.x, lds);
}

// Several consecutive windows in one launch (tgsim_step_n).  Window k + 1 of a source depends only
// on the source's own state after window k, so the next window's heavy sources fill the CUs that the
// last dispatch round of this window leaves idle (one launch tail and one launch gap per fused group
// instead of one per window).  Persistent: the grid is what fits on the chip at once, and each
// workgroup takes tickets in order until none is left (its next ticket claimed during the write-back
// of the current one), so no slot waits for a workgroup dispatch between two sources.
struct FusedSim {
  SimArgs w[kFuseMax];  // window k's arguments (tables and state shared, step fields its own)
};
// Window k's arguments read in place in the kernel-argument segment (scalar loads of invariant
// memory: re-read when needed instead of held in spilled SGPRs).
__device__ __forceinline__ const SimArgs& kernarg_window(uint32_t k) {
  using KernargSimArgs = __attribute__((address_space(4))) const SimArgs;
  const KernargSimArgs* ka =
      (KernargSimArgs*)((__attribute__((address_space(4))) const char*)__builtin_amdgcn_kernarg_segment_ptr() +
                        k * sizeof(SimArgs));
  return *(const SimArgs*)ka;
}

// WINDOW-MAJOR (the default): ticket t is window t / S of the (t mod S)-th source in dispatch
// order; a ticket of window k > 0 polls its source's completion word until window k - 1 has stored
// it, and the queue crosses HBM between the windows (the sc1 hand-off above).  Every claimed ticket
// is held by a resident workgroup and waits only for a lower ticket, so the lowest unfinished ticket
// can always run: no deadlock; the wait is bounded anyway (kErrHandoff, then the host reports -EIO).
// Tickets interleave the windows of all sources at a granularity of one source-window, which keeps
// the launch's tail short (a source-major form, each source's windows back to back with its queue
// resident in LDS, was bit-exact but slower: DESIGN.md §5.2).
__global__ __launch_bounds__(kWave, 3) void k_sim_fused(FusedSim fs, FusedArgs f) {
  const SimArgs& a0 = fs.w[0];
  __shared__ SimLdsT<kHeapCap> lds;
  const uint32_t total = f.n_win * a0.n_src;
  uint32_t t = 0;
  if (threadIdx.x == 0) t = atomicAdd(f.ticket, 1u) - f.ticket_base;
  t = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
  while (t < total) {
    const uint32_t k = t / a0.n_src, pos = t - k * a0.n_src;
    const uint32_t s = a0.order ? a0.order[pos] : pos;
    // the heaviest sources (first in dispatch order) chain their windows through the launch: their
    // waves issue first on their SIMDs, so the chain is not the launch's critical path
    if (pos < f.prio_n) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(0);
    if (k) {
      const uint32_t need = f.step_base + k;
      uint32_t late = 0;
      if (threadIdx.x == 0) {
        for (uint32_t spin = 0;
             (int32_t)(__hip_atomic_load(f.done + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - need) < 0;) {
          __builtin_amdgcn_s_sleep(2);
          if (++spin > (1u << 22)) {
            late = 1;
            break;
          }
        }
      }
      if (__builtin_amdgcn_readfirstlane((int)late) && threadIdx.x == 0) {
        atomicOr(&a0.stats[kStErr], (unsigned long long)kErrHandoff);
        if (a0.err_host)
          __hip_atomic_store(a0.err_host, (uint64_t)kErrHandoff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    const uint32_t next = sim_source<false, kHeapCap, kModeHandoff>(kernarg_window(k), s, t, lds,
                                                            f.persistent ? f.ticket : nullptr, f.ticket_base);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every hand-off store written through
    if (threadIdx.x == 0)
      __hip_atomic_store(f.done + s, f.step_base + k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!f.persistent) break;  // one ticket per workgroup: the dispatcher interleaves other streams' work
    t = next;
  }
}

constexpr uint32_t kSparseQ = 4;  // chunks of 64 queued items / ring entries held in registers
constexpr uint32_t kFifoRounds = 4;  // FIFO sources: items served per step, in rounds of 64

// One served item's record (lanes with live set; x the queue item, d its HTB departure): the
// histogram increment first, whose return value is the record's destination slot (dst_slot); a slot
// below 2^bkt_log goes to the destination's bucket (dst_bkt), any other record to the source's emit
// records (emitted of them so far, wave-uniform; past the region and the pool: dropped,
// kErrEmitPool), with its slot above the delivery time.  The receipt is folded in (gossip).  Returns
// whether the lane's record was written.
__device__ __forceinline__ bool emit_record(const SimArgs& a, const EmitOut& eo, bool live, const uint4& x, uint64_t d,
                                            uint32_t xlen, uint32_t src, uint32_t fw, uint32_t fw_f,
                                            uint32_t& emitted, uint64_t below) {
  unsigned long long rank = 0;
  if (live && a.dst_cnt) {
    if (a.dst_slot) rank = atomicAdd(&a.dst_cnt[x.w], 1ull);
    else atomicAdd(&a.dst_cnt[x.w], 1ull);
  }
  const bool inb = live && a.dst_bkt != nullptr && rank < (1ull << a.bkt_log);
  bool ov = live && !inb;
  const uint32_t i = emitted + (uint32_t)__popcll(__ballot(ov) & below);
  ov = ov && eo.fits(i);
  emitted += (uint32_t)__popcll(__ballot(ov));
  if (!inb && !ov) return false;
  const uint32_t flags = x.y >> 30;
  uint64_t* rw = reinterpret_cast<uint64_t*>(inb ? a.dst_bkt + ((uint64_t)x.w << a.bkt_log) + rank : eo.at(i));
  rw[1] = ((uint64_t)x.w << 32) | src;
  rw[2] = ((uint64_t)flags << 48) | ((uint64_t)xlen << 32) | x.z;
  rw[0] = inb || !a.dst_slot ? d : d | slot_bits(rank);
  if (a.g_first) fold_receipt(recv_fold(a), x.w, x.z, flags, d, (uint64_t)fw << (fw_f & 32u));
  return true;
}

// ---------------------------------------------------------------------------------------------
// k_sim_multi: the FIFO sources k_sim_sparse cannot take in one round of lanes -- more than 64
// offered packets, or more than kFifoRounds x 64 items to serve (the gossip flood's peak).  The same
// FIFO path as sparse_source (the stored queue is one sorted region, the new items extend it in
// order, so HTB serves the prefix below the horizon in that order and the rest stays in place), with
// the candidates written straight behind the queue's tail in offer order: any number of rounds of 64
// offered packets and of served items run in one wave, at a register-only cost per round, and no
// LDS (the wave count per SIMD is set by the registers).  The served prefix (the queue's due items,
// then the due candidates) leaves by moving the head slot.  A source that turns out not to be FIFO
// (a clone that is queued, a new item before its predecessor) goes on to the general worklist
// (k_sim_list), which reads only the stored queue: the slots behind its tail are free space.  One wave
// per source, a grid-stride loop over the list k_sim_sparse wrote.
__device__ __forceinline__ void multi_source(const SimArgs& a, const uint32_t s) {
  const uint32_t lane = threadIdx.x;
  const uint64_t below = (1ull << lane) - 1;
  const uint4* gh = a.heap + (size_t)s * kHeapCap;
  const uint64_t* gr = a.ring + (size_t)s * kHeapCap;
  const SrcState st = a.state[s];
  const SrcParams pp = a.params[s];
  const uint64_t sbeg = a.off[s], send = a.off[s + 1];
  const uint32_t n = (uint32_t)(send - sbeg);
  const uint32_t rn = r_len(st), qn = q_len(st), rh0 = r_head(st);
  auto defer = [&]() {
    if (lane == 0) a.worklist[atomicAdd(a.worklist - 4, 1u)] = s;
  };
  // (k_sim_sparse checked the rest: no correlated draws, below the netem limit even if every offered
  // packet and a clone were queued -- so the candidates fit behind the tail, qn + n < kHeapCap --, at
  // most 256 ring entries, one sorted queue region)
  if (qn + n >= kHeapCap) {
    defer();
    return;
  }
  uint4* const wq = a.heap + (size_t)s * kHeapCap;
  unsigned long long* const sc = a.stats + (size_t)(s % kStatCopies) * kStSlots;
  const uint32_t src = a.shard_begin + s;
  const uint32_t qh = q_head(st);
  uint64_t rg[kSparseQ];
#pragma unroll
  for (uint32_t u = 0; u < kSparseQ; ++u) {
    const uint32_t k = u * kWave + lane;
    rg[u] = k < rn ? gr[(rh0 + k) & (kHeapCap - 1)] : ~0ull;
  }
  const uint4 qt = qn ? gh[(qh + qn - 1) & (kHeapCap - 1)] : make_uint4(0, 0, 0, 0);
  const bool src_on = a.enabled[src] != 0;
  const bool plain = src_on && !a.any_disabled && pp.rule_n == 0;
  const uint32_t ext_v = (pp.shift_ext >> 8 & 1u) ? TGSIM_V_EXTERNAL : TGSIM_V_NO_ROUTE;
  const uint64_t h = a.horizon_ns;
  // ---- netem decisions, 64 offered packets a round; candidates written behind the queue tail in HBM,
  // in offer order
  uint32_t nc = 0, n_due = 0, perr = 0, vcnt = 0, t_clone = 0;
  bool fifo = true, has_last = qn != 0;
  uint4 last = qt;  // the item every next candidate must not precede
  uint64_t T_enq = 0;
  for (uint32_t base = 0; base < n; base += kWave) {
    const bool staged = base + lane < n;
    InRec r = {};
    if (staged) r = a.in[sbeg + base + lane];
    const uint64_t T = a.t0_ns + (uint64_t)r.tick * a.tick_ns;
    const uint32_t len = r.len & 0xFFFFu;
    uint32_t fv = 0u;
    if (staged) fv = plain ? (r.dst == TGSIM_EXTERNAL ? ext_v : kFvPass) : filter(a, pp, src_on, r.dst);
    uint32_t vout = 0xF0u | fv;
    bool cand = false, queued_clone = false;
    uint4 io = make_uint4(0, 0, 0, 0);
    if (staged && fv == kFvPass) {
      uint32_t r0[4];
      philox(src, r.dst, r.seq, 0, a.key0, a.key1, r0);
      const int count = 1 + (pp.thr_dup && pp.thr_dup >= r0[0]) - (pp.thr_loss && pp.thr_loss >= r0[1]);
      if (count == 0) {
        vout = 0xF0u | TGSIM_V_LOSS;
      } else {
        cand = true;
        uint32_t cv = TGSIM_V_NONE;
        if (count == 2) {  // the clone: lost before the queue keeps the source FIFO, queued does not
          uint32_t r2[4];
          philox(src, r.dst, r.seq, 2, a.key0, a.key1, r2);
          if (pp.thr_loss && pp.thr_loss >= r2[0]) cv = TGSIM_V_LOSS;
          else queued_clone = true;
        }
        const uint32_t flo = (pp.thr_cor && pp.thr_cor >= r0[2]) ? TGSIM_FLAG_CORRUPT : 0u;
        const bool reo_o = pp.thr_reo && pp.thr_reo >= r0[3];
        uint64_t eo = reo_o ? T : T + pp.lat_ns;
        if (!reo_o && pp.sigma != 0) {
          uint32_t r1[4];
          philox(src, r.dst, r.seq, 1, a.key0, a.key1, r1);
          eo = delayed(pp, T, r1[0]);
        }
        if (eo > kEMask) { perr = 1; eo = kEMask; }
        io = make_item(eo, len, flo, r.seq, r.dst);
        vout = (cv << 4) | TGSIM_V_SCHEDULED;
      }
    }
    if (__ballot(queued_clone)) fifo = false;
    const uint64_t mc = __ballot(cand);
    // FIFO: no candidate before its predecessor (the candidate before it, or the last item so far)
    const uint64_t bc = mc & below;
    const uint32_t pl = bc ? 63u - (uint32_t)__builtin_clzll(bc) : lane;
    TG_FULL_EXEC("ds_permute");
    uint4 prev = make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute((int)(pl << 2), (int)io.x),
                            (uint32_t)__builtin_amdgcn_ds_bpermute((int)(pl << 2), (int)io.y),
                            (uint32_t)__builtin_amdgcn_ds_bpermute((int)(pl << 2), (int)io.z), 0u);
    if (!bc) prev = last;
    if (__ballot(cand && (bc || has_last) && item_lt(io, prev))) fifo = false;
    if (cand) wq[(qh + qn + nc + (uint32_t)__popcll(bc)) & (kHeapCap - 1)] = io;
    n_due += (uint32_t)__popcll(__ballot(cand && (w0_of(io) & kEMask) < h));
    if (mc) {
      const uint32_t ll = 63u - (uint32_t)__builtin_clzll(mc);
      last = make_uint4(readlane32(io.x, ll), readlane32(io.y, ll), readlane32(io.z, ll), 0u);
      has_last = true;
      T_enq = readlane64(T, ll);
    }
    nc += (uint32_t)__popcll(mc);
    if (staged) a.verdict[sbeg + base + lane] = (uint8_t)vout;  // rewritten by k_sim_list if deferred
    const uint32_t vo = vout & 15u, vc = vout >> 4;
#pragma unroll
    for (uint32_t v = 0; v < 8; ++v) {
      const uint32_t t = ballot_count(staged && vo == v) + ballot_count(staged && vc == v);
      if (lane == v) vcnt += t;
    }
    t_clone += ballot_count(staged && vc != TGSIM_V_NONE);
  }
  if (!fifo) {
    defer();
    return;
  }
  // the candidates' stores complete before the serving rounds read the due ones back (other lanes'
  // stores: the wave's own L1, so a workgroup-scope fence)
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  // ---- the queue's prefix below the horizon: all of it when a candidate is due (every queued item
  // precedes it), else its chunks from the head while they are due entirely
  uint32_t nq = n_due ? qn : 0;
  if (!n_due) {
    for (uint32_t c = 0; c * kWave < qn; ++c) {
      const uint32_t k = c * kWave + lane;
      const uint4 v = k < qn ? gh[(qh + k) & (kHeapCap - 1)] : make_uint4(0, 0, 0, 0);
      const uint32_t d = (uint32_t)__popcll(__ballot(k < qn && (w0_of(v) & kEMask) < h));
      nq += d;
      if (d < kWave) break;
    }
  }
  // ---- the old ring: the prefix departing before the last enqueue is released (as in sparse_source)
  uint64_t* wr = a.ring + (size_t)s * kHeapCap;
  bool ring_stop = T_enq == 0;
  uint32_t k0 = 0;
  if (T_enq) {
#pragma unroll
    for (uint32_t u = 0; u < kSparseQ; ++u) {
      if (!ring_stop && u * kWave < rn) {
        const uint64_t m = __ballot(u * kWave + lane < rn && rg[u] >= T_enq);
        const uint32_t cnt = rn - u * kWave < kWave ? rn - u * kWave : kWave;
        if (m) {
          k0 += (uint32_t)__builtin_ctzll(m);
          ring_stop = true;
        } else {
          k0 += cnt;
        }
      }
    }
  }
  // the kept old entries stay where they are in HBM: the head moves past the released ones
  const uint32_t old_kept = rn - k0, rh1 = (rh0 + k0) & (kHeapCap - 1);
  // ---- in place: the served prefix (a due candidate means the whole queue is due) leaves by moving
  // the head slot; the candidates not served are already behind the tail
  const uint32_t new_head = (qh + nq + n_due) & (kHeapCap - 1);
  const uint32_t wpos = qn - nq + nc - n_due;
  const uint32_t ns_all = nq + n_due;
  // ---- HTB, records, receipts and the ring, for the served items in rounds of 64 lanes: the
  // queue's due items, then the due candidates, contiguous from the head slot
  uint64_t tat_c = st.tat;
  uint32_t emitted = 0, sched_n = 0, sk0 = 0, t_cor = 0, t_lost = 0;
  uint64_t bytes = 0;
  bool releasing = T_enq && !ring_stop;
  EmitOut eo = emit_out(a, s, sbeg, send);
  emit_claim(a, s, eo, ns_all, lane);
  for (uint32_t base = 0; base < ns_all; base += kWave) {
    const uint32_t k = base + lane;
    const uint32_t ns = ns_all - base < kWave ? ns_all - base : kWave;
    const bool hs = lane < ns;
    const uint4 x = hs ? gh[(qh + k) & (kHeapCap - 1)] : make_uint4(0, 0, 0, 0);
    const uint32_t fw_f = a.g_first ? x.z / a.g_degree : 0u;
    const uint32_t fw = a.g_first && hs && x.w - a.shard_begin < a.n_src && fw_f < 64u
                            ? reinterpret_cast<const uint32_t*>(a.g_fwd)[2ull * (x.w - a.shard_begin) + (fw_f >> 5)]
                            : 0u;
    const uint64_t e = w0_of(x) & kEMask;
    const uint32_t xlen = x.y >> 14 & 0xFFFFu;
    const uint64_t c = ((uint64_t)xlen * pp.mult) >> (pp.shift_ext & 0xFFu);
    uint64_t A = hs ? c : 0, Bm = hs ? (e > pp.burst_ns ? e - pp.burst_ns : 0) + c : 0;
    scan_maxplus(A, Bm);
    const uint64_t ta = tat_c + A;
    const uint64_t tat_after = ta > Bm ? ta : Bm;
    const uint64_t before = shr1_u64(tat_after, tat_c);
    const uint64_t d = e > before ? e : before;
    tat_c = readlane64(tat_after, ns - 1);
    bool live = hs && x.w != kDeadDst;
    const bool dead = hs && !live;
    live = emit_record(a, eo, live, x, d, xlen, src, fw, fw_f, emitted, below);
    if (live) bytes += xlen;
    sched_n += (uint32_t)__popcll(__ballot(live));
    t_cor += (uint32_t)__popcll(__ballot(live && (x.y >> 31)));
    t_lost += (uint32_t)__popcll(__ballot(dead));
    if (releasing) {  // a prefix of the served entries departed before the last enqueue
      const uint32_t n1 = (uint32_t)__popcll(__ballot(hs && e < T_enq));
      const uint64_t m = __ballot(lane < n1 && d >= T_enq);
      if (m) {
        sk0 = base + (uint32_t)__builtin_ctzll(m);
        releasing = false;
      } else {
        sk0 = base + n1;
        releasing = n1 == kWave;
      }
    }
    if (hs && k >= sk0) wr[(rh1 + old_kept + k - sk0) & (kHeapCap - 1)] = d;
  }
  const uint32_t rn_new = old_kept + ns_all - sk0;
  if (lane == 0) {
    SrcState ns_;
    ns_.tat = tat_c;
    ns_.heap_n = q_pack(wpos, 0);
    ns_.near_n = wpos | new_head << 16;  // sorted in place
    ns_.ring_n = r_pack(rn_new, rh1);
    ns_.last_dup = st.last_dup;
    ns_.last_cor = st.last_cor;
    ns_.last_reo = st.last_reo;
    a.state[s] = ns_;
    a.emit_n[s] = emitted;
  }
  // ---- statistics
  const uint64_t t_bytes = wave_sum(bytes);
  const bool err = __ballot(perr != 0) != 0;
  if (lane < 8 && vcnt) atomicAdd(&sc[kStVerdict0 + lane], (unsigned long long)vcnt);
  if (lane == 0) {
    const uint64_t qb = 16ull * qn + 8ull * rn + 16ull * wpos + 8ull * rn_new;
    // HBM items of the queue this step touched: the due prefix read, the tail item, the appended ones
    const uint32_t q_moved = nq + (qn ? 1u : 0u) + nc - n_due;
    const uint64_t q_kept = (qn + wpos > q_moved ? 16ull * (qn + wpos - q_moved) : 0ull) + 8ull * old_kept;
    if (q_kept) atomicAdd(&sc[kStCarrySkip], (unsigned long long)q_kept);
    if (n) atomicAdd(&sc[kStOffered], (unsigned long long)n);
    if (sched_n) atomicAdd(&sc[kStScheduled], (unsigned long long)sched_n);
    if (a.dst_bkt && sched_n > emitted) atomicAdd(&sc[kStBktRecs], (unsigned long long)(sched_n - emitted));
    if (t_clone) atomicAdd(&sc[kStCloned], (unsigned long long)t_clone);
    if (t_cor) atomicAdd(&sc[kStCorrupted], (unsigned long long)t_cor);
    if (t_lost) atomicAdd(&sc[kStLost], (unsigned long long)t_lost);
    if (t_bytes) atomicAdd(&sc[kStBytes], (unsigned long long)t_bytes);
    if (qb) atomicAdd(&sc[kStQueue], (unsigned long long)qb);
    if (err) {
      atomicOr(&a.stats[kStErr], (unsigned long long)kErrTimeOverflow);
      if (a.err_host)
        __hip_atomic_store(a.err_host, (uint64_t)kErrTimeOverflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// The multi-round list k_sim_sparse writes: its count is the word after the worklist's count (one
// memset clears both), its sources follow the worklist's statistics words.
__device__ __forceinline__ uint32_t* multi_count(const SimArgs& a) { return a.worklist - 3; }
__device__ __forceinline__ uint32_t* multi_list(const SimArgs& a) { return a.worklist + a.n_src + 8; }

__global__ __launch_bounds__(kWave) void k_sim_multi(SimArgs a) {
  const uint32_t* const list = multi_list(a);
  const uint32_t n = *multi_count(a);
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) multi_source(a, list[i]);
}

// Register-only form of an open-queue step (the sparse senders of a gossip flood): no LDS queue.
// Every queued item (near and pool, up to 256) and every new item stay in registers; the items
// HTB serves this step (e < horizon: at most 64, else the source is deferred) are gathered into
// one lane each, ranked by key and served with one max-plus scan; what is not served is written
// back as the pool (no order needed), the departure ring as the general path leaves it.  Exactly
// the open path of sim_source: HTB serves in key order whatever the interleaving, the ring is
// released up to the last enqueue's offer time, every candidate is admitted.  A source that does
// not fit (correlated draws, a queue that could reach the limit, more than 64 offered packets, 256
// queued items, 256 ring entries or 64 items to serve) writes nothing and goes to the worklist.
// (FIFO sources with more than one round of lanes go to k_sim_multi above instead.)
__device__ __forceinline__ void sparse_source(const SimArgs& a, const uint32_t s) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint64_t below = (1ull << lane) - 1;
  stamp(a, s, lane, 0, __builtin_amdgcn_s_memrealtime());
  // the queue starts at its head slot; the ring (needed only after the netem decisions) is read with
  // the queue, as far as the state says it is live
  const uint4* gh = a.heap + (size_t)s * kHeapCap;
  const uint64_t* gr = a.ring + (size_t)s * kHeapCap;
  const SrcState st = a.state[s];
  const uint64_t sbeg = a.off[s], send = a.off[s + 1];
  const uint32_t n = (uint32_t)(send - sbeg);
  const uint32_t rn = r_len(st), qn = q_len(st), rh0 = r_head(st);
  auto defer = [&](uint32_t why) {
    if (lane == 0) a.worklist[atomicAdd(a.worklist - 4, 1u)] = s;
    (void)why;
  };
  if (q_parked(st)) {  // far items parked in the timing wheel: the general path reads them
    defer(5u);
    return;
  }
  const bool sorted_st = q_near(st) == qn;  // the whole queue is one sorted region
  // FIFO candidates beyond one round of lanes go to k_sim_multi (multi-round, candidates written behind
  // the queue tail in HBM)
  auto defer_multi = [&]() {
    if (lane == 0) {
      multi_list(a)[atomicAdd(multi_count(a), 1u)] = s;
    }
  };
  unsigned long long* const sc = a.stats + (size_t)(s % kStatCopies) * kStSlots;
  const uint4 qh0 = sorted_st && qn && !n ? gh[q_head(st)] : make_uint4(0, 0, 0, 0);
  if (!n && (!qn || (sorted_st && (w0_of(qh0) & kEMask) >= a.horizon_ns))) {
    // nothing offered and nothing eligible before the horizon: the state stays as it is (the ring
    // is released only by an enqueue); only the per-window queue model is counted.  Checked before
    // the capacity limits below: an idle source with a long ring (the end of a flood) is not deferred
    if (lane == 0) {
      a.emit_n[s] = 0;
      const uint64_t qb = 32ull * qn + 16ull * rn;
      if (qb) atomicAdd(&sc[kStQueue], (unsigned long long)qb);
      if (qn) atomicAdd(&sc[kStCarrySkip], (unsigned long long)(32ull * qn - 16ull));
      if (rn) atomicAdd(&sc[kStCarrySkip], (unsigned long long)(16ull * rn));
    }
    return;
  }
  // the parameters only once the source is known not to be idle (most of the million sources of an
  // off-peak gossip window are; their 64-B rows stay unread), beside the offered records' loads
  const SrcParams pp = a.params[s];
  if ((pp.rho_dup | pp.rho_cor | pp.rho_reo) != 0 || (uint64_t)rn + qn + 2ull * n >= a.queue_limit || n > kWave ||
      (!sorted_st && qn > kSparseQ * kWave) || rn > kSparseQ * kWave) {
    const uint32_t why = (pp.rho_dup | pp.rho_cor | pp.rho_reo) != 0 ? 0u : (uint64_t)rn + qn + 2ull * n >= a.queue_limit ? 1u
                         : n > kWave ? 2u : rn > kSparseQ * kWave ? 4u : 3u;
    if (why == 2u && sorted_st && rn <= kSparseQ * kWave) defer_multi();
    else defer(why);
    return;
  }
  const uint32_t src = a.shard_begin + s;
  stamp(a, s, lane, 1, __builtin_amdgcn_s_memrealtime());
  // ---- loads: the queue (a sorted one: its first chunk and its last item; else whole chunks,
  // masked), the rest of the ring, the offered packets
  const uint32_t qh = q_head(st);
  uint4 q[kSparseQ];
  uint64_t rg[kSparseQ];
  q[0] = lane < qn ? gh[(qh + lane) & (kHeapCap - 1)] : make_uint4(0, 0, 0, 0);
  rg[0] = lane < rn ? gr[(rh0 + lane) & (kHeapCap - 1)] : ~0ull;
  auto load_rest = [&]() {
#pragma unroll
    for (uint32_t u = 1; u < kSparseQ; ++u) {
      const uint32_t k = u * kWave + lane;
      q[u] = k < qn ? gh[(qh + k) & (kHeapCap - 1)] : make_uint4(0, 0, 0, 0);
    }
  };
  uint4 qt = make_uint4(0, 0, 0, 0);  // a sorted queue's last item
  if (sorted_st) {
    if (qn > kWave) qt = gh[(qh + qn - 1) & (kHeapCap - 1)];
#pragma unroll
    for (uint32_t u = 1; u < kSparseQ; ++u) q[u] = make_uint4(0, 0, 0, 0);
  } else {
    load_rest();
  }
#pragma unroll
  for (uint32_t u = 1; u < kSparseQ; ++u) {
    const uint32_t k = u * kWave + lane;
    rg[u] = k < rn ? gr[(rh0 + k) & (kHeapCap - 1)] : ~0ull;
  }
  InRec r = {};
  const bool staged = lane < n;
  if (staged) r = a.in[sbeg + lane];
  const uint64_t T = a.t0_ns + (uint64_t)r.tick * a.tick_ns;
  const uint32_t len = r.len & 0xFFFFu;
  // ---- filter and netem decisions (queue-independent; every candidate is admitted)
  const bool src_on = a.enabled[src] != 0;
  const bool plain = src_on && !a.any_disabled && pp.rule_n == 0;
  const uint32_t ext_v = (pp.shift_ext >> 8 & 1u) ? TGSIM_V_EXTERNAL : TGSIM_V_NO_ROUTE;
  uint32_t fv = 0u;
  if (staged) fv = plain ? (r.dst == TGSIM_EXTERNAL ? ext_v : kFvPass) : filter(a, pp, src_on, r.dst);
  uint32_t vout = 0xF0u | fv;
  bool cand = false;
  uint32_t cst = 0, perr = 0;
  uint4 io = make_uint4(0, 0, 0, 0), ic = make_uint4(0, 0, 0, 0);
  if (staged && fv == kFvPass) {
    uint32_t r0[4];
    philox(src, r.dst, r.seq, 0, a.key0, a.key1, r0);
    const int count = 1 + (pp.thr_dup && pp.thr_dup >= r0[0]) - (pp.thr_loss && pp.thr_loss >= r0[1]);
    if (count == 0) {
      vout = 0xF0u | TGSIM_V_LOSS;
    } else {
      cand = true;
      if (count == 2) {
        uint32_t r2[4];
        philox(src, r.dst, r.seq, 2, a.key0, a.key1, r2);
        if (pp.thr_loss && pp.thr_loss >= r2[0]) {
          cst = 1;
        } else {
          cst = 2;
          uint32_t flc = TGSIM_FLAG_DUP;
          if (pp.thr_cor && pp.thr_cor >= r2[1]) flc |= TGSIM_FLAG_CORRUPT;
          uint64_t ec = (pp.thr_reo && pp.thr_reo >= r2[2]) ? T : delayed(pp, T, r2[3]);
          if (ec > kEMask) { perr = 1; ec = kEMask; }
          ic = make_item(ec, len, flc, r.seq, r.dst);
        }
      }
      const uint32_t flo = (pp.thr_cor && pp.thr_cor >= r0[2]) ? TGSIM_FLAG_CORRUPT : 0u;
      const bool reo_o = pp.thr_reo && pp.thr_reo >= r0[3];
      uint64_t eo = reo_o ? T : T + pp.lat_ns;
      if (!reo_o && pp.sigma != 0) {
        uint32_t r1[4];
        philox(src, r.dst, r.seq, 1, a.key0, a.key1, r1);
        eo = delayed(pp, T, r1[0]);
      }
      if (eo > kEMask) { perr = 1; eo = kEMask; }
      io = make_item(eo, len, flo, r.seq, r.dst);
      const uint32_t cv = cst == 0 ? TGSIM_V_NONE : cst == 1 ? TGSIM_V_LOSS : TGSIM_V_SCHEDULED;
      vout = (cv << 4) | TGSIM_V_SCHEDULED;
    }
  }
  const uint64_t mc = __ballot(cand);
  const uint64_t T_enq = mc ? readlane64(T, 63u - (uint32_t)__builtin_clzll(mc)) : 0ull;
  stamp(a, s, lane, 2, __builtin_amdgcn_s_memrealtime());
  const uint64_t h = a.horizon_ns;
  uint4 x = make_uint4(0, 0, 0, 0);
  uint32_t ns = 0;
  bool over = false;
  // moves the lanes with f set (k of them) to lanes [ns, ns + k), in lane order, into x
  auto gather = [&](bool f, const uint4& v) {
    const uint64_t m = __ballot(f);
    if (!m) return;
    const uint32_t k = (uint32_t)__popcll(m);
    if (ns + k > kWave) {
      over = true;
      return;
    }
    const uint32_t to = (f ? ns + (uint32_t)__popcll(m & below) : ns + k + (uint32_t)__popcll(~m & below)) & (kWave - 1);
    TG_FULL_EXEC("ds_permute");
    const uint4 pv = make_uint4((uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.x),
                                (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.y),
                                (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.z),
                                (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)v.w));
    if (lane >= ns && lane < ns + k) x = pv;
    ns += k;
  };
  uint4* wq = a.heap + (size_t)s * kHeapCap;
  uint32_t wpos = 0;
  // The departure ring: old ring ++ served.  The last enqueue (at T_enq, after serving the items
  // eligible before it) released the prefix departing before T_enq; the old ring's part of it is
  // known before HTB runs, so the kept old entries are written back (and their registers freed) as
  // soon as the source is known not to defer.
  uint64_t* wr = a.ring + (size_t)s * kHeapCap;
  uint32_t old_kept = rn;     // old entries still in the ring
  uint32_t rh1 = rh0;         // the ring's head slot after the release
  bool ring_stop = T_enq == 0;  // the release stopped inside the old ring (or nothing was released)
  auto write_old_ring = [&]() {  // (the kept old entries stay in place in HBM: only the head moves)
    uint32_t k0 = 0;
    if (T_enq) {
#pragma unroll
      for (uint32_t u = 0; u < kSparseQ; ++u) {
        if (!ring_stop && u * kWave < rn) {
          const uint64_t m = __ballot(u * kWave + lane < rn && rg[u] >= T_enq);
          const uint32_t cnt = rn - u * kWave < kWave ? rn - u * kWave : kWave;
          if (m) {
            k0 += (uint32_t)__builtin_ctzll(m);
            ring_stop = true;
          } else {
            k0 += cnt;
          }
        }
      }
    }
    old_kept = rn - k0;
    rh1 = (rh0 + k0) & (kHeapCap - 1);
  };
  // ---- FIFO sources (no jitter, no reordering, no duplicates: gossip): the stored queue is sorted
  // (a whole near region) and the new items, in offer order, are sorted and not before its last
  // item, so (queue ++ new) is sorted: HTB serves its prefix below the horizon, in that order, and
  // the rest goes back sorted, shifted down, with no gather of the queue, no rank and no compaction.
  bool fifo = sorted_st && __ballot(cand && cst == 2) == 0;
  if (fifo && mc) {
    const uint64_t bc = mc & below;  // the candidate before each candidate, or the queue's last item
    const uint32_t pl = bc ? 63u - (uint32_t)__builtin_clzll(bc) : lane;
    TG_FULL_EXEC("ds_permute");
    uint4 prev = make_uint4((uint32_t)__builtin_amdgcn_ds_bpermute((int)(pl << 2), (int)io.x),
                            (uint32_t)__builtin_amdgcn_ds_bpermute((int)(pl << 2), (int)io.y),
                            (uint32_t)__builtin_amdgcn_ds_bpermute((int)(pl << 2), (int)io.z), 0u);
    bool first = cand && !bc;
    if (qn) {
      if (qn <= kWave) {
        const uint32_t tl = qn - 1;
        qt = make_uint4(readlane32(q[0].x, tl), readlane32(q[0].y, tl), readlane32(q[0].z, tl), 0u);
      }
      if (first) prev = qt;
    } else {
      first = false;  // nothing queued: the first candidate has no predecessor
    }
    fifo = __ballot(cand && (bc || first) && item_lt(io, prev)) == 0;
  }
  uint32_t new_head = 0;
  uint32_t q_moved = 0;  // queue items read or written in HBM (FIFO path: not the whole queue)
  uint32_t fifo_nq = 0, ns_all = 0, cpos = 0;  // FIFO: due queue items, all served, a due candidate's place
  bool due_f = false;                           // FIFO: a due candidate
  if (fifo) {
    // the queue's prefix below the horizon: its first chunk, and while a chunk is due entirely the
    // next one (the served items run in rounds of 64 below, at most kFifoRounds)
    uint32_t nq = (uint32_t)__popcll(__ballot(lane < qn && (w0_of(q[0]) & kEMask) < h));
    for (uint32_t c = 1; c < kFifoRounds && nq == c * kWave && qn > nq; ++c) {
      const uint32_t k = c * kWave + lane;
      const uint4 v = k < qn ? gh[(qh + k) & (kHeapCap - 1)] : make_uint4(0, 0, 0, 0);
      nq += (uint32_t)__popcll(__ballot(k < qn && (w0_of(v) & kEMask) < h));
    }
    const bool due_o = cand && (w0_of(io) & kEMask) < h;  // a prefix of the candidates
    const uint64_t dm = __ballot(due_o);
    const uint32_t n_due = (uint32_t)__popcll(dm);
    if (nq + n_due > kFifoRounds * kWave || (nq == kFifoRounds * kWave && qn > nq)) {
      defer_multi();
      return;
    }
    write_old_ring();
    fifo_nq = nq;
    ns_all = nq + n_due;
    due_f = due_o;
    cpos = nq + (uint32_t)__popcll(dm & below);
    x = lane < nq ? q[0] : make_uint4(0, 0, 0, 0);
    ns = nq < kWave ? nq : kWave;
    gather(due_o && cpos < kWave, io);
    // in place: the served prefix leaves by moving the head slot, the candidates not served are
    // appended behind the tail; nothing else moves
    const uint32_t cr = (uint32_t)__popcll(mc & below);
    if (cand && !due_o) wq[(qh + qn + cr - n_due) & (kHeapCap - 1)] = io;
    new_head = (qh + nq) & (kHeapCap - 1);
    wpos = qn - nq + (uint32_t)__popcll(mc) - n_due;
    q_moved = (qn < kWave ? qn : kWave) + (qn > kWave ? 1u : 0u) + (uint32_t)__popcll(mc) - n_due +
              (nq > kWave ? nq - kWave : 0u);
  } else {
    if (sorted_st) {  // sorted, but the new items do not extend it in order: the general path
      if (qn > kSparseQ * kWave) {
        defer(6u);
        return;
      }
      load_rest();
    }
    // ---- gather every item HTB serves this step (e < horizon) into lanes [0, ns)
    bool due_q[kSparseQ];
#pragma unroll
    for (uint32_t u = 0; u < kSparseQ; ++u) {
      due_q[u] = u * kWave + lane < qn && (w0_of(q[u]) & kEMask) < h;
      gather(due_q[u], q[u]);
    }
    const bool due_o = cand && (w0_of(io) & kEMask) < h, due_c = cand && cst == 2 && (w0_of(ic) & kEMask) < h;
    gather(due_o, io);
    gather(due_c, ic);
    // remaining items: everything not served, written back as the pool
    uint32_t nrem = qn + (uint32_t)__popcll(mc) + (uint32_t)__popcll(__ballot(cand && cst == 2)) - ns;
    if (over || nrem > kSparseQ * kWave) {
      defer(7u);
      return;
    }
    write_old_ring();
    // ---- write back the items HTB does not serve this step as the pool (no order needed); the
    // registers holding the queue are free for the rest
    auto keep = [&](bool f, const uint4& v) {
      const uint64_t m = __ballot(f);
      if (f) wq[wpos + (uint32_t)__popcll(m & below)] = v;
      wpos += (uint32_t)__popcll(m);
    };
#pragma unroll
    for (uint32_t u = 0; u < kSparseQ; ++u) keep(u * kWave + lane < qn && !due_q[u], q[u]);
    keep(cand && !due_o, io);
    keep(cand && cst == 2 && !due_c, ic);
    // ---- rank the served items by (e, seq, clone first) and put each in its rank's lane
    const bool hs = lane < ns;
    uint32_t rank = 0;
    for (uint32_t j = 0; j < ns; ++j) {
      const uint4 o = make_uint4(readlane32(x.x, j), readlane32(x.y, j), readlane32(x.z, j), 0u);
      rank += (hs && (item_lt(o, x) || (!item_lt(x, o) && j < lane))) ? 1u : 0u;
    }
    const uint32_t to = (hs ? rank : lane) & (kWave - 1);
    TG_FULL_EXEC("ds_permute");
    x = make_uint4((uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)x.x),
                   (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)x.y),
                   (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)x.z),
                   (uint32_t)__builtin_amdgcn_ds_permute((int)(to << 2), (int)x.w));
  }
  if (!fifo) ns_all = ns;
  // ---- HTB, records, receipts and the ring, for the served items in rounds of 64 lanes (more than
  // one only on the FIFO path: the queue's due prefix, then the due candidates, in order)
  uint64_t tat_c = st.tat;
  uint32_t emitted = 0, sched_n = 0, sk0 = 0, t_sched = 0, t_cor = 0, t_lost = 0;
  uint64_t bytes = 0;
  bool releasing = T_enq && !ring_stop;  // served entries departing before the last enqueue are released
  EmitOut eo = emit_out(a, s, sbeg, send);
  emit_claim(a, s, eo, ns_all, lane);
  for (uint32_t base = 0;; base += kWave) {
    const bool hs = lane < ns;
    // the destinations' forwarded masks, for the receipts folded in below (in flight during the scan)
    // (the 32-bit half of the mask that holds the record's flood bit: one register across the scan)
    const uint32_t fw_f = a.g_first ? x.z / a.g_degree : 0u;
    const uint32_t fw = a.g_first && hs && x.w - a.shard_begin < a.n_src && fw_f < 64u
                            ? reinterpret_cast<const uint32_t*>(a.g_fwd)[2ull * (x.w - a.shard_begin) + (fw_f >> 5)]
                            : 0u;
    // HTB: d = max(e, TAT before), TAT' = max(TAT, e - burst) + cost, one max-plus scan
    const uint64_t e = w0_of(x) & kEMask;
    const uint32_t xlen = x.y >> 14 & 0xFFFFu;
    const uint64_t c = ((uint64_t)xlen * pp.mult) >> (pp.shift_ext & 0xFFu);
    uint64_t A = hs ? c : 0, Bm = hs ? (e > pp.burst_ns ? e - pp.burst_ns : 0) + c : 0;
    scan_maxplus(A, Bm);
    const uint64_t ta = tat_c + A;
    const uint64_t tat_after = ta > Bm ? ta : Bm;
    const uint64_t before = shr1_u64(tat_after, tat_c);
    const uint64_t d = e > before ? e : before;
    if (ns) tat_c = readlane64(tat_after, ns - 1);
    stamp(a, s, lane, 3, __builtin_amdgcn_s_memrealtime());
    // records of the served items (dead destinations leave the sender and are lost)
    bool live = hs && x.w != kDeadDst;
    const bool dead = hs && !live;
    live = emit_record(a, eo, live, x, d, xlen, src, fw, fw_f, emitted, below);
    if (live) bytes += xlen;
    sched_n += (uint32_t)__popcll(__ballot(live));
    t_cor += (uint32_t)__popcll(__ballot(live && (x.y >> 31)));
    t_lost += (uint32_t)__popcll(__ballot(dead));
    // the served entries join the ring, behind the old entries kept; a prefix of them departing
    // before the last enqueue was released with the old ring (when that released all of it)
    if (releasing) {
      const uint32_t n1 = (uint32_t)__popcll(__ballot(hs && e < T_enq));
      const uint64_t m = __ballot(lane < n1 && d >= T_enq);
      if (m) {
        sk0 = base + (uint32_t)__builtin_ctzll(m);
        releasing = false;
      } else {
        sk0 = base + n1;
        releasing = n1 == kWave;
      }
    }
    if (hs && base + lane >= sk0) wr[(rh1 + old_kept + base + lane - sk0) & (kHeapCap - 1)] = d;
    if (base + kWave >= ns_all) break;
    // the next round (FIFO): the queue's due items from HBM, then the due candidates
    const uint32_t nb = base + kWave, k = nb + lane;
    x = k < fifo_nq ? gh[(qh + k) & (kHeapCap - 1)] : make_uint4(0, 0, 0, 0);
    ns = fifo_nq > nb ? (fifo_nq - nb < kWave ? fifo_nq - nb : kWave) : 0u;
    gather(due_f && cpos >= nb && cpos < nb + kWave, io);
  }
  t_sched = sched_n;
  const uint32_t rn_new = old_kept + ns_all - sk0;
  if (lane == 0) {
    SrcState ns_;
    ns_.tat = tat_c;
    ns_.heap_n = q_pack(wpos, 0);
    ns_.near_n = fifo ? wpos | new_head << 16 : 0;  // sorted in place (FIFO), or all of it pool, compacted
    ns_.ring_n = r_pack(rn_new, rh1);
    ns_.last_dup = st.last_dup;
    ns_.last_cor = st.last_cor;
    ns_.last_reo = st.last_reo;
    a.state[s] = ns_;
    a.emit_n[s] = emitted;
  }
  if (staged) a.verdict[sbeg + lane] = (uint8_t)vout;
  stamp(a, s, lane, 4, __builtin_amdgcn_s_memrealtime());
  stamp(a, s, lane, 5, ((uint64_t)s << 32) | n);
  stamp(a, s, lane, 7, ((uint64_t)qn << 32) | rn);
  // ---- statistics (per-lane counts reduced over the wave)
  const uint32_t vo = vout & 15u, vc = vout >> 4;
  uint32_t vcnt = 0;  // lane v < 8: packets and clones with verdict v
#pragma unroll
  for (uint32_t v = 0; v < 8; ++v) {
    const uint32_t t = ballot_count(staged && vo == v) + ballot_count(staged && vc == v);
    if (lane == v) vcnt = t;
  }
  const uint32_t t_clone = ballot_count(staged && vc != TGSIM_V_NONE);
  const uint64_t t_bytes = wave_sum(bytes);
  const bool err = __ballot(perr != 0) != 0;
  if (lane < 8 && vcnt) atomicAdd(&sc[kStVerdict0 + lane], (unsigned long long)vcnt);
  if (lane == 0) {
    const uint64_t qb = 16ull * qn + 8ull * rn + 16ull * wpos + 8ull * rn_new;
    // the per-window model counts the whole queue loaded and stored; the FIFO path left most of it
    const uint64_t q_kept = (fifo && qn + wpos > q_moved ? 16ull * (qn + wpos - q_moved) : 0ull) + 8ull * old_kept;
    if (q_kept) atomicAdd(&sc[kStCarrySkip], (unsigned long long)q_kept);
    if (n) atomicAdd(&sc[kStOffered], (unsigned long long)n);
    if (t_sched) atomicAdd(&sc[kStScheduled], (unsigned long long)t_sched);
    if (a.dst_bkt && t_sched > emitted) atomicAdd(&sc[kStBktRecs], (unsigned long long)(t_sched - emitted));
    if (t_clone) atomicAdd(&sc[kStCloned], (unsigned long long)t_clone);
    if (t_cor) atomicAdd(&sc[kStCorrupted], (unsigned long long)t_cor);
    if (t_lost) atomicAdd(&sc[kStLost], (unsigned long long)t_lost);
    if (t_bytes) atomicAdd(&sc[kStBytes], (unsigned long long)t_bytes);
    if (qb) atomicAdd(&sc[kStQueue], (unsigned long long)qb);
    if (err) {
      atomicOr(&a.stats[kStErr], (unsigned long long)kErrTimeOverflow);
      if (a.err_host)
        __hip_atomic_store(a.err_host, (uint64_t)kErrTimeOverflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// (A one-lane-per-source pass listing the active sources, so that idle peers cost no wave, was
// measured and dropped: 4.17-4.21 against 4.40-4.41 G pkt/s at 1M peers -- an idle wave exits after
// its first loads, cheaper than the pass over a million sources.)
// Sources per workgroup (one wave each) and their placement.  Workgroups are dealt round-robin
// over the 8 XCDs (MI355X_MICROARCH.md §Workgroup dispatch: blocks b and b + 8 share one), each with
// its own L2, so source s = blockIdx.x put neighbouring sources -- whose 32-B states, 64-B
// parameters, 8-B offsets, offered records and emit counts share 128-B lines -- on eight different
// L2s, each fetching the whole line.  With kSparseXcd the blocks of one XCD take one contiguous
// eighth of the sources, so a line is fetched by one L2.
constexpr uint32_t kSparseWpg = 1;
constexpr bool kSparseXcd = true;  // the 1M-peer window's simulate bytes -11 % at equal time
__host__ __device__ inline uint32_t sparse_blocks(uint32_t n_src) {
  const uint32_t nb = (n_src + kSparseWpg - 1) / kSparseWpg;
  return kSparseXcd ? (nb + 7) / 8 * 8 : nb;
}
__global__ __launch_bounds__(kWave * kSparseWpg, 7) void k_sim_sparse(SimArgs a) {
  // the source index must stay wave-uniform for the compiler (a VGPR index turns every per-source
  // load into a vector load: 126 VGPR spills at 7 waves per SIMD), hence readfirstlane
  const uint32_t b = blockIdx.x;
  const uint32_t w = kSparseWpg > 1 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0u;
  const uint32_t blk = kSparseXcd ? (b & 7u) * (gridDim.x >> 3) + (b >> 3) : b;
  const uint32_t s = blk * kSparseWpg + w;
  if (s < a.n_src) sparse_source(a, s);
}

// The general path for the worklist k_sim_sparse left: a grid-stride loop over the list (its
// length is read on the device, so the launch needs no host round trip).
__global__ __launch_bounds__(kWave) void k_sim_list(SimArgs a) {
  __shared__ SimLdsT<kHeapCap> lds;
  const uint32_t n = a.worklist[-4];
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t s = a.worklist[i];
    if (a.g_first) sim_source<false, kHeapCap, kModePlain, true, true>(a, s, s, lds);
    else sim_source<false, kHeapCap, kModePlain, false, true>(a, s, s, lds);
    wave_lds_sync();  // the write-back's LDS reads are done before the next source's loads land
  }
}

// ---------------------------------------------------------------------------------------------
// Longest-processing-time-first dispatch order: sources bucketed by the HTB records they emitted
// (8 buckets per octave), heaviest first (one workgroup, LDS counting sort; each weight is read
// once, so the order is a permutation whatever happens to the weights meanwhile).  Only the
// dispatch order changes; every source's result is independent of it.
constexpr uint32_t kOrderMax = 32768;  // sources the one-workgroup order kernel handles
__device__ __forceinline__ uint32_t weight_bucket(uint32_t c) {  // 0..255, monotone in c
  const uint32_t v = c | 1u, lz = __clz(v);
  return (31u - lz) * 8u + ((v << lz) >> 28 & 7u);
}

__global__ __launch_bounds__(1024) void k_order(const uint32_t* weight, uint32_t n, uint32_t* order) {
  __shared__ uint32_t cnt[256], base[256];
  __shared__ uint8_t key[kOrderMax];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) cnt[i] = 0;
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < n; s += blockDim.x) {
    const uint32_t k = 255u - weight_bucket(weight[s]);
    key[s] = (uint8_t)k;
    atomicAdd(&cnt[k], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int b = 0; b < 256; ++b) {
      base[b] = acc;
      acc += cnt[b];
    }
  }
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < n; s += blockDim.x) order[atomicAdd(&base[key[s]], 1u)] = s;
}

// ---------------------------------------------------------------------------------------------
// K9: configuration apply.  A removed data link (disconnect, re-addressing: docker_network.go:65-75,
// :84-87) takes its qdiscs with it: the netem queue and the departure ring are emptied (mask bit 4)
// and their items counted as flushed.
__global__ void k_apply_cfg(const CfgPatch* __restrict__ patches, uint32_t n, SrcParams* params,
                            SrcState* state, unsigned long long* stats) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const CfgPatch c = patches[i];
  params[c.s] = c.p;
  SrcState st = state[c.s];
  if (c.mask & 1u) st.last_dup = c.last_dup;
  if (c.mask & 2u) st.last_cor = c.last_cor;
  if (c.mask & 4u) st.last_reo = c.last_reo;
  if (c.mask & 8u) st.tat = 0;
  if (c.mask & 16u) {
    const uint32_t k = q_len(st) + q_parked(st) + r_len(st);
    if (k) atomicAdd(&stats[(size_t)(i % kStatCopies) * kStSlots + kStFlushed], (unsigned long long)k);
    st.heap_n = st.ring_n = st.near_n = 0;
  }
  state[c.s] = st;
}

// Packets still queued (not yet served by HTB) towards a destination whose link went away at this
// step boundary: they will leave the sender and find no port (or an address no longer in use), so
// they are marked dead in place; the queue order and occupancy are unchanged.  One wavefront per
// source, gone[] is per global peer.
// Compacts every queue the sparse kernel left in place (head slot != 0) back to slot 0, for the fused
// kernels' bounded loads: one wavefront per source, the whole queue in registers, then stored.
__global__ __launch_bounds__(256) void k_unrotate(uint4* heap, SrcState* state, uint32_t n_src) {
  const uint32_t s = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (s >= n_src) return;
  SrcState st = state[s];
  const uint32_t qh = q_head(st), qn = q_len(st);
  if (!qh) return;
  uint4* q = heap + (size_t)s * kHeapCap;
  uint4 v[kHeapCap / kWave];
#pragma unroll
  for (uint32_t u = 0; u < kHeapCap / kWave; ++u) {  // branch-free: a lane past the end re-reads the head
    const uint32_t k = u * kWave + lane;
    v[u] = q[(qh + (k < qn ? k : 0u)) & (kHeapCap - 1)];
  }
  __builtin_amdgcn_s_waitcnt(0);  // every lane's reads land before any lane writes
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (uint32_t u = 0; u < kHeapCap / kWave; ++u) {
    const uint32_t k = u * kWave + lane;
    if (k < qn) q[k] = v[u];
  }
  if (lane == 0) state[s].near_n = q_near(st);
}

__global__ __launch_bounds__(256) void k_purge(uint4* heap, uint4* wheel, const WheelMeta* wmeta, const SrcState* state,
                                               uint32_t n_src, const uint8_t* gone) {
  const uint32_t s = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (s >= n_src) return;
  const SrcState st = state[s];
  const uint32_t qn = q_len(st), qh = q_head(st);
  uint4* q = heap + (size_t)s * kHeapCap;
  for (uint32_t k = lane; k < qn; k += kWave) {
    const uint32_t j = (qh + k) & (kHeapCap - 1);
    const uint32_t d = q[j].w;
    if (d != kDeadDst && gone[d]) q[j].w = kDeadDst;
  }
  if (q_parked(st)) {  // and the items parked in the timing wheel, bucket by bucket
    const uint32_t cnt = wmeta[s].cnt[lane];
    uint4* w = wheel + (size_t)s * kWheelB * kWheelCB;
    for (uint32_t b = 0; b < kWheelB; ++b) {
      const uint32_t c = (uint32_t)__shfl((int)cnt, (int)b, 64);
      if (lane < c) {
        const uint32_t d = w[b * kWheelCB + lane].w;
        if (d != kDeadDst && gone[d]) w[b * kWheelCB + lane].w = kDeadDst;
      }
    }
  }
}

// K7 sync counters: table[state] += n on the device; the new value also goes to the pinned host
// mirror (barrier polls read it there) and to the pinned result word, then the pinned marker word
// is released with the call's sequence number (the host spins on it instead of synchronizing).
__global__ void k_signal(unsigned long long* table, uint64_t* mirror, uint32_t state, uint32_t n, uint64_t* result,
                         uint64_t* marker, uint64_t seq) {
  const unsigned long long v = atomicAdd(&table[state], (unsigned long long)n) + n;
  __hip_atomic_store(&mirror[state], (uint64_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(result, (uint64_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  __hip_atomic_store(marker, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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

// One wavefront per source, one lane per tick: the per-tick Poisson counts of 64 ticks are drawn
// in parallel and turned into record positions by a wave prefix sum.
__global__ __launch_bounds__(256) void k_gen_count(GenArgs g, uint64_t* counts) {
  const uint32_t s = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  const uint32_t lane = threadIdx.x % kWave;
  if (s >= g.n_src) return;
  const uint32_t src = g.shard_begin + s;
  uint32_t total = 0;
  if (g.n_peers >= 2) {
    for (uint32_t t = lane; t < g.n_ticks; t += kWave) {
      uint32_t r[4];
      philox(src, (uint32_t)(g.now_tick + t), 0x53544F52u, 0, g.k0, g.k1, r);
      total += poisson_count(g, r[0]);
    }
  }
  const uint64_t sum = wave_sum(total);
  if (lane == 0) counts[s] = sum;
}

__global__ __launch_bounds__(256) void k_gen_write(GenArgs g, const uint64_t* off, uint32_t* gen_seq, InRec* out) {
  const uint32_t s = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  const uint32_t lane = threadIdx.x % kWave;
  if (s >= g.n_src || g.n_peers < 2) return;
  const uint32_t src = g.shard_begin + s;
  uint64_t o = off[s];
  uint32_t seq = gen_seq[s];
  for (uint32_t t0 = 0; t0 < g.n_ticks; t0 += kWave) {
    const uint32_t t = t0 + lane;
    const uint32_t at = (uint32_t)(g.now_tick + t);
    uint32_t cnt = 0;
    if (t < g.n_ticks) {
      uint32_t r[4];
      philox(src, at, 0x53544F52u, 0, g.k0, g.k1, r);
      cnt = poisson_count(g, r[0]);
    }
    const int32_t incl = scan_sum_i32((int32_t)cnt);
    const uint32_t excl = (uint32_t)incl - cnt;
    for (uint32_t j = 0; j < cnt; ++j) {
      uint32_t q[4];
      philox(src, at, 0x53544F52u, j + 1, g.k0, g.k1, q);
      uint32_t d = q[0] % (g.n_peers - 1);
      d += d >= src;
      InRec rec;
      rec.dst = d;
      rec.seq = seq + excl + j;
      rec.tick = t;
      rec.len = 64u + q[1] % 1437u;
      out[o + excl + j] = rec;
    }
    const uint32_t tot = readlane32((uint32_t)incl, kWave - 1);
    o += tot;
    seq += tot;
  }
  if (lane == 0) gen_seq[s] = seq;
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

__device__ __forceinline__ void gossip_recv_one(const GossipArgs& g, const tgsim_delivery& r) {
  const uint32_t f = r.seq / g.degree;
  if (f >= g.n_floods || (r.flags & TGSIM_FLAG_CORRUPT)) return;
  const uint32_t s = r.dst - g.shard_begin;
  if (g.fwd[s] >> f & 1ull) return;
  uint64_t t = r.t_ns / g.tick_ns + 1;
  if (t > 0xFFFFFFFEull) t = 0xFFFFFFFEull;
  // the first receipt ever of flood f at s (exactly one delivery sees "none") marks it pending, so
  // the forward kernels read only the rows of peers with something to forward
  if (atomicMin(&g.first[(uint64_t)s * 64 + f], (uint32_t)t) == 0xFFFFFFFFu)
    atomicOr(reinterpret_cast<unsigned long long*>(&g.pend[s]), 1ull << f);
}

__global__ void k_gossip_recv(GossipArgs g, const tgsim_delivery* in, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) gossip_recv_one(g, in[i]);
}

// Same, with the record count on the device (a delivery whose size the host never reads).
__global__ __launch_bounds__(256) void k_gossip_recv_dev(GossipArgs g, const tgsim_delivery* in, const uint64_t* n_dev) {
  const uint64_t n = *n_dev;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    gossip_recv_one(g, in[i]);
}

// Receipts of the records a shard receives, straight from the inbound buffer (flat, or slotted
// chunks whose empty slots are skipped) before they are ordered: the next window's generation waits
// for this kernel only.  skip_own: records from this shard's own sources were folded in at emission.
__global__ __launch_bounds__(256) void k_gossip_recv_in(GossipArgs g, const tgsim_delivery* in, uint64_t n,
                                                        uint64_t slot, uint32_t skip_own) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (slot) {
      const uint64_t r = i / (slot + 1), j = i - r * (slot + 1);
      if (j == 0 || j > in[r * (slot + 1)].t_ns) continue;
    }
    const tgsim_delivery rec = in[i];
    if (skip_own && rec.src - g.shard_begin < g.n_src) continue;
    gossip_recv_one(g, rec);
  }
}

// The out-neighbour table (the hash of (seed, peer, k) once per peer and k, not at every forward).
__global__ __launch_bounds__(256) void k_gossip_nbr(GossipArgs g, uint32_t* nbr) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)g.n_src * g.degree) return;
  const uint32_t s = (uint32_t)(i / g.degree), k = (uint32_t)(i % g.degree);
  nbr[i] = gossip_neighbour(g, g.shard_begin + s, k);
}


// Floods due in [win0, win0 + n_ticks) for local peer s: lane f holds flood f's earliest receipt
// tick (a coalesced 256-B row); late receipts are flagged.  One wavefront handles kGossipPeers
// peers with all their rows in flight at once (one peer per wavefront left every wave waiting on
// two dependent loads: the launch was latency-bound at a third of the HBM rate).
constexpr uint32_t kGossipPeers = 8;
__device__ __forceinline__ bool gossip_due(const GossipArgs& g, uint64_t pend, uint32_t t, uint32_t lane) {
  const bool due = (pend >> lane & 1ull) && (uint64_t)t < g.win0 + g.n_ticks;
  if (due && (uint64_t)t < g.win0) atomicOr(g.err, 1u);
  return due;
}

// Rows of kGossipPeers peers: the pending masks first (8 B per peer), then only the receipt ticks of
// pending floods (most peers have none in a window: the 256-B rows stay unread).
__device__ __forceinline__ void gossip_rows(const GossipArgs& g, uint32_t s0, uint32_t lane, uint32_t (&t)[kGossipPeers],
                                            uint64_t (&pend)[kGossipPeers]) {
#pragma unroll
  for (uint32_t i = 0; i < kGossipPeers; ++i) pend[i] = s0 + i < g.n_src ? g.pend[s0 + i] : 0ull;
#pragma unroll
  for (uint32_t i = 0; i < kGossipPeers; ++i)
    t[i] = (pend[i] >> lane & 1ull) ? g.first[(uint64_t)(s0 + i) * 64 + lane] : 0xFFFFFFFFu;
}

__global__ __launch_bounds__(256) void k_gossip_count(GossipArgs g, uint64_t* counts) {
  const uint32_t s0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * kGossipPeers, lane = threadIdx.x & 63u;
  if (s0 >= g.n_src) return;
  uint32_t t[kGossipPeers];
  uint64_t pend[kGossipPeers];
  gossip_rows(g, s0, lane, t, pend);
  uint64_t c = 0;  // lane i: the count of peer s0 + i
#pragma unroll
  for (uint32_t i = 0; i < kGossipPeers; ++i) {
    const uint64_t n = (uint64_t)ballot_count(gossip_due(g, pend[i], t[i], lane)) * g.degree;
    if (lane == i) c = n;
  }
  if (lane < kGossipPeers && s0 + lane < g.n_src) counts[s0 + lane] = c;
}

// Degree <= 8: every load is issued up front, in two dependent levels (the masks, offsets and the
// 8 peers' neighbour lists, one per lane; then the pending receipt ticks), and nothing is read
// after the first store.  The 8 peers' records are contiguous in the CSR (off[s0] on), so they are
// written one record per lane, 64 consecutive records (1 KiB) per store: each due flood leaves its
// (flood, tick) in an LDS table at its rank, and lane L of round u writes record 64u + L.  (Written
// flood by flood -- 8 stores of 16 B per due flood at a 128-B stride, 64 store instructions per wave
// -- the kernel took 0.6 ms in the flood's peak windows, profiles/r06/gossip/.)
__global__ __launch_bounds__(256) void k_gossip_write8(GossipArgs g, const uint64_t* __restrict__ off,
                                                       InRec* __restrict__ out, uint64_t out_cap,
                                                       const uint64_t* total) {
  __shared__ uint32_t tab[4][kGossipPeers * kWave];  // per wave: [peer][rank] = flood | tick << 8
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t s0 = (blockIdx.x * 4 + wv) * kGossipPeers, lane = threadIdx.x & 63u;
  if (s0 >= g.n_src) return;
  if (total && *total > out_cap) return;  // written again into a larger buffer (resolve_gen)
  if (*g.err) return;  // a late receipt (k_gossip_count): the window is dropped, fwd/pend stay as they are
  const uint32_t deg = g.degree;
  const bool pl = lane < kGossipPeers && s0 + lane < g.n_src;  // lane i < 8: peer s0 + i's words
  const uint64_t pend_l = pl ? g.pend[s0 + lane] : 0ull;
  const uint64_t fwd_l = pl ? g.fwd[s0 + lane] : 0ull;
  const uint64_t o_base = off[s0];
  // lane i * deg + k: neighbour k of peer s0 + i
  const uint32_t nbr_l = lane < kGossipPeers * deg && s0 + lane / deg < g.n_src ? g.nbr[(uint64_t)s0 * deg + lane] : 0u;
  uint64_t pend[kGossipPeers];
  uint32_t t[kGossipPeers];
#pragma unroll
  for (uint32_t i = 0; i < kGossipPeers; ++i) {
    pend[i] = readlane64(pend_l, i);
    t[i] = (pend[i] >> lane & 1ull) ? g.first[(uint64_t)(s0 + i) * 64 + lane] : 0xFFFFFFFFu;
  }
  uint64_t due_l = 0;  // lane i: the floods peer s0 + i forwards in this window
  uint32_t pre[kGossipPeers + 1];  // records of the peers before peer i (wave-uniform)
  pre[0] = 0;
#pragma unroll
  for (uint32_t i = 0; i < kGossipPeers; ++i) {
    const bool me = gossip_due(g, pend[i], t[i], lane);
    const uint64_t due = __ballot(me);
    if (lane == i) due_l = due;
    pre[i + 1] = pre[i] + (uint32_t)__popcll(due) * deg;
    if (!due) continue;
    // earliest receipt first, ties by flood id (seq order within a tick)
    uint32_t rank = 0;
    for (uint64_t m = due; m; m &= m - 1) {
      const uint32_t j = (uint32_t)__builtin_ctzll(m);
      const uint32_t tj = readlane32(t[i], j);
      rank += (tj < t[i] || (tj == t[i] && j < lane)) ? 1u : 0u;
    }
    if (me) tab[wv][i * kWave + rank] = lane | (uint32_t)(t[i] - g.win0) << 8;
  }
  wave_lds_sync();
  const uint32_t n_rec = pre[kGossipPeers];
  for (uint32_t base = 0; base < n_rec; base += kWave) {
    const uint32_t r = base + lane;
    uint32_t i = 0;
#pragma unroll
    for (uint32_t p = 1; p < kGossipPeers; ++p) i += r >= pre[p] ? 1u : 0u;
    uint32_t pi = pre[0];
#pragma unroll
    for (uint32_t p = 1; p < kGossipPeers; ++p) pi = i == p ? pre[p] : pi;
    const uint32_t q = r - pi, j = q / deg, k = q - j * deg;
    const uint32_t e = r < n_rec ? tab[wv][i * kWave + j] : 0u;
    TG_FULL_EXEC("ds_bpermute");
    const uint32_t nb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((i * deg + k) << 2), (int)nbr_l);
    if (r < n_rec) {
      InRec rec;
      rec.dst = nb;
      rec.seq = (e & 63u) * deg + k;
      rec.tick = e >> 8;
      rec.len = g.msg_len;
      out[o_base + r] = rec;
    }
  }
  if (pl && due_l) {
    g.fwd[s0 + lane] = fwd_l | due_l;
    g.pend[s0 + lane] = pend_l & ~due_l;  // receipts for a later window stay pending
  }
}

__global__ __launch_bounds__(256) void k_gossip_write(GossipArgs g, const uint64_t* off, InRec* out,
                                                      uint64_t out_cap, const uint64_t* total) {
  const uint32_t s0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * kGossipPeers, lane = threadIdx.x & 63u;
  if (s0 >= g.n_src) return;
  if (total && *total > out_cap) return;  // written again into a larger buffer (resolve_gen)
  if (*g.err) return;  // a late receipt (k_gossip_count): the window is dropped, fwd/pend stay as they are
  uint32_t t[kGossipPeers];
  uint64_t pend[kGossipPeers];
  gossip_rows(g, s0, lane, t, pend);
#pragma unroll
  for (uint32_t i = 0; i < kGossipPeers; ++i) {
    const uint32_t s = s0 + i;
    const bool me = gossip_due(g, pend[i], t[i], lane);
    const uint64_t due = __ballot(me);
    if (!due) continue;
    if (lane == 0) {
      g.fwd[s] |= due;
      g.pend[s] = pend[i] & ~due;  // receipts for a later window stay pending
    }
    // earliest receipt first, ties by flood id (seq order within a tick)
    uint32_t rank = 0;
    for (uint64_t m = due; m; m &= m - 1) {
      const uint32_t j = (uint32_t)__builtin_ctzll(m);
      const uint32_t tj = readlane32(t[i], j);
      rank += (tj < t[i] || (tj == t[i] && j < lane)) ? 1u : 0u;
    }
    if (!me) continue;
    const uint32_t src = g.shard_begin + s;
    const uint64_t o = off[s] + (uint64_t)rank * g.degree;
    for (uint32_t k = 0; k < g.degree; ++k) {
      InRec rec;
      rec.dst = g.nbr ? g.nbr[(uint64_t)s * g.degree + k] : gossip_neighbour(g, src, k);
      rec.seq = lane * g.degree + k;
      rec.tick = (uint32_t)(t[i] - g.win0);
      rec.len = g.msg_len;
      out[o + k] = rec;
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
    sh[16] = acc;
  }
  __syncthreads();
  total = sh[16];
  const uint64_t r = x - v + sh[w];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void k_scan_local(const uint64_t* in, uint64_t* out, uint64_t n,
                                                    uint64_t* block_sums, uint64_t* clear) {
  __shared__ uint64_t sh[17];
  const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
  uint64_t v[4], s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = base + i < n ? in[base + i] : 0;
    s += v[i];
  }
  if (clear) {  // the counts, read, are zero again for the next histogram
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (base + i < n) clear[base + i] = 0;
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
  __shared__ uint64_t sh[17];
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

__global__ __launch_bounds__(256) void k_scan_add(uint64_t* out, uint64_t n, const uint64_t* sums,
                                                  uint64_t* pos, const uint64_t* total) {
  const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
  const uint64_t add = sums[blockIdx.x];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (base + i < n) {
      const uint64_t v = out[base + i] + add;
      out[base + i] = v;
      if (pos) pos[base + i] = v;
    }
  if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = *total;
}

// Exclusive scan of up to kSmallScan counts in one workgroup (out[n] = total; pos = a copy).
constexpr uint32_t kSmallScan = 16384;
__global__ __launch_bounds__(1024) void k_scan_small(const uint64_t* in, uint64_t* out, uint64_t n,
                                                     uint64_t* pos, uint64_t* total_out, uint64_t* clear) {
  __shared__ uint64_t sh[17];
  const uint32_t per = (uint32_t)((n + 1023) / 1024);  // <= 16
  const uint64_t base = (uint64_t)threadIdx.x * per;
  uint64_t v[16], s = 0;
#pragma unroll
  for (uint32_t i = 0; i < 16; ++i) {
    v[i] = (i < per && base + i < n) ? in[base + i] : 0;
    s += v[i];
  }
  if (clear) {
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i)
      if (i < per && base + i < n) clear[base + i] = 0;
  }
  uint64_t total;
  uint64_t pre = block_excl_scan(s, sh, total);
#pragma unroll
  for (uint32_t i = 0; i < 16; ++i) {
    if (i < per && base + i < n) {
      out[base + i] = pre;
      if (pos) pos[base + i] = pre;
    }
    pre += v[i];
  }
  if (threadIdx.x == 0) {
    out[n] = total;
    if (total_out) *total_out = total;
  }
}

// ---------------------------------------------------------------------------------------------
// Route: group the emitted records by the destination shard, deterministically and without
// contended atomics: per (rank, source) counts -> one exclusive scan over [rank][source] -> every
// source writes its records of rank r at off[r * S + s] in emission order.
struct RouteArgs {
  EmitRead emit;
  const uint32_t* emit_n;
  const uint64_t* off;           // CSR offsets of the step input (the emit regions, EmitRead)
  uint32_t n_src;
  uint32_t n_ranks;
  uint32_t bounds[9];
  uint64_t* cnt;                 // [n_ranks][n_src] records per (rank, source)
  const uint64_t* pos;           // exclusive scan of cnt
  tgsim_delivery* out;
  uint64_t out_cap;              // records beyond it are not written (the host reports -ENOSPC)
  uint64_t slot_cap;             // 0: flat, rank-major; else rank r's records at out[r * stride + 1 ..]
  uint64_t stride;               // slotted: records from one rank's chunk to the next (slot_cap + 1, or
                                 // n_win * (slot_cap + 1) for a fused group's window)
};

__device__ __forceinline__ uint32_t rank_of(const RouteArgs& a, uint32_t dst) {
  uint32_t r = 0;
  for (uint32_t i = 1; i < a.n_ranks; ++i) r += dst >= a.bounds[i];
  return r;
}

template <uint32_t W>  // wavefronts per workgroup, one source each
__global__ __launch_bounds__(64 * W) void k_route_count(RouteArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nw = gridDim.x * W;
  for (uint32_t s = blockIdx.x * W + (threadIdx.x >> 6); s < a.n_src; s += nw) {
    const uint32_t n = a.emit_n[s];
    if (a.n_ranks == 1) {
      if (lane == 0) a.cnt[s] = n;
      continue;
    }
    const uint64_t o0 = a.off[s], o1 = a.off[s + 1];
    const uint32_t pidx = n > 2 * (o1 - o0) + a.emit.r ? a.emit.pool_idx[s] : 0u;
    uint32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
      const uint32_t i = i0 + lane;
      const uint32_t rk = i < n ? rank_of(a, emit_rec(a.emit, s, o0, o1, i, pidx)->dst) : 0xFFFFFFFFu;
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

template <uint32_t W>
__global__ __launch_bounds__(64 * W) void k_route_scatter(RouteArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nw = gridDim.x * W;
  for (uint32_t s = blockIdx.x * W + (threadIdx.x >> 6); s < a.n_src; s += nw) {
    const uint32_t n = a.emit_n[s];
    const uint64_t o0 = a.off[s], o1 = a.off[s + 1];
    const uint32_t pidx = n > 2 * (o1 - o0) + a.emit.r ? a.emit.pool_idx[s] : 0u;
    uint64_t run[8], edge[8];
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) {
      run[q] = q < a.n_ranks ? a.pos[(size_t)q * a.n_src + s] : 0;
      edge[q] = (a.slot_cap && q < a.n_ranks) ? a.pos[(size_t)q * a.n_src] : 0;
    }
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
      const uint32_t i = i0 + lane;
      tgsim_delivery r;
      uint32_t rk = 0xFFFFFFFFu;
      if (i < n) {
        r = *emit_rec(a.emit, s, o0, o1, i, pidx);
        rk = rank_of(a, r.dst);
      }
      const uint64_t below = (1ull << lane) - 1;
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q) {
        const uint64_t m = __ballot(rk == q);
        if (rk == q) {
          const uint64_t p = run[q] + __popcll(m & below);
          if (a.slot_cap) {
            const uint64_t j = p - edge[q];
            if (j < a.slot_cap) a.out[q * a.stride + 1 + j] = r;
          } else if (p < a.out_cap) {
            a.out[p] = r;
          }
        }
        run[q] += __popcll(m);
      }
    }
  }
}

// Per-rank record ranges of the routed output: edges[r] = pos[r * n_src] (pos[n_ranks * n_src] is
// the total), gathered so the host reads them with one copy.
// Per-rank record edges straight into the host's pinned slot, then the slot's sequence word
// (system-scope release): the host polls that word instead of synchronizing on an event, which
// would also wait for the next step's k_sim queued behind this kernel.
__global__ void k_route_edges(const uint64_t* pos, uint32_t n_src, uint32_t n_ranks, uint64_t* slot, uint64_t seq,
                              tgsim_delivery* out, uint64_t slot_cap, uint32_t* overflow, uint64_t stride,
                              uint64_t* dev_counts) {
  const uint32_t r = threadIdx.x;
  if (r <= n_ranks) slot[r] = pos[(size_t)r * n_src];
  // per-rank counts in device memory as well: the exchange's count all-to-all reads them on the
  // device, so the host waits once, for the received counts, not first for these
  if (dev_counts && r < n_ranks) {
    const uint64_t c = pos[(size_t)(r + 1) * n_src] - pos[(size_t)r * n_src];
    dev_counts[r] = c;
    atomicMax(reinterpret_cast<unsigned long long*>(dev_counts + 8), (unsigned long long)c);  // the largest so far
  }
  if (slot_cap && r < n_ranks) {  // slotted output: each rank's chunk starts with its record count
    const uint64_t c = pos[(size_t)(r + 1) * n_src] - pos[(size_t)r * n_src];
    tgsim_delivery h = {};
    h.t_ns = c < slot_cap ? c : slot_cap;
    out[r * stride] = h;
    if (c > slot_cap) *overflow = 1u;  // sticky, in pinned host memory: the host fails with -ENOSPC
  }
  __threadfence_system();
  if (r == 0) __hip_atomic_store(&slot[15], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------------------------
// Delivery: counting sort by destination (counts -> exclusive scan -> scatter through per-dst
// cursors), then each destination's records ordered by (t, src, seq, clone first).
// Records addressed outside [dst_begin, dst_begin + n_dst) are skipped (the host reports them as
// -EINVAL when it reads the count; with discarded deliveries they are dropped).
// Slotted input (slot != 0): n = ranks * (slot + 1) records, each rank's chunk a count header then
// up to `slot` records; the slots past the count are skipped.
__device__ __forceinline__ bool slot_empty(const tgsim_delivery* in, uint64_t i, uint64_t slot) {
  if (!slot) return false;
  const uint64_t r = i / (slot + 1), j = i - r * (slot + 1);
  return j == 0 || j > in[r * (slot + 1)].t_ns;
}
// Histogram / cursor index of record i: its destination, in its window's segment block when the
// slotted input is a fused group's (chunk c = rank * n_win + window).
__device__ __forceinline__ uint64_t seg_of(uint64_t i, uint64_t slot, uint32_t n_win, uint32_t n_dst, uint32_t d) {
  if (n_win <= 1) return d;
  return (uint64_t)((i / (slot + 1)) % n_win) * n_dst + d;
}

__global__ void k_dst_hist(const tgsim_delivery* in, uint64_t n, uint32_t dst_begin, uint32_t n_dst, uint64_t* cnt,
                           uint64_t slot, uint32_t n_win) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || slot_empty(in, i, slot)) return;
  const uint32_t d = in[i].dst - dst_begin;
  if (d < n_dst) atomicAdd(reinterpret_cast<unsigned long long*>(&cnt[seg_of(i, slot, n_win, n_dst, d)]), 1ull);
}

// Slotted input, chunk by chunk: blockIdx.y is the chunk (count header, then up to `slot` records),
// the blocks of a chunk stride over the records its header announces.  The grid is sized for the
// records a chunk usually holds, not for its capacity: a chunk sized by a bound (the one-rank routed
// exchange reserves the whole step capacity) costs what it holds.
template <bool kScatter>
__global__ __launch_bounds__(256) void k_dst_slot(const tgsim_delivery* in, uint64_t slot, uint32_t dst_begin,
                                                  uint32_t n_dst, uint64_t* cnt_or_pos, tgsim_delivery* out,
                                                  uint32_t n_win) {
  const uint64_t c = blockIdx.y;
  const tgsim_delivery* ch = in + c * (slot + 1);
  const uint64_t n = ch[0].t_ns < slot ? ch[0].t_ns : slot;
  const uint64_t seg0 = n_win > 1 ? (c % n_win) * n_dst : 0;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const tgsim_delivery r = ch[1 + j];
    const uint32_t d = r.dst - dst_begin;
    if (d >= n_dst) continue;
    unsigned long long* w = reinterpret_cast<unsigned long long*>(&cnt_or_pos[seg0 + d]);
    if constexpr (kScatter) out[atomicAdd(w, 1ull)] = r;
    else atomicAdd(w, 1ull);
  }
}

// Flat input (records received from every shard): pos[] starts as the exclusive scan of counts.
__global__ void k_dst_scatter(const tgsim_delivery* in, uint64_t n, uint32_t dst_begin, uint32_t n_dst,
                              uint64_t* pos, tgsim_delivery* out, uint64_t slot, uint32_t n_win) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || slot_empty(in, i, slot)) return;
  const tgsim_delivery r = in[i];
  const uint32_t d = r.dst - dst_begin;
  if (d < n_dst)
    out[atomicAdd(reinterpret_cast<unsigned long long*>(&pos[seg_of(i, slot, n_win, n_dst, d)]), 1ull)] = r;
}

// Single shard: straight from k_sim's per-source emit regions (counts were taken by k_sim).
// A record's place in the scatter buffer: from its destination slot (records of a slotted window:
// doff[d] + slot, no atomic; a slot that did not fit claims one behind the first kSlotNone places
// with the cursor, which starts at doff[d]), else from the destination's cursor.
template <bool kSlot>
__device__ __forceinline__ uint64_t scatter_at(tgsim_delivery& r, uint32_t dst_begin, const uint64_t* doff,
                                               unsigned long long* pos) {
  const uint32_t d = r.dst - dst_begin;
  if constexpr (kSlot) {
    const uint64_t k = r.t_ns >> kSlotShift;
    r.t_ns &= kEMask;
    return k < kSlotNone ? doff[d] + k : kSlotNone + atomicAdd(&pos[d], 1ull);
  }
  return atomicAdd(&pos[d], 1ull);
}

template <bool kSlot>
__global__ __launch_bounds__(256) void k_local_scatter(EmitRead emit, const uint32_t* emit_n,
                                                       const uint64_t* off, uint32_t n_src, uint32_t dst_begin,
                                                       const uint64_t* doff, uint64_t* pos, tgsim_delivery* out) {
  if (emit.guard_total && *emit.guard_total > emit.guard_cap) return;  // (EmitRead::guard_total)
  const uint32_t lane = threadIdx.x & 63u, wpb = blockDim.x >> 6;  // (4 waves, or 1: see k_dst_sort_flat)
  const uint32_t nw = gridDim.x * wpb;
  for (uint32_t s = blockIdx.x * wpb + (threadIdx.x >> 6); s < n_src; s += nw) {
    const uint32_t n = emit_n[s];
    const uint64_t o0 = off[s], o1 = off[s + 1];
    const uint32_t pidx = n > 2 * (o1 - o0) + emit.r ? emit.pool_idx[s] : 0u;
    for (uint32_t i = lane; i < n; i += kWave) {
      tgsim_delivery r = *emit_rec(emit, s, o0, o1, i, pidx);
      out[scatter_at<kSlot>(r, dst_begin, doff, reinterpret_cast<unsigned long long*>(pos))] = r;
    }
  }
}

// The same with one lane per source (a few records each: the gossip windows): 64 sources' counts
// and offsets in one coalesced load, then their records four at a time in lockstep, every load,
// cursor atomic and store of a round independent of the others; a pass over the records'
// destinations first, so that a destination's records share one cursor atomic.  The wave per source above walks
// its sources one after another, each behind four dependent round trips with 57 of 64 lanes idle.
// kMode: kScatterEach one cursor atomic per record; kScatterAgg one per destination of a source (below);
// kScatterSlot records that carry their destination slot, no atomic.
constexpr int kScatterEach = 0, kScatterAgg = 1, kScatterSlot = 2;
template <int kMode>
__global__ __launch_bounds__(256) void k_local_scatter_ls(EmitRead emit,
                                                          const uint32_t* __restrict__ emit_n,
                                                          const uint64_t* __restrict__ off, uint32_t n_src,
                                                          uint32_t dst_begin, const uint64_t* __restrict__ doff,
                                                          uint64_t* pos, tgsim_delivery* __restrict__ out) {
  if (emit.guard_total && *emit.guard_total > emit.guard_cap) return;  // (EmitRead::guard_total)
  const uint32_t s = blockIdx.x * 256 + threadIdx.x;
  uint32_t n = 0, cap = 0;
  const tgsim_delivery* base = emit.base;  // the source's region: its first cap records
  const tgsim_delivery* over = emit.pool;  // the rest, from the pool
  if (s < n_src) {
    n = emit_n[s];
    const uint64_t o0 = off[s], o1 = off[s + 1];
    cap = (uint32_t)(2 * (o1 - o0)) + emit.r;
    base = emit.base + 2 * o0 + (uint64_t)emit.r * s;
    if (n > cap) over = emit.pool + emit.pool_idx[s];
  }
  auto rec = [&](uint32_t i) -> const tgsim_delivery& { return i < cap ? base[i] : over[i - cap]; };
  unsigned long long* p = reinterpret_cast<unsigned long long*>(pos);
  if constexpr (kMode != kScatterAgg) {  // one cursor atomic per record (storm shapes), or none (slots)
    for (uint32_t i = 0; __ballot(i < n); i += 4) {
      tgsim_delivery r[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u)
        if (i + u < n) r[u] = rec(i + u);
      uint64_t at[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u)
        if (i + u < n) at[u] = scatter_at<kMode == kScatterSlot>(r[u], dst_begin, doff, p);
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u)
        if (i + u < n) out[at[u]] = r[u];
    }
    return;
  }
  // A source's records of a window go to few destinations (a gossip peer's 8 neighbours): the first
  // kScatterDst distinct ones take one cursor atomic each for all their records (every cursor atomic
  // is a memory-side request; at the flood's peak one per record held this kernel at the memory
  // side's atomic rate, 28 M in 1.35 ms), the records of any other destination one each.
  constexpr uint32_t kScatterDst = 8;
  uint32_t dd[kScatterDst], cn[kScatterDst];
  uint32_t nd = 0;
#pragma unroll
  for (uint32_t j = 0; j < kScatterDst; ++j) dd[j] = cn[j] = 0;
  for (uint32_t i = 0; __ballot(i < n); i += 4) {
    uint32_t d[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) d[u] = i + u < n ? rec(i + u).dst : ~0u;
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      if (i + u >= n) continue;
      bool hit = false;
#pragma unroll
      for (uint32_t j = 0; j < kScatterDst; ++j)
        if (j < nd && dd[j] == d[u]) {
          cn[j]++;
          hit = true;
        }
      if (!hit && nd < kScatterDst) {
#pragma unroll
        for (uint32_t j = 0; j < kScatterDst; ++j)
          if (j == nd) {
            dd[j] = d[u];
            cn[j] = 1;
          }
        nd++;
      }
    }
  }
  uint64_t at[kScatterDst];
#pragma unroll
  for (uint32_t j = 0; j < kScatterDst; ++j)
    at[j] = j < nd ? atomicAdd(&p[dd[j] - dst_begin], (unsigned long long)cn[j]) : 0ull;
  for (uint32_t i = 0; __ballot(i < n); i += 4) {
    tgsim_delivery r[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u)
      if (i + u < n) r[u] = rec(i + u);
    uint64_t w[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      if (i + u >= n) continue;
      bool hit = false;
#pragma unroll
      for (uint32_t j = 0; j < kScatterDst; ++j)
        if (j < nd && dd[j] == r[u].dst) {
          w[u] = at[j]++;
          hit = true;
        }
      if (!hit) w[u] = atomicAdd(&p[r[u].dst - dst_begin], 1ull);
    }
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u)
      if (i + u < n) out[w[u]] = r[u];
  }
}

// K5 for a fused group (tgsim_step_n): the g windows' histograms are ONE array of g * N counts
// (window-major), so one scan, one scatter and one per-destination sort cover the whole group, and
// the sorted output is the windows' deliveries one after the other (the drain order of g
// tgsim_step calls).  Single-wave workgroups throughout: they fit beside the next group's
// k_sim_fused waves on a CU whose LDS those fill (no room for a 256- or 1024-thread block), so
// the delivery of one group runs under the next group's simulation.
__device__ __forceinline__ uint64_t scan_sum_u64(uint64_t v) {
#define STEP(C, R) v += dpp64<C, R>(0ull, v);
  TG_SCAN_STEPS(STEP)
#undef STEP
  return v;
}
__global__ __launch_bounds__(64) void k_scan_w1(const uint64_t* in, uint64_t n, uint64_t* blk) {
  const uint64_t base = (uint64_t)blockIdx.x * 1024;
  uint64_t s = 0;
#pragma unroll
  for (uint32_t u = 0; u < 16; ++u) {
    const uint64_t e = base + u * kWave + threadIdx.x;
    s += e < n ? in[e] : 0ull;
  }
  s = wave_sum(s);
  if (threadIdx.x == 0) blk[blockIdx.x] = s;
}
__global__ __launch_bounds__(64) void k_scan_w2(uint64_t* in, uint64_t n, const uint64_t* blk, uint64_t* out,
                                                uint64_t* pos, uint64_t* total_out, uint32_t clear) {
  const uint32_t lane = threadIdx.x;
  uint64_t pre = 0;
  for (uint32_t j = lane; j < blockIdx.x; j += kWave) pre += blk[j];
  pre = wave_sum(pre);
  const uint64_t base = (uint64_t)blockIdx.x * 1024;
  uint64_t x[16];
#pragma unroll
  for (uint32_t u = 0; u < 16; ++u) {
    const uint64_t e = base + u * kWave + lane;
    x[u] = e < n ? in[e] : 0ull;
  }
  if (clear) {  // the histogram free for its next window (k_scan_w1 of this scan has read it)
#pragma unroll
    for (uint32_t u = 0; u < 16; ++u) {
      const uint64_t e = base + u * kWave + lane;
      if (e < n) in[e] = 0;
    }
  }
#pragma unroll
  for (uint32_t u = 0; u < 16; ++u) {
    const uint64_t e = base + u * kWave + lane;
    const uint64_t incl = scan_sum_u64(x[u]);
    if (e < n) {
      out[e] = pre + incl - x[u];
      if (pos) pos[e] = pre + incl - x[u];
    }
    pre += readlane64(incl, kWave - 1);
  }
  if (blockIdx.x + 1 == gridDim.x && lane == 0) {
    out[n] = pre;
    if (total_out) *total_out = pre;
  }
}
__global__ __launch_bounds__(64) void k_local_scatter_group(GroupDeliver g) {
  const uint32_t w = blockIdx.x / g.n_src, s = blockIdx.x - w * g.n_src;
  const uint32_t n = g.emit_n[w][s];
  const tgsim_delivery* base = g.emit[w] + 2 * g.off[w][s] + (uint64_t)kHeapCap * s;
  unsigned long long* pos = reinterpret_cast<unsigned long long*>(g.pos + (uint64_t)w * g.n_dst);
  for (uint32_t i = threadIdx.x; i < n; i += kWave) {
    const tgsim_delivery r = base[i];
    g.out[atomicAdd(&pos[r.dst], 1ull)] = r;
  }
}

// Delivery order inside a destination: (t, src, seq, clone first).
__device__ __forceinline__ bool rec_lt(uint64_t ta, uint64_t qa, uint32_t ca, uint64_t tb, uint64_t qb, uint32_t cb) {
  return ta != tb ? ta < tb : (qa != qb ? qa < qb : ca < cb);
}
struct RecKey {
  uint64_t t, sq;
  uint32_t c;  // 0 for the clone, 1 for the original
};
__device__ __forceinline__ RecKey rec_key(const tgsim_delivery& r) {
  return RecKey{r.t_ns, ((uint64_t)r.src << 32) | r.seq, (r.flags & TGSIM_FLAG_DUP) ? 0u : 1u};
}

// Sorts the (up to) 64 records of [b, b + n) held one per lane: each lane counts the keys before
// its own (ties: lane order, which keeps runs stable).
__device__ __forceinline__ uint32_t wave_rank(const RecKey& k, uint32_t n, uint32_t lane) {
  uint32_t rank = 0;
  for (uint32_t j = 0; j < n; ++j) {
    const uint64_t t = readlane64(k.t, j), q = readlane64(k.sq, j);
    const uint32_t c = readlane32(k.c, j);
    rank += (rec_lt(t, q, c, k.t, k.sq, k.c) || (!rec_lt(k.t, k.sq, k.c, t, q, c) && j < lane)) ? 1u : 0u;
  }
  return rank;
}

// One wavefront per destination.  Up to 64 records: ranked in registers and stored at their rank.
// Longer segments: runs of 64 ranked the same way, then bottom-up merge passes between the scatter
// buffer and the output (each element's place = its index in its run + its rank in the other
// run, a binary search), so no scratch memory is needed.  The destination's count is reset to
// zero for the next step's histogram.
// A record this wave wrote earlier in the kernel, read from L2 (sc1: not from the CU's L1).
__device__ __forceinline__ tgsim_delivery load_rec_l2(const tgsim_delivery* p) {
  const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
  uint64_t w[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) w[i] = __hip_atomic_load(q + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_bit_cast(tgsim_delivery, w);
}

// ld(j): the segment's record j as the first pass reads it (by default in[b + j]; the bucketed
// delivery reads the first ones from the destination's bucket); in[b, b + n) is then the work space.
template <typename Ld>
__device__ void sort_segment_ld(tgsim_delivery* in, uint64_t b, uint32_t n, tgsim_delivery* out, uint32_t lane, Ld ld) {
  if (n <= kWave) {
    tgsim_delivery r;
    RecKey k{~0ull, ~0ull, 1u};
    if (lane < n) {
      r = ld(lane);
      k = rec_key(r);
    }
    const uint32_t rank = wave_rank(k, n, lane);
    if (lane < n) out[b + rank] = r;
  } else {
    // runs of 64, sorted in place in the scatter buffer
    for (uint32_t c0 = 0; c0 < n; c0 += kWave) {
      const uint32_t m = min(kWave, n - c0);
      tgsim_delivery r;
      RecKey k{~0ull, ~0ull, 1u};
      if (lane < m) {
        r = ld(c0 + lane);
        k = rec_key(r);
      }
      const uint32_t rank = wave_rank(k, m, lane);
      __builtin_amdgcn_s_waitcnt(0);  // every lane's read of the run lands before any write
      if (lane < m) in[b + c0 + rank] = r;
    }
    tgsim_delivery* src = in + b;
    tgsim_delivery* dst = out + b;
    for (uint32_t w = kWave; w < n; w <<= 1) {
      // this wave's writes of the previous level have landed in L2; its reads of them bypass the
      // CU's L1, which may hold a line another wave read before (segments share boundary lines)
      __builtin_amdgcn_s_waitcnt(0);
      for (uint32_t lo = 0; lo < n; lo += 2 * w) {
        const uint32_t mid = min(lo + w, n), hi = min(lo + 2 * w, n);
        for (uint32_t i = lo + lane; i < hi; i += kWave) {
          const tgsim_delivery r = load_rec_l2(src + i);
          const RecKey k = rec_key(r);
          const bool inA = i < mid;
          // rank in the other run: A elements count B keys < k, B elements count A keys <= k
          uint32_t a0 = inA ? mid : lo, a1 = inA ? hi : mid;
          while (a0 < a1) {
            const uint32_t m2 = (a0 + a1) >> 1;
            const RecKey o = rec_key(load_rec_l2(src + m2));
            const bool before = inA ? rec_lt(o.t, o.sq, o.c, k.t, k.sq, k.c)
                                    : !rec_lt(k.t, k.sq, k.c, o.t, o.sq, o.c);
            if (before) a0 = m2 + 1;
            else a1 = m2;
          }
          const uint32_t other = inA ? a0 - mid : a0 - lo;
          const uint32_t own = inA ? i - lo : i - mid;
          dst[lo + own + other] = r;
        }
      }
      tgsim_delivery* t = src;
      src = dst;
      dst = t;
    }
    if (src != out + b) {
      __builtin_amdgcn_s_waitcnt(0);
      for (uint32_t i = lane; i < n; i += kWave) out[b + i] = load_rec_l2(src + i);
    }
  }
}
__device__ __forceinline__ void sort_segment(tgsim_delivery* in, uint64_t b, uint32_t n, tgsim_delivery* out,
                                             uint32_t lane) {
  sort_segment_ld(in, b, n, out, lane, [&](uint32_t j) { return in[b + j]; });
}

// One destination per wavefront (segments of tens of records and more: storm).
template <uint32_t W>  // wavefronts per workgroup, one destination each
__global__ __launch_bounds__(64 * W) void k_dst_sort_wide(tgsim_delivery* in, const uint64_t* off, uint64_t* cnt,
                                                          uint32_t n_dst, tgsim_delivery* out) {
  const uint32_t d = blockIdx.x * W + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  if (d >= n_dst) return;
  const uint32_t n = (uint32_t)(off[d + 1] - off[d]);
  if (n == 0) return;
  sort_segment(in, off[d], n, out, lane);
  if (lane == 0 && cnt) cnt[d] = 0;
}

// A local delivery without a host round trip sizes its scatter and output buffers by a bound
// (tgsim_engine deliver_local_from); when the window's exact total (the scan's, on the device)
// exceeds it, this empties the window's record counts so that no later kernel writes past the
// buffers, and raises the sticky error (-ENOSPC at the next call).
__global__ __launch_bounds__(1024) void k_deliver_guard(const uint64_t* total, uint64_t cap, uint32_t* emit_n,
                                                       uint32_t n_src, uint64_t* cnt, uint64_t* off, uint32_t n_dst,
                                                       uint64_t* err_host) {
  if (*total <= cap) return;
  const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x, st = gridDim.x * blockDim.x;
  if (i0 == 0 && err_host) __hip_atomic_store(err_host, (uint64_t)kErrDeliverCap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (uint32_t i = i0; i < n_src; i += st) emit_n[i] = 0;
  for (uint32_t i = i0; i < n_dst; i += st) cnt[i] = 0;
  for (uint32_t i = i0; i <= n_dst; i += st) off[i] = 0;  // every segment empty: the sort writes nothing
}

// Per-destination order of the scattered records, flattened over the records instead of the
// destinations: a wavefront takes 64 consecutive records of the scatter buffer (a few destinations'
// segments, or part of one), so no lane idles on a short segment and a window at the flood's peak
// (~28 M records in 1 M segments) runs 440 k wave-iterations, not a wavefront per destination.  The
// keys of the 192 records around the chunk are staged in LDS: a segment of at most 64 records that
// holds one of the chunk's records lies inside them, and each record's rank is the number of its
// segment's keys before its own (ties, which the key order never has, by position).  A longer
// segment is sorted whole (sort_segment) by the wavefront holding its first record.  A persistent
// grid walks the chunks up to the device's total (off[n_dst]); the destination counts are not read.
// kW waves per workgroup (1: beside a running k_sim, whose waves leave no CU room for a 4-wave block
// with 15 KiB of LDS)
template <uint32_t kW>
__global__ __launch_bounds__(64 * kW) void k_dst_sort_flat(tgsim_delivery* in, const uint64_t* off, uint32_t n_dst,
                                                           uint32_t dst_begin, tgsim_delivery* out) {
  __shared__ uint64_t kt[kW][3 * kWave], kq[kW][3 * kWave];
  __shared__ uint32_t kc[kW][3 * kWave];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint64_t total = off[n_dst];
  const uint64_t n_chunks = (total + kWave - 1) / kWave;
  for (uint64_t c = (uint64_t)blockIdx.x * kW + wv; c < n_chunks; c += (uint64_t)gridDim.x * kW) {
    const uint64_t w0 = c * kWave;  // the staged window is [w0 - 64, w0 + 128)
    tgsim_delivery r;
#pragma unroll
    for (uint32_t u = 0; u < 3; ++u) {
      const uint64_t j = w0 + u * kWave + lane;  // + 64
      uint64_t t = ~0ull, q = ~0ull;
      uint32_t cl = 1u;
      if (j >= kWave && j - kWave < total) {
        const tgsim_delivery x = in[j - kWave];
        t = x.t_ns;
        q = ((uint64_t)x.src << 32) | x.seq;
        cl = (x.flags & TGSIM_FLAG_DUP) ? 0u : 1u;
        if (u == 1) r = x;
      }
      kt[wv][u * kWave + lane] = t;
      kq[wv][u * kWave + lane] = q;
      kc[wv][u * kWave + lane] = cl;
    }
    const uint64_t i = w0 + lane;
    const bool have = i < total;
    uint64_t sb = 0, se = 0;
    if (have) {
      const uint32_t d = r.dst - dst_begin;
      sb = off[d];
      se = off[d + 1];
    }
    wave_lds_sync();
    const bool small = have && se - sb <= kWave;
    if (small) {
      const uint64_t t = r.t_ns, q = ((uint64_t)r.src << 32) | r.seq;
      const uint32_t cl = (r.flags & TGSIM_FLAG_DUP) ? 0u : 1u;
      uint32_t rank = 0;
      for (uint64_t j = sb; j < se; ++j) {
        const uint32_t x = (uint32_t)(j + kWave - w0);
        const uint64_t ot = kt[wv][x], oq = kq[wv][x];
        const uint32_t oc = kc[wv][x];
        rank += (rec_lt(ot, oq, oc, t, q, cl) || (!rec_lt(t, q, cl, ot, oq, oc) && j < i)) ? 1u : 0u;
      }
      out[sb + rank] = r;
    }
    for (uint64_t big = __ballot(have && !small && i == sb); big; big &= big - 1) {
      const uint32_t gl = (uint32_t)__builtin_ctzll(big);
      const uint64_t b = readlane64(sb, gl);
      sort_segment(in, b, (uint32_t)(readlane64(se, gl) - b), out, lane);
    }
    wave_lds_sync();  // this chunk's LDS reads are done before the next chunk's writes
  }
}

// Per-destination order of a bucketed window (SimArgs::dst_bkt): destination d's first kC records (in
// slot order) are in its bucket, any more in the scatter buffer at doff[d] + slot (the slot scatter of
// the emit records).  kL = min(kC, 16) lanes per destination, kWave / kL destinations per wavefront,
// each lane kC / kL bucket entries, every load of a wavefront in flight at once (entries past a
// destination's count are read and ignored): a segment of at most kC records is ranked among its
// group's keys in LDS and each record stored at its rank; a longer one is sorted whole by the
// wavefront (sort_segment_ld, its first kC records read from the bucket).  No record pass before
// this kernel: the buckets are the simulate kernels' output.  A bounded delivery whose exact total
// (total) exceeds its buffers (cap) writes nothing and raises kErrDeliverCap.
template <uint32_t kC>
__global__ __launch_bounds__(256) void k_dst_sort_bkt(const tgsim_delivery* __restrict__ bkt, tgsim_delivery* sc,
                                                      const uint64_t* __restrict__ doff, uint32_t n_dst,
                                                      tgsim_delivery* __restrict__ out, const uint64_t* total,
                                                      uint64_t cap, uint64_t* err_host) {
  constexpr uint32_t kL = kC < 16 ? kC : 16;  // lanes per destination
  constexpr uint32_t kG = kWave / kL;         // destinations per wavefront
  constexpr uint32_t kR = kC / kL;            // bucket entries per lane
  __shared__ uint64_t kt[4][kG * kC], kq[4][kG * kC];
  __shared__ uint32_t kc[4][kG * kC];
  if (total && *total > cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && err_host)
      __hip_atomic_store(err_host, (uint64_t)kErrDeliverCap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t g = lane / kL, k = lane % kL;
  // a grid of resident workgroups walks the destination groups (launch_sort_bkt): workgroup slots are
  // taken once, not once per four wavefronts' worth of destinations, beside the simulate waves
  const uint32_t n_grp = (n_dst + 4 * kG - 1) / (4 * kG);
  for (uint32_t grp = blockIdx.x; grp < n_grp; grp += gridDim.x) {
    const uint32_t d0 = (grp * 4 + wv) * kG, d = d0 + g;
    const bool in_range = d < n_dst;
    uint64_t sb = 0, se = 0;
    tgsim_delivery r[kR];
    if (in_range) {
      sb = doff[d];
      se = doff[d + 1];
    }
    const uint64_t cnt = se - sb;
    const bool small = cnt <= kC;
    // only a destination's records are read, behind its offsets (read whole, the bucket lines past the
    // records were most of the kernel's HBM traffic at the 1M-peer flood: 935 MB per window for
    // 415 MB of records); a longer segment is read by sort_segment_ld below
    const uint32_t n_ld = small ? (uint32_t)cnt : 0u;
#pragma unroll
    for (uint32_t u = 0; u < kR; ++u)
      if (u * kL + k < n_ld) r[u] = bkt[(uint64_t)d * kC + u * kL + k];
#pragma unroll
    for (uint32_t u = 0; u < kR; ++u) {
      const uint32_t j = u * kL + k;
      const bool v = small && j < cnt;
      kt[wv][g * kC + j] = v ? r[u].t_ns : ~0ull;
      kq[wv][g * kC + j] = v ? ((uint64_t)r[u].src << 32) | r[u].seq : ~0ull;
      kc[wv][g * kC + j] = v ? ((r[u].flags & TGSIM_FLAG_DUP) ? 0u : 1u) : 1u;
    }
    wave_lds_sync();
#pragma unroll
    for (uint32_t u = 0; u < kR; ++u) {
      const uint32_t j = u * kL + k;
      if (small && j < cnt) {
        const uint64_t t = kt[wv][g * kC + j], q = kq[wv][g * kC + j];
        const uint32_t cl = kc[wv][g * kC + j];
        uint32_t rank = 0;
        for (uint32_t i = 0; i < (uint32_t)cnt; ++i) {
          const uint32_t x = g * kC + i;
          const uint64_t ot = kt[wv][x], oq = kq[wv][x];
          const uint32_t oc = kc[wv][x];
          rank += (rec_lt(ot, oq, oc, t, q, cl) || (!rec_lt(t, q, cl, ot, oq, oc) && i < j)) ? 1u : 0u;
        }
        out[sb + rank] = r[u];
      }
    }
    for (uint64_t big = __ballot(k == 0 && cnt > kC); big; big &= big - 1) {
      const uint32_t gl = (uint32_t)__builtin_ctzll(big);
      const uint64_t b = readlane64(sb, gl);
      const uint32_t n = (uint32_t)(readlane64(se, gl) - b);
      const tgsim_delivery* bk = bkt + (uint64_t)(d0 + gl / kL) * kC;
      sort_segment_ld(sc, b, n, out, lane, [&](uint32_t j) { return j < kC ? bk[j] : sc[b + j]; });
    }
    wave_lds_sync();  // this group's LDS reads are done before the next group's writes
  }
}

// ---------------------------------------------------------------------------------------------
// K8 metrics (opt-in): per-instance counters and log2 histograms folded after each step, one
// wavefront per instance, no atomics on the counters (an instance is one wavefront's).
__device__ __forceinline__ uint32_t log2_bin(uint64_t x) {  // 0: none, b: 2^(b-1) <= x < 2^b
  const uint32_t b = x ? 64u - (uint32_t)__builtin_clzll(x) : 0u;
  return b < kMetricBins ? b : kMetricBins - 1;
}

__device__ __forceinline__ uint32_t wave_total(uint32_t v) {
  return readlane32((uint32_t)scan_sum_i32((int32_t)v), kWave - 1);
}

// Per source: offered packets and bytes, verdict counts (originals + clones), HTB records served
// and their bytes (the step's emit region), and the backlog histogram at the step end.
__global__ __launch_bounds__(256) void k_metrics_src(MetricsArgs m) {
  const uint32_t s = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (s >= m.n_src) return;
  const uint64_t b0 = m.off[s], b1 = m.off[s + 1];
  uint32_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t bytes = 0;
  for (uint64_t i = b0 + lane; i < b1; i += kWave) {
    const uint32_t vb = m.verdict[i], vo = vb & 15u, vc = vb >> 4;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) v[k] += (vo == k ? 1u : 0u) + (vc == k ? 1u : 0u);
    bytes += m.in[i].len & 0xFFFFu;
  }
  const uint32_t n_emit = m.emit_n[s];
  const uint32_t pidx = n_emit > 2 * (b1 - b0) + m.emit.r ? m.emit.pool_idx[s] : 0u;
  uint64_t sbytes = 0;
  for (uint32_t i = lane; i < n_emit; i += kWave) sbytes += emit_rec(m.emit, s, b0, b1, i, pidx)->len;
  unsigned long long* row = m.src + (size_t)s * kMetricSrcWords;
  uint32_t tv[8];
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) tv[k] = wave_total(v[k]);
  const uint64_t tb = wave_sum(bytes), ts = wave_sum(sbytes);
  if (lane == 0) {
    row[0] += b1 - b0;
    row[1] += tb;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) row[2 + k] += tv[k];
    row[10] += n_emit;
    row[11] += ts;
    const SrcState st = m.state[s];
    atomicAdd(&m.hist[log2_bin((uint64_t)q_len(st) + q_parked(st) + r_len(st))], 1ull);
  }
}

// Per destination of this shard: the records delivered to it in this step (its segment of the
// delivery-ordered output) and their bytes; histogram of the per-destination record counts.
__global__ __launch_bounds__(256) void k_metrics_dst(const tgsim_delivery* recs, const uint64_t* off, uint32_t n_dst,
                                                     unsigned long long* dst, unsigned long long* hist) {
  const uint32_t d = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (d >= n_dst) return;
  const uint64_t b0 = off[d], b1 = off[d + 1];
  uint64_t bytes = 0;
  for (uint64_t i = b0 + lane; i < b1; i += kWave) bytes += recs[i].len;
  const uint64_t tb = wave_sum(bytes);
  if (lane == 0) {
    dst[(size_t)d * kMetricDstWords] += b1 - b0;
    dst[(size_t)d * kMetricDstWords + 1] += tb;
    atomicAdd(&hist[kMetricBins + log2_bin(b1 - b0)], 1ull);
  }
}

// ---------------------------------------------------------------------------------------------
// Host-side launchers.

void launch_sim(const SimArgs& a, uint32_t n_wg, hipStream_t st) {
  if (a.g_first) hipLaunchKernelGGL(k_sim_recv, dim3(n_wg), dim3(kWave), 0, st, a);
  else hipLaunchKernelGGL(k_sim, dim3(n_wg), dim3(kWave), 0, st, a);  // n_wg = ceil(n_src / kSpw)
}

void launch_sim_fused(const SimArgs& a, const FusedArgs& f, uint32_t n_wg, hipStream_t st) {
  const uint32_t total = f.n_win * a.n_src;  // tickets
  FusedSim fs;
  for (uint32_t k = 0; k < kFuseMax; ++k) {
    fs.w[k] = a;
    if (k >= f.n_win) continue;
    const FusedWindow& w = f.w[k];
    fs.w[k].off = w.off;
    fs.w[k].in = w.in;
    fs.w[k].verdict = w.verdict;
    fs.w[k].emit = w.emit;
    fs.w[k].emit_n = w.emit_n;
    fs.w[k].dst_cnt = w.dst_cnt;
    fs.w[k].t0_ns = w.t0_ns;
    fs.w[k].horizon_ns = w.horizon_ns;
  }
  const dim3 grid(f.persistent && n_wg < total ? n_wg : total);
  hipLaunchKernelGGL(k_sim_fused, grid, dim3(kWave), 0, st, fs, f);
}

uint32_t sim_fused_resident() {
  int dev = 0, per_cu = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sim_fused, kWave, 0) != hipSuccess || per_cu <= 0)
    return 2048;
  return (uint32_t)(per_cu * cus);
}

// Behind the last sparse kernel: the deferral counts to pinned host memory (the next step's sparse/dense
// choice reads them without waiting) and every counter zeroed for the next sparse step.
__global__ void k_work_done(uint32_t* work, uint32_t* host) {
  const uint32_t i = threadIdx.x;
  if (i < 2) __hip_atomic_store(&host[i], work[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (i < 4) work[i] = 0u;
}

void launch_sim_sparse(const SimArgs& a, hipStream_t st, uint32_t* work_host, uint32_t list_hint) {
  if (!a.n_src) return;
  hipLaunchKernelGGL(k_sim_sparse, dim3(sparse_blocks(a.n_src)), dim3(kWave * kSparseWpg), 0, st, a);
  // (grids of 5,120 and 10,240 waves: the same 1M-peer window, within noise)
  hipLaunchKernelGGL(k_sim_multi, dim3(a.n_src < 2048 ? a.n_src : 2048), dim3(kWave), 0, st, a);
  // k_sim_list's grid from the last sparse step's deferrals (its length is read on the device; a
  // grid-stride loop covers any count): each of its workgroups needs 16 KiB of LDS, and at the
  // 1M-peer flood's peak, with the delivery kernels holding the LDS, 16,384 workgroups that found an
  // empty list still waited 1.1 ms for it (the simulate stream's critical path)
  const uint32_t want = std::max<uint32_t>(64u, 2u * list_hint);
  const uint32_t lg = std::min<uint32_t>(std::min<uint32_t>(a.n_src, 16384u), want);
  hipLaunchKernelGGL(k_sim_list, dim3(lg), dim3(kWave), 0, st, a);
  hipLaunchKernelGGL(k_work_done, dim3(1), dim3(64), 0, st, a.worklist - 4, work_host);
}

void launch_order(const uint32_t* weight, uint32_t n, uint32_t* order, hipStream_t st) {
  if (n > kOrderMax) return;
  hipLaunchKernelGGL(k_order, dim3(1), dim3(1024), 0, st, weight, n, order);
}

void launch_apply_cfg(const CfgPatch* p, uint32_t n, SrcParams* params, SrcState* state,
                      unsigned long long* stats, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_apply_cfg, dim3((n + 255) / 256), dim3(256), 0, st, p, n, params, state, stats);
}

void launch_unrotate(uint4* heap, SrcState* state, uint32_t n_src, hipStream_t st) {
  if (n_src) hipLaunchKernelGGL(k_unrotate, dim3((n_src + 3) / 4), dim3(256), 0, st, heap, state, n_src);
}

void launch_purge(uint4* heap, uint4* wheel, const WheelMeta* wmeta, const SrcState* state, uint32_t n_src,
                  const uint8_t* gone, hipStream_t st) {
  if (n_src) hipLaunchKernelGGL(k_purge, dim3((n_src + 3) / 4), dim3(256), 0, st, heap, wheel, wmeta, state, n_src, gone);
}

// Publishes *v0 (and *v1 when given) into pinned host words, then the sequence number (release):
// the host spins on slot[2] instead of synchronizing a stream.
__global__ void k_publish(const uint64_t* v0, const uint32_t* v1, uint64_t* slot, uint64_t seq) {
  __hip_atomic_store(&slot[0], *v0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&slot[1], (uint64_t)(v1 ? *v1 : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  __hip_atomic_store(&slot[2], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// n device words to pinned host memory, then the sequence word host[n] (release, system scope): the
// host spins on one word instead of synchronizing a stream.
__global__ void k_publish_words(const uint64_t* src, uint32_t n, uint64_t* host, uint64_t seq) {
  const uint32_t i = threadIdx.x;
  if (i < n) __hip_atomic_store(&host[i], src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  __syncthreads();
  if (i == 0) __hip_atomic_store(&host[n], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_publish_words(const uint64_t* src, uint32_t n, uint64_t* host, uint64_t seq, hipStream_t st) {
  hipLaunchKernelGGL(k_publish_words, dim3(1), dim3(64), 0, st, src, n, host, seq);
}

void launch_publish(const uint64_t* v0, const uint32_t* v1, uint64_t* slot, uint64_t seq, hipStream_t st) {
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(1), 0, st, v0, v1, slot, seq);
}

void launch_signal(unsigned long long* table, uint64_t* mirror, uint32_t state, uint32_t n, uint64_t* result,
                   uint64_t* marker, uint64_t seq, hipStream_t st) {
  hipLaunchKernelGGL(k_signal, dim3(1), dim3(1), 0, st, table, mirror, state, n, result, marker, seq);
}

void launch_gen(const GenArgsHost& h, uint64_t* counts, const uint64_t* off, uint32_t* gen_seq,
                InRec* out, int phase, hipStream_t st) {
  GenArgs g;
  for (int i = 0; i < 16; ++i) g.tab[i] = h.tab[i];
  g.k0 = h.k0; g.k1 = h.k1; g.n_src = h.n_src; g.shard_begin = h.shard_begin;
  g.n_peers = h.n_peers; g.n_ticks = h.n_ticks; g.now_tick = h.now_tick;
  const dim3 wgrid((h.n_src + 3) / 4), wblk(256);  // one wavefront per source
  if (phase == 0) hipLaunchKernelGGL(k_gen_count, wgrid, wblk, 0, st, g, counts);
  else hipLaunchKernelGGL(k_gen_write, wgrid, wblk, 0, st, g, off, gen_seq, out);
}

void launch_metrics_src(const MetricsArgs& m, hipStream_t st) {
  if (m.n_src) hipLaunchKernelGGL(k_metrics_src, dim3((m.n_src + 3) / 4), dim3(256), 0, st, m);
}

void launch_metrics_dst(const tgsim_delivery* recs, const uint64_t* off, uint32_t n_dst, unsigned long long* dst,
                        unsigned long long* hist, hipStream_t st) {
  if (n_dst) hipLaunchKernelGGL(k_metrics_dst, dim3((n_dst + 3) / 4), dim3(256), 0, st, recs, off, n_dst, dst, hist);
}

void launch_gossip_nbr(const GossipArgs& g, uint32_t* nbr, hipStream_t st) {
  const uint64_t n = (uint64_t)g.n_src * g.degree;
  if (n) hipLaunchKernelGGL(k_gossip_nbr, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, g, nbr);
}

void launch_gossip_recv_in(const GossipArgs& g, const tgsim_delivery* recs, uint64_t n, uint64_t slot, bool skip_own,
                           hipStream_t st) {
  if (!n) return;
  const uint64_t wgs = std::min<uint64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_gossip_recv_in, dim3((uint32_t)wgs), dim3(256), 0, st, g, recs, n, slot, skip_own ? 1u : 0u);
}

void launch_gossip_recv_dev(const GossipArgs& g, const tgsim_delivery* recs, const uint64_t* n_dev, hipStream_t st) {
  hipLaunchKernelGGL(k_gossip_recv_dev, dim3(2048), dim3(256), 0, st, g, recs, n_dev);
}

void launch_gossip(const GossipArgs& g, const tgsim_delivery* recs, uint64_t n, uint64_t* counts,
                   const uint64_t* off, InRec* out, int phase, hipStream_t st, uint64_t out_cap,
                   const uint64_t* total) {
  if (phase == 0) {
    if (n) hipLaunchKernelGGL(k_gossip_recv, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, g, recs, n);
    return;
  }
  const uint32_t waves = (g.n_src + kGossipPeers - 1) / kGossipPeers;  // kGossipPeers peers per wavefront
  const dim3 grid((waves + 3) / 4), blk(256);
  if (phase == 1) hipLaunchKernelGGL(k_gossip_count, grid, blk, 0, st, g, counts);
  else if (g.nbr && g.degree <= kWave / kGossipPeers)
    hipLaunchKernelGGL(k_gossip_write8, grid, blk, 0, st, g, off, out, out_cap, total);
  else
    hipLaunchKernelGGL(k_gossip_write, grid, blk, 0, st, g, off, out, out_cap, total);
}

void launch_scan(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* block_sums,
                 uint64_t* total, hipStream_t st, uint64_t* pos, uint64_t* clear) {
  if (n == 0) {
    (void)hipMemsetAsync(out, 0, sizeof(uint64_t), st);
    if (total) (void)hipMemsetAsync(total, 0, sizeof(uint64_t), st);
    return;
  }
  if (n <= kSmallScan) {
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(1024), 0, st, in, out, n, pos, total, clear);
    return;
  }
  const uint64_t nb = (n + 1023) / 1024;
  hipLaunchKernelGGL(k_scan_local, dim3((uint32_t)nb), dim3(256), 0, st, in, out, n, block_sums, clear);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(256), 0, st, block_sums, nb, total);
  hipLaunchKernelGGL(k_scan_add, dim3((uint32_t)nb), dim3(256), 0, st, out, n, block_sums, pos,
                     (const uint64_t*)total);
}

void launch_route_edges(const uint64_t* pos, uint32_t n_src, uint32_t n_ranks, uint64_t* slot, uint64_t seq,
                        hipStream_t st, tgsim_delivery* out, uint64_t slot_cap, uint32_t* overflow, uint64_t chunk_stride,
                        uint64_t* dev_counts) {
  hipLaunchKernelGGL(k_route_edges, dim3(1), dim3(64), 0, st, pos, n_src, n_ranks, slot, seq, out, slot_cap,
                     overflow, chunk_stride ? chunk_stride : slot_cap + 1, dev_counts);
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
  a.out_cap = h.out_cap;
  a.slot_cap = h.slot_cap;
  a.stride = h.chunk_stride ? h.chunk_stride : h.slot_cap + 1;
  if (h.waves_per_block == 1) {  // one wave per source, single-wave workgroups
    const uint32_t grid = h.n_src ? h.n_src : 1;
    if (phase == 0) hipLaunchKernelGGL(k_route_count<1>, dim3(grid), dim3(64), 0, st, a);
    else hipLaunchKernelGGL(k_route_scatter<1>, dim3(grid), dim3(64), 0, st, a);
    return;
  }
  uint32_t grid = (h.n_src + 3) / 4;
  if (grid > 4096) grid = 4096;
  if (grid == 0) grid = 1;
  if (phase == 0) hipLaunchKernelGGL(k_route_count<4>, dim3(grid), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(k_route_scatter<4>, dim3(grid), dim3(256), 0, st, a);
}

// Blocks per chunk of a slotted input: enough for the chunk's expected records (slot_hint, e.g. the
// last exchange's largest count) at 4 records per thread, at most 1,024.
static uint32_t slot_blocks(uint64_t slot, uint64_t slot_hint) {
  const uint64_t want = (slot_hint && slot_hint < slot ? slot_hint : slot) / 1024 + 1;
  return (uint32_t)(want < 1024 ? want : 1024);
}

void launch_dst_slot(const tgsim_delivery* in, uint64_t n_chunks, uint64_t slot, uint64_t slot_hint, uint32_t dst_begin,
                     uint32_t n_dst, uint64_t* cnt_or_pos, tgsim_delivery* out, hipStream_t st, uint32_t n_win) {
  if (!n_chunks) return;
  // a fused group's delivery runs beside k_sim_fused: single-wave workgroups fit where a CU has no
  // room left for a 256-thread block
  const uint32_t b = n_win > 1 ? 64u : 256u;
  const dim3 grid(slot_blocks(slot, slot_hint) * (256u / b), (uint32_t)n_chunks);
  if (out)
    hipLaunchKernelGGL(k_dst_slot<true>, grid, dim3(b), 0, st, in, slot, dst_begin, n_dst, cnt_or_pos, out, n_win);
  else
    hipLaunchKernelGGL(k_dst_slot<false>, grid, dim3(b), 0, st, in, slot, dst_begin, n_dst, cnt_or_pos, out, n_win);
}

void launch_dst_hist(const tgsim_delivery* in, uint64_t n, uint32_t dst_begin, uint32_t n_dst, uint64_t* cnt,
                     hipStream_t st, uint64_t slot, uint32_t n_win) {
  if (!n) return;
  const uint32_t b = n_win > 1 ? 64u : 256u;  // a fused group's: single-wave workgroups
  hipLaunchKernelGGL(k_dst_hist, dim3((uint32_t)((n + b - 1) / b)), dim3(b), 0, st, in, n, dst_begin, n_dst, cnt,
                     slot, n_win);
}

void launch_dst_scatter(const tgsim_delivery* in, uint64_t n, uint32_t dst_begin, uint32_t n_dst, uint64_t* pos,
                        tgsim_delivery* out, hipStream_t st, uint64_t slot, uint32_t n_win) {
  if (!n) return;
  const uint32_t b = n_win > 1 ? 64u : 256u;
  hipLaunchKernelGGL(k_dst_scatter, dim3((uint32_t)((n + b - 1) / b)), dim3(b), 0, st, in, n, dst_begin, n_dst,
                     pos, out, slot, n_win);
}

void launch_deliver_guard(const uint64_t* total, uint64_t cap, uint32_t* emit_n, uint32_t n_src, uint64_t* cnt,
                          uint64_t* off, uint32_t n_dst, uint64_t* err_host, hipStream_t st) {
  // one workgroup: the check needs one dispatch slot (on the low-priority delivery stream behind a
  // million-wave k_sim_sparse, 1,024 of them waited up to 1.5 ms); the clearing is the error path
  hipLaunchKernelGGL(k_deliver_guard, dim3(1), dim3(1024), 0, st, total, cap, emit_n, n_src, cnt, off, n_dst, err_host);
}

constexpr uint32_t kLaneScatterMin = 65536;  // sources: below, the wavefront-per-source scatter
void launch_local_scatter(const EmitRead& emit, const uint32_t* emit_n, const uint64_t* off, uint32_t n_src,
                          uint32_t dst_begin, const uint64_t* doff, uint64_t* pos, tgsim_delivery* out,
                          hipStream_t st, uint64_t n_hint, bool few_dst, bool single_wave) {
  if (!n_src) return;
  const uint32_t lwg = (n_src + 255) / 256;
  // up to tens of records per source and enough sources to fill the chip with one lane each (gossip at
  // 1M peers, even at the flood's peak): one lane per source.  With fewer sources (the sub-capacity
  // storm's 10,000: 40 workgroups) a wavefront per source spreads the records over 10,000 waves
  // (A/B: 1.17-1.19 against 1.09-1.12 G pkt/s)
  if (n_hint <= 64ull * n_src && n_src >= kLaneScatterMin) {
    // few_dst (gossip: a peer forwards to its neighbours): one cursor atomic per destination of a
    // source (1M-peer gossip +1-2 %); with records to many destinations that pass over the records
    // costs more than it saves (sub-capacity storm 1.09 against 1.15-1.17 G pkt/s)
    // (records with their destination slot need no cursor at all)
    if (emit.slot)
      hipLaunchKernelGGL(k_local_scatter_ls<kScatterSlot>, dim3(lwg), dim3(256), 0, st, emit, emit_n, off, n_src,
                         dst_begin, doff, pos, out);
    else if (few_dst)
      hipLaunchKernelGGL(k_local_scatter_ls<kScatterAgg>, dim3(lwg), dim3(256), 0, st, emit, emit_n, off, n_src,
                         dst_begin, doff, pos, out);
    else
      hipLaunchKernelGGL(k_local_scatter_ls<kScatterEach>, dim3(lwg), dim3(256), 0, st, emit, emit_n, off, n_src,
                         dst_begin, doff, pos, out);
    return;
  }
  const uint32_t wpb = single_wave ? 1u : 4u, wgs = std::min<uint32_t>((n_src + wpb - 1) / wpb, 16384 / wpb);
  if (emit.slot)
    hipLaunchKernelGGL(k_local_scatter<true>, dim3(wgs), dim3(64 * wpb), 0, st, emit, emit_n, off, n_src, dst_begin,
                       doff, pos, out);
  else
    hipLaunchKernelGGL(k_local_scatter<false>, dim3(wgs), dim3(64 * wpb), 0, st, emit, emit_n, off, n_src, dst_begin,
                       doff, pos, out);
}

void launch_dst_sort(tgsim_delivery* in, const uint64_t* off, uint64_t* cnt, uint32_t n_dst,
                     tgsim_delivery* out, hipStream_t st, uint64_t n_hint, uint32_t dst_begin, bool single_wave) {
  if (!n_dst) return;
  if (!cnt && single_wave) {
    const uint64_t chunks = (n_hint + kWave - 1) / kWave;
    hipLaunchKernelGGL(k_dst_sort_flat<1>, dim3((uint32_t)(chunks < 32768 ? (chunks ? chunks : 1) : 32768)), dim3(64), 0,
                       st, in, off, n_dst, dst_begin, out);
    return;
  }
  if (!cnt && n_hint <= 48ull * n_dst) {
    // up to tens of records per destination (gossip, sparse windows): 64 records per wave-iteration
    // over the records, on a grid of at most 8,192 workgroups of 4 waves.  At the 1M-peer flood's
    // peak it replaced a wavefront per destination (or lane groups of 8-32 for short segments):
    // 4.66-4.70 against 4.57-4.60 G pkt/s
    const uint64_t chunks = (n_hint + kWave - 1) / kWave, wgs = (chunks + 3) / 4;
    hipLaunchKernelGGL(k_dst_sort_flat<4>, dim3((uint32_t)(wgs < 8192 ? (wgs ? wgs : 1) : 8192)), dim3(256), 0, st, in, off,
                       n_dst, dst_begin, out);
    return;
  }
  hipLaunchKernelGGL(k_dst_sort_wide<4>, dim3((n_dst + 3) / 4), dim3(256), 0, st, in, off, cnt, n_dst, out);
}

template <uint32_t kC>
static void launch_sort_bkt(const tgsim_delivery* bkt, tgsim_delivery* sc, const uint64_t* doff, uint32_t n_dst,
                            tgsim_delivery* out, hipStream_t st, const uint64_t* total, uint64_t cap,
                            uint64_t* err_host) {
  constexpr uint32_t per_wg = 4 * (kWave / (kC < 16 ? kC : 16));
  const uint32_t groups = (n_dst + per_wg - 1) / per_wg;
  // 1,024 resident workgroups (four waves per SIMD): at the 1M-peer flood the sort then leaves the
  // simulate kernels room beside it (A/B, 1M-peer gossip G pkt/s: 256 3.3, 512 5.16, 768 5.61,
  // 1,024 5.60-5.64, 1,536 5.46, 2,048 5.46, 4,096 5.48, 8,192 5.32, one per group 5.30)
  const uint32_t grid = std::min<uint32_t>(groups, 1024u);
  hipLaunchKernelGGL(k_dst_sort_bkt<kC>, dim3(grid), dim3(256), 0, st, bkt, sc, doff, n_dst, out, total, cap, err_host);
}
void launch_dst_sort_bkt(const tgsim_delivery* bkt, uint32_t bkt_log, tgsim_delivery* sc, const uint64_t* doff,
                         uint32_t n_dst, tgsim_delivery* out, hipStream_t st, const uint64_t* total, uint64_t cap,
                         uint64_t* err_host) {
  if (!n_dst) return;
  switch (bkt_log) {
    case 3: launch_sort_bkt<8>(bkt, sc, doff, n_dst, out, st, total, cap, err_host); break;
    case 4: launch_sort_bkt<16>(bkt, sc, doff, n_dst, out, st, total, cap, err_host); break;
    case 5: launch_sort_bkt<32>(bkt, sc, doff, n_dst, out, st, total, cap, err_host); break;
    default: launch_sort_bkt<64>(bkt, sc, doff, n_dst, out, st, total, cap, err_host); break;
  }
}

void launch_dst_sort_w1(tgsim_delivery* in, const uint64_t* off, uint64_t* cnt, uint32_t n_dst,
                        tgsim_delivery* out, hipStream_t st) {
  if (n_dst) hipLaunchKernelGGL(k_dst_sort_wide<1>, dim3(n_dst), dim3(64), 0, st, in, off, cnt, n_dst, out);
}

void launch_scan_w(uint64_t* in, uint64_t* out, uint64_t n, uint64_t* block_sums, uint64_t* total,
                   hipStream_t st, uint64_t* pos, bool clear) {
  const uint32_t nb = (uint32_t)((n + 1023) / 1024);
  if (!nb) {
    launch_scan(in, out, n, block_sums, total, st, pos);
    return;
  }
  hipLaunchKernelGGL(k_scan_w1, dim3(nb), dim3(64), 0, st, in, n, block_sums);
  hipLaunchKernelGGL(k_scan_w2, dim3(nb), dim3(64), 0, st, in, n, (const uint64_t*)block_sums, out, pos, total,
                     clear ? 1u : 0u);
}

void launch_local_scatter_group(const GroupDeliver& g, uint32_t n_win, hipStream_t st) {
  if (g.n_src && n_win) hipLaunchKernelGGL(k_local_scatter_group, dim3(n_win * g.n_src), dim3(64), 0, st, g);
}

// Cross-lane guard violations so far (TGSIM_CHECK builds; -ENOSYS in the product build).
int64_t exec_faults() {
#ifdef TGSIM_CHECK
  unsigned int n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(tg_exec_faults), sizeof n) != hipSuccess) return -EIO;
  return n;
#else
  return -ENOSYS;
#endif
}


}  // namespace tgsim
