// tgsim_engine.cpp — host runtime of libtgsim.so: the C ABI of include/tgsim.h.
//
// Replaces the reference sidecar's netlink programming (pkg/sidecar/link.go, route.go,
// docker_network.go) with compiled SoA state on the GPU, and the kernel data path with the HIP
// kernels of tgsim_kernels.hip.  Configuration is compiled on the host exactly as netlink v1.1.0
// + the kernel would install it, staged, and scattered into HBM by the
// config-apply kernel at the next step.
#include <errno.h>
#include <stdlib.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <map>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "tgsim_launch.h"

using namespace tgsim;

// Host spin-waits on words the device publishes to pinned memory: a pause per poll, and no yield of
// the core before about this many polls (a few ms).
inline void spin_pause() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#endif
}
constexpr uint32_t kSpinBeforeYield = 1u << 16;

// Events that order work between this engine's own streams (and its timing events) skip the
// system-scope fence a recorded event otherwise makes (a writeback of the device caches that the
// next command on the stream waits for; A/B, profiles/r06/ab_nofence/: C5 +1.6 %, sub-capacity +3 %,
// C3 +0.6 %).  Events the host relies on to see device writes in host memory keep it.
constexpr unsigned kEvSync = hipEventDisableTiming | hipEventDisableSystemFence;
constexpr unsigned kEvTiming = hipEventDefault | hipEventDisableSystemFence;

namespace {

// ------------------------------------------------------------------------------------------------
// netlink / kernel unit conversions (link.go:143-183 and netlink v1.1.0 NewNetem/NewHtbClass).

uint32_t go_float_to_u32(double x) {  // Go on amd64: CVTTSD2SQ then low 32 bits
  if (!(x > -9.2233720368547758e18 && x < 9.2233720368547758e18)) return 0;
  return static_cast<uint32_t>(static_cast<int64_t>(x));
}

uint32_t pct_to_u32(float pct) {  // netlink Percentage2u32 (float32 arithmetic)
  if (pct == 100.0f) return 0xFFFFFFFFu;
  volatile float frac = pct / 100.0f;
  volatile float scaled = 4294967296.0f * frac;
  return go_float_to_u32(static_cast<double>(scaled));
}

uint32_t duration_us(int64_t ns) {  // link.go:143-151
  int64_t us = ns / 1000;
  if (us > static_cast<int64_t>(UINT32_MAX)) us = UINT32_MAX;
  return static_cast<uint32_t>(us);
}

uint32_t us_to_ticks(uint32_t us) { return go_float_to_u32(static_cast<double>(us) * 15.625); }

// psched_ratecfg_precompute: the smallest shift whose mult = (NSEC_PER_SEC << shift) / rate has bit 31
// set (or whose factor reaches bit 63).  floor(f / rate) >= 2^31 exactly when f >= 2^31 * rate (rate is
// a u32: no overflow), so the shift is found with shifts alone and one division (the kernel's loop
// divides at every step: ~30 divisions a configure call).
void psched_precompute(uint64_t rate, uint32_t* mult, uint32_t* shift) {
  *mult = 1;
  *shift = 0;
  if (!rate) return;
  const uint64_t need = rate << 31;
  uint64_t factor = 1000000000ull;
  while (factor < need && !(factor & 0x8000000000000000ull)) {
    factor <<= 1;
    ++*shift;
  }
  *mult = static_cast<uint32_t>(factor / rate);
}

struct Compiled {
  SrcParams p;     // rule_off/rule_n/allow_ext left for the caller
  bool corrupt_attr, reorder_attr, corr_attr;
  uint32_t rho_dup_new, rho_cor_new, rho_reo_new, thr_cor_new;
};

Compiled compile_shape(const tgsim_shape& s) {
  Compiled c;
  memset(&c, 0, sizeof c);
  const uint32_t lat_us = duration_us(s.latency_ns), jit_us = duration_us(s.jitter_ns);
  const uint32_t lat_ticks = us_to_ticks(lat_us);
  const uint32_t jit_ticks = lat_ticks ? us_to_ticks(jit_us) : jit_us;
  c.p.lat_ns = static_cast<uint64_t>(lat_ticks) << 6;
  int32_t sigma = static_cast<int32_t>(static_cast<uint32_t>(static_cast<uint64_t>(jit_ticks) << 6));
  if (static_cast<uint32_t>(sigma) == 0x80000000u) sigma = 0x7FFFFFFF;
  c.p.sigma = sigma;
  c.p.thr_loss = pct_to_u32(s.loss);
  c.p.thr_dup = pct_to_u32(s.duplicate);
  c.p.thr_reo = pct_to_u32(s.reorder);
  c.thr_cor_new = pct_to_u32(s.corrupt);
  c.rho_dup_new = c.p.thr_dup ? pct_to_u32(s.duplicate_corr) : 0;
  c.rho_cor_new = pct_to_u32(s.corrupt_corr);
  c.rho_reo_new = pct_to_u32(s.reorder_corr);
  c.corrupt_attr = c.thr_cor_new != 0;
  c.reorder_attr = c.p.thr_reo != 0;
  c.corr_attr = c.rho_dup_new != 0;
  const uint64_t rate_bytes = (s.bandwidth_bps ? s.bandwidth_bps : UINT64_MAX) / 8;
  const uint32_t buffer = go_float_to_u32(static_cast<double>(rate_bytes) / 1e9 + 1600.0);
  const uint32_t buffer_us = go_float_to_u32(1e6 * (static_cast<double>(buffer) / static_cast<double>(rate_bytes)));
  c.p.burst_ns = static_cast<uint64_t>(us_to_ticks(buffer_us)) << 6;
  uint32_t mult, shift;
  psched_precompute(static_cast<uint32_t>(rate_bytes), &mult, &shift);  // TcRateSpec.Rate is u32
  c.p.mult = mult;
  c.p.shift_ext = shift;
  return c;
}

// Philox on the host (initial correlation state of init_crandom()).
void philox_host(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t r[4]) {
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c0;
    const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * c2;
    const uint32_t n0 = static_cast<uint32_t>(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = static_cast<uint32_t>(p0 >> 32) ^ c3 ^ k1;
    c0 = n0;
    c1 = static_cast<uint32_t>(p1);
    c2 = n2;
    c3 = static_cast<uint32_t>(p0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  r[0] = c0; r[1] = c1; r[2] = c2; r[3] = c3;
}

// Longest-prefix-match rule set -> sorted disjoint intervals carrying the winning action.
std::vector<Interval> compile_rules(const std::map<uint64_t, uint8_t>& rules) {
  struct R { uint64_t lo, hi; uint32_t len, act; };
  std::vector<R> rs;
  for (const auto& kv : rules) {
    const uint32_t net = static_cast<uint32_t>(kv.first >> 8), len = kv.first & 0xFF;
    const uint64_t size = len == 0 ? (1ull << 32) : (1ull << (32 - len));
    rs.push_back({net, static_cast<uint64_t>(net) + size - 1, len, kv.second});
  }
  std::sort(rs.begin(), rs.end(), [](const R& a, const R& b) { return a.lo != b.lo ? a.lo < b.lo : a.len < b.len; });
  std::vector<Interval> out;
  auto emit = [&](uint64_t lo, uint64_t hi, uint32_t act) {
    if (lo > hi || act == TGSIM_ACCEPT) return;
    if (!out.empty() && out.back().act == act && static_cast<uint64_t>(out.back().hi) + 1 == lo)
      out.back().hi = static_cast<uint32_t>(hi);
    else
      out.push_back({static_cast<uint32_t>(lo), static_cast<uint32_t>(hi), act});
  };
  struct Frame { uint64_t hi; uint32_t act; };
  std::vector<Frame> stk;
  uint64_t cur = 0;
  for (const R& r : rs) {
    while (!stk.empty() && stk.back().hi < r.lo) {
      emit(cur, stk.back().hi, stk.back().act);
      cur = stk.back().hi + 1;
      stk.pop_back();
    }
    if (r.lo > cur) emit(cur, r.lo - 1, stk.empty() ? TGSIM_ACCEPT : stk.back().act);
    cur = r.lo;
    stk.push_back({r.hi, r.act});
  }
  while (!stk.empty()) {
    emit(cur, stk.back().hi, stk.back().act);
    cur = stk.back().hi + 1;
    stk.pop_back();
  }
  return out;
}

// ------------------------------------------------------------------------------------------------
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t c = n < 64 ? 64 : n + n / 2;  // growing buffers (gossip windows) reallocate rarely
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), c * sizeof(T));
    if (e == hipSuccess) cap = c;
    return e;
  }
  hipError_t ensure_exact(size_t n) {  // no growth headroom (buffers sized once)
    if (n <= cap) return hipSuccess;
    release();
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), n * sizeof(T));
    if (e == hipSuccess) cap = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct HostSrc {
  SrcParams p;          // installed netem/HTB parameters (rule_off/rule_n filled at flush)
  uint32_t shape_epoch = 0;
  bool allow_ext = false;
  std::map<uint64_t, uint8_t> rules;  // (net << 8 | len) -> Reject/Drop
  uint32_t patch_mask = 0;            // pending state patch (CfgPatch.mask)
  uint32_t last[3] = {0, 0, 0};
  uint32_t patch_gen = 0;             // == Eng::patch_gen: a patch is pending, at patch_idx
  uint32_t patch_idx = 0;
};

struct StagedPkt {
  tgsim_pkt p;
  uint64_t idx;
};

}  // namespace

struct tgsim_engine_s {
  tgsim_opts o{};
  std::string err;
  int dev = 0;
  hipStream_t st = nullptr;      // simulate stream: inputs, k_sim, dispatch order
  hipStream_t dst_st = nullptr;  // delivery stream of inbound records (tgsim_deliver*), overlaps the next k_sim
  hipStream_t rt_st = nullptr;   // routing stream: a sharded step's records grouped by destination shard
                                 // beside the next k_sim (which writes the other emit pair)
  hipEvent_t ev_rt = nullptr;    // recorded after the last routing on rt_st (it reads d_off)
  hipEvent_t ev_dst = nullptr;   // recorded after the last delivery on dst_st
  hipEvent_t ev_recv = nullptr;  // recorded after the last delivery's scatter (and gossip receipts)
  hipEvent_t ev_sim = nullptr;   // sim-stream point a delivery waits for
  hipEvent_t ev_sim_t = nullptr; // the last window's timing event right behind its k_sim, or null:
                                 // a delivery or routing waits for it instead of a marker of its own
  // k_sim duration per launch: event pairs harvested lazily (the step does not synchronize), with
  // the number of windows the launch simulated (a fused launch counts each of its windows)
  struct PendingTiming {
    hipEvent_t first, second;
    uint32_t windows;
  };
  std::vector<PendingTiming> ev_pending;
  std::vector<PendingTiming> dv_pending;  // delivery spans on dst_st (first kernel to the sort), per window
  double dv_ms = 0;
  uint64_t dv_windows = 0;
  uint32_t dv_every = 1;   // TGSIM_DV_TIMING: time every k-th delivery (0: none)
  uint32_t sim_every = 1;  // TGSIM_SIM_TIMING: time every k-th per-window simulate launch (0: none)
  uint64_t sim_count = 0;
  uint64_t dv_count = 0;   // deliveries so far (the sampling counter)
  std::vector<hipEvent_t> ev_pool;
  uint32_t* h_gerr = nullptr;   // pinned copy of the gossip driver's late-receipt flag
  uint64_t* h_pub = nullptr;    // pinned words a scan publishes: [0] total, [1] flag, [2] sequence;
                                // [4..6] the same for a gossip window generated ahead of its size
  hipEvent_t ev_gpub = nullptr;
  uint64_t* dm_pub = nullptr;
  uint64_t pub_seq = 0;
  hipEvent_t ev_pub = nullptr;
  uint64_t* h_err = nullptr;    // pinned host word k_sim stores the sticky error bits into
  uint64_t* d_err_host = nullptr;  // its device address
  uint32_t* h_xerr = nullptr;   // pinned sticky flag: a slotted exchange chunk overflowed (k_route_edges)
  uint32_t* h_work = nullptr;   // pinned: sources the last sparse step deferred to k_sim_list, to k_sim_multi
  uint32_t* dm_work = nullptr;  // its device address (k_work_done stores there)
  uint32_t* d_xerr = nullptr;   // its device address
  // launched, unfinished routed steps (tgsim_step_sim_launch), oldest at route_head: pinned
  // per-rank record edges behind an event, per slot
  static constexpr uint32_t kRouteSlots = 2;
  uint64_t* h_edges = nullptr;  // kRouteSlots x 16 words
  DevBuf<uint64_t> d_rsend;     // kRouteSlots x 16: the per-rank counts of each launched routing, on the
                                // device (words 8..15 of slot 0: [8] the largest per-rank count so far)
  hipEvent_t ev_route[kRouteSlots] = {};
  uint32_t route_ranks[kRouteSlots] = {};
  size_t route_cap[kRouteSlots] = {};
  uint64_t route_seq[kRouteSlots] = {};
  uint64_t route_next_seq = 0;
  uint32_t route_head = 0, route_n = 0;
  uint32_t S = 0, N = 0;
  uint64_t now_tick = 0;
  uint32_t key0 = 0, key1 = 0;

  std::vector<uint8_t> enabled;
  uint32_t n_disabled = 0;  // peers with Enable=false (0 lets k_sim skip the enabled[dst] gather)
  std::vector<uint32_t> ip;
  std::vector<uint8_t> ip6_set;                 // an IPv6 address was assigned (cfg.IPv6 != nil)
  std::vector<std::array<uint8_t, 16>> ip6;
  std::vector<uint8_t> k8s_init;                // K8sNetwork.initialized (k8s_network.go:119-125)
  std::vector<uint8_t> gone;                    // link removed since the last step (purge pending)
  std::vector<uint32_t> link_gen;               // per peer: data links removed so far (tgsim_link_generation)
  bool any_gone = false;
  DevBuf<uint8_t> d_gone;
  std::vector<HostSrc> src;
  bool peers_dirty = true, rules_dirty = true, any_patch = false, params_dirty = true;
  // K7 sync counters: device table, pinned host mirror, pinned result/marker words, own stream
  hipStream_t sy_st = nullptr;
  hipEvent_t ev_sig = nullptr;  // after the last issued signal
  DevBuf<unsigned long long> d_sync;
  uint64_t* h_mirror = nullptr;
  uint64_t* dm_mirror = nullptr;
  uint64_t* h_sig = nullptr;    // [0] result of the last signal, [1] marker
  uint64_t* dm_sig = nullptr;
  uint64_t sig_seq = 0;

  DevBuf<SrcParams> d_params;
  DevBuf<SrcState> d_state;
  DevBuf<uint8_t> d_enabled;
  DevBuf<uint32_t> d_ip;
  DevBuf<Interval> d_rules;
  DevBuf<uint4> d_heap;
  DevBuf<uint64_t> d_ring;
  DevBuf<uint4> d_wheel;       // timing wheel: [s][kWheelB][kWheelCB] parked far items
  DevBuf<WheelMeta> d_wmeta;   // [s] bucket counts, base id, width (read only while items are parked)
  bool wheel_failed = false;   // no memory for the wheel: dense windows run without parking
  DevBuf<CfgPatch> d_patch_t[2];   // the patch sets on the device, one per turn
  // pinned staging of the configuration patches, two sets in turn: a set is refilled once the copy
  // that last read it has run (its event), so a reshape never waits for the simulation in flight
  CfgPatch* h_patch[2] = {nullptr, nullptr};
  hipEvent_t ev_patch[2] = {nullptr, nullptr};   // after the apply that last read the turn's sets
  hipEvent_t ev_pcopy = nullptr;                 // after the last patch copy (on the sync stream)
  uint32_t patch_turn = 0;
  uint32_t patch_gen = 1;   // the generation of the patches being staged (bumped at each flush)
  size_t patch_n = 0;       // patches staged in patch_stage
  std::vector<CfgPatch> patch_stage;  // (cacheable host memory; copied to the pinned set at the flush)
  DevBuf<uint32_t> d_gen_seq;

  // step input
  std::vector<StagedPkt> staged;
  std::vector<uint64_t> perm;  // internal index -> submit index (empty: identity)
  struct GenWindow {
    DevBuf<uint64_t> off;
    DevBuf<InRec> in;
    uint64_t n = 0;
    uint32_t ticks = 0;
    // a gossip window whose forwards were written before the host knew their total (published to
    // h_pub[4..6] with sequence pub_seq): resolved by the step that consumes it
    bool pending = false;
    uint64_t pub_seq = 0;
    GossipArgs g{};
    // the simulate call (run_sim / step_n) that sent the window back to the free list; 0: never used
    uint64_t retired_call = 0;
  };
  std::vector<GenWindow> gen_q;   // device-generated traffic, one window per future step
  uint64_t sim_calls = 0;         // run_sim and fused-group calls that enqueued their simulate kernel
                                  // (behind its emit set's last reader) so far (GenWindow::retired_call)
  std::vector<GenWindow> gen_free;
  uint64_t gen_q_ticks = 0;
  uint64_t n_in = 0;
  DevBuf<uint64_t> d_off, d_cnt, d_blk, d_tot;
  DevBuf<InRec> d_in;
  DevBuf<uint8_t> d_verdict;
  uint64_t n_verdict = 0;
  std::vector<uint64_t> last_perm;

  // step output
  // emit regions and per-destination histogram written by k_sim; a single-shard step reads them
  // on the delivery stream while the next k_sim writes the other pair (swapped by deliver_local;
  // ev_local: the delivery that last read the pair)
  // Emit sets: window k's k_sim writes set k % 3 (d_emit, ...) while the deliveries of the windows
  // before it read the others (*_alt: window k - 1's, *_alt2: k - 2's; rotate_emit after every window);
  // k_sim waits only for the delivery of window k - 3.  (A third set was first tried in round 3, when
  // a classic set was ~38 GB at 1M peers and it thrashed; compact sets and buckets
  // are a few GB.)
  DevBuf<tgsim_delivery> d_emit, d_emit_alt, d_emit_alt2;
  // TGSIM_EMIT_SETS: 3 (default) lets the delivery of window k lag until window k + 3 starts (alt2: the
  // set of window k - 2); the sets are allocated as they are first used
  uint32_t emit_sets = 3;
  // where each emit set's records are (classic regions, or compact regions and a pool: DESIGN §4),
  // and the per-source pool indices of each set
  EmitRead el{}, el_alt{}, el_alt2{};
  DevBuf<uint32_t> d_pidx, d_pidx_alt, d_pidx_alt2;
  int emit_compact = 1;           // TGSIM_EMIT_COMPACT: 0 every window in the classic layout, 1 auto,
                                  // 2 every sparse window compact (tests)
  bool dst_slot = true;           // TGSIM_DST_SLOT: sparse windows place records by destination slot
  bool dst_bkt = true;            // TGSIM_DST_BKT: ... and write them into destination buckets
  uint32_t emit_r = 64;           // TGSIM_EMIT_R: a compact region's reserve beyond 2 records per offered packet
  uint32_t emit_pool = 64;        // TGSIM_EMIT_POOL: the compact pool's records per source
  // the choice tgsim_sim_capacity made for the next window (run_sim takes it, so the exchange's
  // buffers and the window agree even if the deferral count read in between changed)
  int next_sparse = -1;
  uint64_t next_sparse_n = 0;  // the window size it was made for
  uint32_t wide_windows = 0;              // windows after a mid-run reshape whose bounded local delivery
                                          // reserves the full netem limit per source (deliver_local_from)
  uint64_t deliver_slack = 128;           // TGSIM_DELIVER_SLACK: queued items per source a bounded local
                                          // delivery allows for (besides 2 per offered packet)
  bool slack_forced = false;              // TGSIM_DELIVER_SLACK set: the bounded form at any size
  DevBuf<uint32_t> d_emit_n, d_emit_n_alt, d_emit_n_alt2;
  DevBuf<uint64_t> d_lcnt, d_lcnt_alt, d_lcnt_alt2;  // stays zero between steps (the delivery's scan clears it)
  DevBuf<tgsim_delivery> d_dbkt, d_dbkt_alt, d_dbkt_alt2;  // destination buckets of a sparse window (SimArgs::dst_bkt)
  hipEvent_t ev_local = nullptr, ev_local_alt = nullptr, ev_local_alt2 = nullptr;
  DevBuf<uint64_t> d_rcnt, d_rpos, d_rblk, d_rtot;  // routing: [rank][source] counts, scan
  DevBuf<tgsim_delivery> d_bucket, d_scatter, d_sorted;
  DevBuf<uint64_t> d_dcnt, d_doff, d_dpos, d_dblk, d_dtot;  // d_dcnt stays zero between steps
  // a bucketed window's scan outputs, per emit set (its scan runs on the simulate stream while the
  // delivery two windows back, of the other set, may still read the other set's)
  DevBuf<uint64_t> d_sdoff, d_sdpos, d_sdblk, d_sdtot, d_sdoff_alt, d_sdpos_alt, d_sdblk_alt, d_sdtot_alt;
  DevBuf<uint64_t> d_sdoff_alt2, d_sdpos_alt2, d_sdblk_alt2, d_sdtot_alt2;
  uint64_t h_dtot = 0;
  DevBuf<tgsim_delivery> d_drain;
  uint64_t drain_head = 0, drain_n = 0;
  DevBuf<unsigned long long> d_stats;

  double sim_ms = 0;
  uint64_t sim_launches = 0;
  bool stamps_on = false;
  DevBuf<uint32_t> d_order;  // dispatch order of the next k_sim, computed behind this one
  DevBuf<uint32_t> d_work;   // sparse steps: k_sim_sparse's deferred sources, [0] = count, then ids
  int sparse_mode = -1;      // TGSIM_SPARSE: -1 auto, 0 never, 1 always
  bool rotated = false;      // a sparse step may have left queues in place (head slot != 0)
  bool sparse_seen = false;  // h_work holds a measured worklist size
  uint32_t dense_streak = 0; // dense steps chosen because the last sparse step deferred too much
  static constexpr uint32_t dense_div = 4;  // dense when the last sparse step deferred > S / dense_div
  bool order_valid = false;
  // fused windows (tgsim_step_n): per group parity p and window i the emit regions, their counts
  // and the per-destination histogram; ev_fgrp[p]: after the deliveries that last read set p
  struct LocalSet {
    DevBuf<tgsim_delivery> emit;
    DevBuf<uint32_t> emit_n;
  };
  LocalSet fset[2][kFuseMax];
  DevBuf<uint64_t> f_lcnt[2];  // [window][destination] histograms of a group (zero between groups)
  hipEvent_t ev_fgrp[2] = {};
  uint32_t fgrp = 0;                    // parity of the next fused group
  DevBuf<uint8_t> f_verdict[kFuseMax];  // verdicts of a group's windows but the last (discarded)
  DevBuf<uint32_t> d_done, d_ticket;    // per-source completion words (window-major), ticket counter
  uint32_t step_no = 0, ticket_no = 0;  // windows and tickets issued by fused launches so far
  uint64_t fused_windows = 0;
  uint64_t sparse_windows = 0;  // windows run by the sparse kernels (tgsim_debug_sparse_windows)
  uint32_t fused_wgs = 0;
  uint32_t routed_pct = 0;      // sharded (routed) groups: 0 = one workgroup per ticket (the grid turns
                                // over), else a persistent grid of this % of the resident workgroups
  CommSlot comm{};              // tgsim_comm_init's exchange state (tgsim_comm.cpp)
  static constexpr uint32_t prio_heavy = 512;  // heaviest sources of a fused launch at wave priority 3 (A/B: 128 +1 %, 512 +7.5 %, 2048 +7 %, 4096 +5 %)  // k_sim_fused's persistent grid (resident workgroups), at the first launch
  int fuse_max = 8;  // TGSIM_FUSE: windows per fused launch, up to kFuseMax (1: never fuse; A/B at 30 windows: 4 34.8, 8 36.3, 16 36.3 G pkt/s)
  DevBuf<uint64_t> d_stamps;
  uint64_t n_stamp_wg = 0;

  // K8 metrics (TGSIM_OPT_METRICS): per-source and per-destination tables, two histograms
  bool metrics_on = false;
  DevBuf<unsigned long long> d_msrc, d_mdst, d_mhist;

  // gossip workload (C4)
  bool gossip_on = false;
  bool gossip_late = false;  // sticky until tgsim_gossip_init: a receipt preceded a generated window
  tgsim_gossip gossip{};
  DevBuf<uint32_t> d_gfirst, d_gerr, d_gnbr;
  DevBuf<uint64_t> d_gfwd, d_gpend;

  int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
  int hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return fail(-EIO, "%s: %s", what, hipGetErrorString(e));
  }
};

using Eng = tgsim_engine_s;

#define HIPCHK(expr)                              \
  do {                                            \
    int _rc = E->hip((expr), #expr);              \
    if (_rc) return _rc;                          \
  } while (0)

namespace {

// Source s is about to change: a configuration patch is pending for it from now on (k_apply_cfg at
// the next step), with its own slot in the staging array (written by write_patch when the configure
// call ends, so the flush only copies the array).
HostSrc& begin_patch(Eng* E, uint32_t s) {
  HostSrc& h = E->src[s];
  if (h.patch_gen != E->patch_gen) {
    h.patch_gen = E->patch_gen;
    h.patch_mask = 0;
    h.patch_idx = static_cast<uint32_t>(E->patch_n++);
  }
  E->any_patch = true;
  return h;
}

// The staged patch of source s (when one is pending) from its host state.
void write_patch(Eng* E, uint32_t s) {
  const HostSrc& h = E->src[s];
  if (h.patch_gen != E->patch_gen || E->patch_stage.size() <= h.patch_idx) return;
  CfgPatch& c = E->patch_stage[h.patch_idx];
  memset(&c, 0, sizeof c);
  c.s = s;
  c.mask = h.patch_mask;
  c.last_dup = h.last[0];
  c.last_cor = h.last[1];
  c.last_reo = h.last[2];
  c.p = h.p;
  c.p.shift_ext = (c.p.shift_ext & 0xFFu) | (h.allow_ext ? 0x100u : 0u);
}

void reset_source(Eng* E, uint32_t s) {
  HostSrc& h = begin_patch(E, s);
  tgsim_shape zero;
  memset(&zero, 0, sizeof zero);
  Compiled c = compile_shape(zero);  // HTB class created with Rate MaxUint64 (link.go:98-105)
  const uint32_t keep_off = h.p.rule_off, keep_n = h.p.rule_n;
  h.p = c.p;
  h.p.rule_off = keep_off;
  h.p.rule_n = keep_n;
  h.p.thr_cor = 0;
  h.p.rho_dup = h.p.rho_cor = h.p.rho_reo = 0;
  h.patch_mask |= 1u | 2u | 4u | 8u | 16u;
  h.last[0] = h.last[1] = h.last[2] = 0;
}

bool owns(const Eng* E, uint32_t peer) { return peer >= E->o.shard_begin && peer < E->o.shard_end; }

// The instance's data link goes away (NetworkDisconnect, docker_network.go:65-75 and :84-87; CNI
// DelNetworkList, k8s_network.go:134 and :151): its qdiscs die with whatever they held (flushed at
// the next step), and packets still queued towards it at any sender will find no port (k_purge at
// the next step marks them dead).  Every shard applies this to its replicated peer tables.
void link_down(Eng* E, uint32_t peer) {
  if (E->enabled[peer]) {
    E->enabled[peer] = 0;
    E->n_disabled++;
    E->peers_dirty = true;
  }
  E->gone[peer] = 1;
  E->any_gone = true;
  E->link_gen[peer]++;
  if (owns(E, peer)) begin_patch(E, peer - E->o.shard_begin).patch_mask |= 16u;
}

// A new data link (NetworkConnect + NewNetlinkLink, docker_network.go:90-137; CNI AddNetworkList,
// k8s_network.go:158-244): fresh HTB class and netem qdisc, the requested addresses.
void link_up(Eng* E, uint32_t peer, const tgsim_config* cfg) {
  if (!E->enabled[peer]) {
    E->enabled[peer] = 1;
    E->n_disabled--;
    E->peers_dirty = true;
  }
  if (cfg->has_ipv4 && cfg->ipv4 != E->ip[peer]) {
    E->ip[peer] = cfg->ipv4;
    E->peers_dirty = true;
  }
  E->ip6_set[peer] = cfg->has_ipv6 ? 1 : 0;  // IPAMConfig.IPv6Address only when cfg.IPv6 != nil
  if (cfg->has_ipv6) memcpy(E->ip6[peer].data(), cfg->ipv6, 16);
  if (owns(E, peer)) reset_source(E, peer - E->o.shard_begin);
}

// link.Shape (link.go:155-183): HTB ClassChange + netem QdiscChange (netem_change semantics).
void apply_shape(Eng* E, uint32_t peer, const tgsim_shape& shape, const Compiled* pre = nullptr) {
  HostSrc& h = begin_patch(E, peer - E->o.shard_begin);
  const Compiled c = pre ? *pre : compile_shape(shape);
  h.shape_epoch++;
  uint32_t rnd[4];
  philox_host(peer, 0xFFFFFFFEu, h.shape_epoch, 3, E->key0, E->key1, rnd);  // init_crandom()
  h.p.lat_ns = c.p.lat_ns;
  h.p.sigma = c.p.sigma;
  h.p.thr_loss = c.p.thr_loss;
  h.p.thr_dup = c.p.thr_dup;
  h.p.thr_reo = c.p.thr_reo;
  h.p.burst_ns = c.p.burst_ns;
  h.p.mult = c.p.mult;
  h.p.shift_ext = c.p.shift_ext;
  if (c.corr_attr) {
    h.p.rho_dup = c.rho_dup_new;
    h.last[0] = rnd[0];
    h.patch_mask |= 1u;
  }
  if (c.corrupt_attr) {  // absent attribute: q->corrupt and its correlation persist
    h.p.thr_cor = c.thr_cor_new;
    h.p.rho_cor = c.rho_cor_new;
    h.last[1] = rnd[1];
    h.patch_mask |= 2u;
  }
  if (c.reorder_attr) {
    h.p.rho_reo = c.rho_reo_new;
    h.last[2] = rnd[2];
    h.patch_mask |= 4u;
  }
}

// link.AddRules (link.go:187-217): cumulative; Accept deletes; host bits -> EINVAL.
int add_rules(Eng* E, uint32_t peer, const tgsim_config* cfg) {
  HostSrc& h = E->src[peer - E->o.shard_begin];
  for (uint32_t i = 0; i < cfg->n_rules; ++i) {
    const tgsim_rule& r = cfg->rules[i];
    const bool bad_len = r.len > 32;
    const uint32_t mask = (!bad_len && r.len) ? (0xFFFFFFFFu << (32 - r.len)) : 0u;
    const bool bad = bad_len || (r.prefix & ~mask) != 0;
    const uint64_t key = (static_cast<uint64_t>(r.prefix) << 8) | r.len;
    if (r.action == TGSIM_ACCEPT) {
      if (!bad && h.rules.erase(key)) E->rules_dirty = true;
      continue;
    }
    if (r.action != TGSIM_REJECT && r.action != TGSIM_DROP)
      return E->fail(-EINVAL, "invalid filter action %u", r.action);
    if (bad) return E->fail(-EINVAL, "invalid argument");
    auto it = h.rules.find(key);
    if (it == h.rules.end() || it->second != r.action) {
      h.rules[key] = r.action;
      E->rules_dirty = true;
    }
  }
  return 0;
}

// handleRoutingPolicy (route.go:102-117): AllowAll enables the external routes, anything else
// (DenyAll, empty, unknown: the default case :110-112) removes them.
void apply_policy(Eng* E, uint32_t peer, uint8_t policy) {
  if (!owns(E, peer)) return;
  HostSrc& h = E->src[peer - E->o.shard_begin];
  const bool allow = policy == TGSIM_ALLOW_ALL;
  if (allow != h.allow_ext) {
    begin_patch(E, peer - E->o.shard_begin);
    h.allow_ext = allow;
  }
}

bool ip_changed(const Eng* E, uint32_t peer, const tgsim_config* cfg) {
  return cfg->has_ipv4 && cfg->ipv4 != E->ip[peer];
}
bool ip6_changed(const Eng* E, uint32_t peer, const tgsim_config* cfg) {
  // a link without an IPv6 address differs from any requested one (the reference dereferences
  // link.IPv6.IP there, docker_network.go:77)
  return cfg->has_ipv6 && (!E->ip6_set[peer] || memcmp(E->ip6[peer].data(), cfg->ipv6, 16) != 0);
}

// DockerNetwork.ConfigureNetwork (docker_network.go:51-148).
int configure_docker(Eng* E, uint32_t peer, const tgsim_config* cfg, const Compiled* pre = nullptr) {
  const char* net = cfg->network ? cfg->network : "";
  if (strcmp(net, "default") != 0) return E->fail(-EINVAL, "unsupported network: %s", net);
  apply_policy(E, peer, cfg->routing_policy);  // :57, before anything else
  bool online = E->enabled[peer] != 0;
  if (!cfg->enable) {  // :65-75
    if (online) link_down(E, peer);
    return 0;
  }
  if (online && (ip6_changed(E, peer, cfg) || ip_changed(E, peer, cfg))) {  // :77-88
    link_down(E, peer);
    online = false;
  }
  if (!online) link_up(E, peer, cfg);  // :90-137
  if (!owns(E, peer)) return 0;
  apply_shape(E, peer, cfg->shape, pre);  // :139
  return add_rules(E, peer, cfg);    // :143
}

// K8sNetwork.ConfigureNetwork (k8s_network.go:114-256).
int configure_k8s(Eng* E, uint32_t peer, const tgsim_config* cfg, const Compiled* pre = nullptr) {
  const char* net = cfg->network ? cfg->network : "";
  if (strcmp(net, "default") != 0) return E->fail(-EINVAL, "configured network is not `default`");  // :115-117
  if (!E->k8s_init[peer]) {  // :119-125: InitializeNetwork deletes the address the pod came with
    E->k8s_init[peer] = 1;
    if (E->enabled[peer]) link_down(E, peer);
  }
  bool online = E->enabled[peer] != 0;
  if (!cfg->enable) {  // :130-140 (the routing policy is left as it is)
    if (online) link_down(E, peer);
    return 0;
  }
  // :142-155; k8s links carry no IPv6 address (:238), so any requested one is a change
  if (online && (cfg->has_ipv6 || ip_changed(E, peer, cfg))) {
    link_down(E, peer);
    online = false;
  }
  if (!online) {
    if (cfg->has_ipv6) return E->fail(-EAFNOSUPPORT, "ipv6 not supported");  // :161-163, already disconnected
    link_up(E, peer, cfg);
  }
  if (owns(E, peer)) {
    apply_shape(E, peer, cfg->shape, pre);      // :246-248
    const int rc = add_rules(E, peer, cfg);     // :249-251
    if (rc) return rc;
  }
  apply_policy(E, peer, cfg->routing_policy);  // :252-254, last
  return 0;
}

constexpr uint32_t kWideAfterReshape = 16;
constexpr uint64_t kExactBoundBytes = 1ull << 31;  // local delivery buffers sized for the worst case up to 2 GiB

hipError_t sync_stream_ready(Eng* E) {
  if (E->sy_st) return hipSuccess;
  int lo = 0, hi = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (e != hipSuccess) return e;
  e = hipStreamCreateWithPriority(&E->sy_st, hipStreamNonBlocking, hi);
  if (e != hipSuccess) return e;
  return hipEventRecord(E->ev_sig, E->sy_st);
}

int flush_config(Eng* E) {
  if (E->any_gone) {  // packets queued towards a removed link: marked dead in every sender's queue
    HIPCHK(E->d_gone.ensure(E->N));
    HIPCHK(hipMemcpyAsync(E->d_gone.p, E->gone.data(), E->N, hipMemcpyHostToDevice, E->st));
    launch_purge(E->d_heap.p, E->d_wheel.p, E->d_wmeta.p, E->d_state.p, E->S, E->d_gone.p, E->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(E->st));
    std::fill(E->gone.begin(), E->gone.end(), 0);
    E->any_gone = false;
  }
  if (E->peers_dirty) {
    HIPCHK(hipMemcpyAsync(E->d_enabled.p, E->enabled.data(), E->N, hipMemcpyHostToDevice, E->st));
    HIPCHK(hipMemcpyAsync(E->d_ip.p, E->ip.data(), sizeof(uint32_t) * E->N, hipMemcpyHostToDevice, E->st));
    E->peers_dirty = false;
  }
  const bool rules_changed = E->rules_dirty;
  if (E->rules_dirty) {
    std::vector<Interval> all;
    for (uint32_t s = 0; s < E->S; ++s) {
      HostSrc& h = E->src[s];
      std::vector<Interval> iv = compile_rules(h.rules);
      h.p.rule_off = static_cast<uint32_t>(all.size());
      h.p.rule_n = static_cast<uint32_t>(iv.size());
      all.insert(all.end(), iv.begin(), iv.end());
    }
    if (all.empty()) all.push_back({0, 0, 0});
    HIPCHK(E->d_rules.ensure(all.size()));
    HIPCHK(hipMemcpyAsync(E->d_rules.p, all.data(), sizeof(Interval) * all.size(), hipMemcpyHostToDevice, E->st));
    E->rules_dirty = false;
    E->params_dirty = true;
  }
  if (E->params_dirty) {
    std::vector<SrcParams> ps(E->S);
    for (uint32_t s = 0; s < E->S; ++s) {
      ps[s] = E->src[s].p;
      ps[s].shift_ext = (ps[s].shift_ext & 0xFFu) | (E->src[s].allow_ext ? 0x100u : 0u);
    }
    HIPCHK(hipMemcpyAsync(E->d_params.p, ps.data(), sizeof(SrcParams) * E->S, hipMemcpyHostToDevice, E->st));
    HIPCHK(hipStreamSynchronize(E->st));
    E->params_dirty = false;
    if (E->now_tick) E->wide_windows = kWideAfterReshape;
  }
  if (E->any_patch) {
    // The patches were staged in pinned memory by the configure calls (write_patch); the copy and
    // k_apply_cfg queue behind the window in flight on the simulate stream and the host goes on (a
    // stream synchronize here, and a pass over every source to build the patches, had held each
    // reshaping step until the previous window finished: the C5 epochs' host gap)
    const size_t k = std::min(E->patch_n, E->patch_stage.size());
    const uint32_t t = E->patch_turn;
    if (k) {
      if (rules_changed)  // intervals recompiled above: the staged params carry the old rule ranges
        for (size_t i = 0; i < k; ++i) {
          CfgPatch& c = E->patch_stage[i];
          c.p.rule_off = E->src[c.s].p.rule_off;
          c.p.rule_n = E->src[c.s].p.rule_n;
        }
      // into the pinned set of this turn once its last copy has run (its event: long done in a step
      // loop), one streaming copy
      if (E->ev_patch[t]) HIPCHK(hipEventSynchronize(E->ev_patch[t]));
      if (!E->h_patch[t])
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&E->h_patch[t]), sizeof(CfgPatch) * (E->S ? E->S : 1),
                             hipHostMallocDefault));
      memcpy(E->h_patch[t], E->patch_stage.data(), sizeof(CfgPatch) * k);
      // the copy runs on the sync stream, beside the window in flight on the simulate stream (in line
      // it sat between two windows: ~45 us of a 1 ms C5 epoch); the apply waits for it
      HIPCHK(E->d_patch_t[t].ensure(E->S));  // (sized once: never reallocated under a copy or apply)
      HIPCHK(sync_stream_ready(E));
      if (!E->ev_pcopy) HIPCHK(hipEventCreateWithFlags(&E->ev_pcopy, kEvSync));
      if (E->ev_patch[t]) HIPCHK(hipStreamWaitEvent(E->sy_st, E->ev_patch[t], 0));
      HIPCHK(hipMemcpyAsync(E->d_patch_t[t].p, E->h_patch[t], sizeof(CfgPatch) * k, hipMemcpyHostToDevice, E->sy_st));
      HIPCHK(hipEventRecord(E->ev_pcopy, E->sy_st));
      HIPCHK(hipStreamWaitEvent(E->st, E->ev_pcopy, 0));
      launch_apply_cfg(E->d_patch_t[t].p, static_cast<uint32_t>(k), E->d_params.p, E->d_state.p, E->d_stats.p, E->st);
      HIPCHK(hipGetLastError());
      if (!E->ev_patch[t]) HIPCHK(hipEventCreateWithFlags(&E->ev_patch[t], kEvSync));
      HIPCHK(hipEventRecord(E->ev_patch[t], E->st));
      E->patch_turn = t ^ 1u;
      if (E->now_tick) E->wide_windows = kWideAfterReshape;
    }
    E->patch_n = 0;
    E->patch_gen++;
    E->any_patch = false;
  }
  return 0;
}

// Builds the CSR input of the step from the host-staged packets.
int stage_host_input(Eng* E, uint32_t n_ticks) {
  std::vector<StagedPkt>& v = E->staged;
  for (size_t i = 0; i < v.size(); ++i)
    if (v[i].p.tick >= n_ticks)
      return E->fail(-EINVAL, "packet %zu: tick %u beyond step of %u ticks", i, v[i].p.tick, n_ticks);
  std::stable_sort(v.begin(), v.end(), [](const StagedPkt& a, const StagedPkt& b) {
    if (a.p.src != b.p.src) return a.p.src < b.p.src;
    if (a.p.tick != b.p.tick) return a.p.tick < b.p.tick;
    return a.p.seq < b.p.seq;
  });
  std::vector<uint64_t> off(E->S + 1, 0);
  std::vector<InRec> recs(v.size());
  E->perm.assign(v.size(), 0);
  for (size_t i = 0; i < v.size(); ++i) {
    off[v[i].p.src - E->o.shard_begin + 1]++;
    recs[i].dst = v[i].p.dst;
    recs[i].seq = v[i].p.seq;
    recs[i].tick = v[i].p.tick;
    recs[i].len = v[i].p.len;
    E->perm[i] = v[i].idx;
  }
  for (uint32_t s = 0; s < E->S; ++s) off[s + 1] += off[s];
  E->n_in = v.size();
  HIPCHK(E->d_off.ensure(E->S + 1));
  HIPCHK(E->d_in.ensure(E->n_in ? E->n_in : 1));
  HIPCHK(hipStreamWaitEvent(E->st, E->ev_dst, 0));  // a local delivery may still read d_off
  HIPCHK(hipStreamWaitEvent(E->st, E->ev_rt, 0));   // and so may a routing
  HIPCHK(hipMemcpyAsync(E->d_off.p, off.data(), sizeof(uint64_t) * (E->S + 1), hipMemcpyHostToDevice, E->st));
  if (E->n_in)
    HIPCHK(hipMemcpyAsync(E->d_in.p, recs.data(), sizeof(InRec) * E->n_in, hipMemcpyHostToDevice, E->st));
  HIPCHK(hipStreamSynchronize(E->st));
  E->staged.clear();
  return 0;
}

// Device exclusive scan of cnt[0..n) into off[0..n] (off[n] = total); returns total on host.
int wait_published(Eng* E, const uint64_t* word, uint64_t want, hipEvent_t ev, const char* what);

// Device exclusive scan of cnt[0..n) into off[0..n] (off[n] = total); returns total on host.  The
// total (and *flag, when given) reach the host through pinned words the device publishes behind a
// sequence number: the host spins on them instead of synchronizing the stream, whose wake-up can
// lag the device by hundreds of microseconds (the closed gossip loop pays it every window).
int scan_counts(Eng* E, DevBuf<uint64_t>& cnt, DevBuf<uint64_t>& off, DevBuf<uint64_t>& blk,
                DevBuf<uint64_t>& tot, uint64_t n, uint64_t* total, uint64_t* pos = nullptr,
                hipStream_t stream = nullptr, const uint32_t* flag = nullptr, uint32_t* flag_out = nullptr,
                bool clear = false) {
  hipStream_t sq = stream ? stream : E->st;
  HIPCHK(off.ensure(n + 1));
  HIPCHK(blk.ensure((n + 1023) / 1024 + 1));
  HIPCHK(tot.ensure(1));
  launch_scan(cnt.p, off.p, n, blk.p, tot.p, sq, pos, clear ? cnt.p : nullptr);
  HIPCHK(hipGetLastError());
  launch_publish(tot.p, flag, E->dm_pub, ++E->pub_seq, sq);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(E->ev_pub, sq));
  int rc = wait_published(E, &E->h_pub[2], E->pub_seq, E->ev_pub, "traffic generation (scan total)");
  if (rc) return rc;
  *total = __atomic_load_n(&E->h_pub[0], __ATOMIC_ACQUIRE);
  if (flag_out) *flag_out = static_cast<uint32_t>(__atomic_load_n(&E->h_pub[1], __ATOMIC_ACQUIRE));
  return 0;
}

constexpr uint32_t kOrderMaxSources = 32768;  // = kOrderMax of the order kernel

constexpr size_t kEventPool = 160;  // two pairs a window: 40 windows before the first harvest

hipError_t take_event(Eng* E, hipEvent_t* ev) {
  if (!E->ev_pool.empty()) {
    *ev = E->ev_pool.back();
    E->ev_pool.pop_back();
    return hipSuccess;
  }
  return hipEventCreateWithFlags(ev, kEvTiming);
}

// Folds finished k_sim event pairs into the running average (wait: block until all are done).
int harvest_timing(Eng* E, bool wait) {
  // without waiting, only once many are pending or the pool runs dry: every event query is host time in
  // the step's launch path, which short windows (the sub-capacity storm's 0.12 ms) cannot afford per
  // window, and so is every hipEventCreate (a drained pool in a 70-window flood created ~280 of them)
  if (!wait && E->ev_pending.size() + E->dv_pending.size() < 256 && E->ev_pool.size() >= 4) return 0;
  size_t k = 0;
  for (; k < E->ev_pending.size(); ++k) {
    auto& pr = E->ev_pending[k];
    if (wait) {
      HIPCHK(hipEventSynchronize(pr.second));
    } else if (hipEventQuery(pr.second) != hipSuccess) {
      break;
    }
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, pr.first, pr.second));
    E->sim_ms += ms;
    E->sim_launches += pr.windows;
    E->ev_pool.push_back(pr.first);
    E->ev_pool.push_back(pr.second);
  }
  E->ev_pending.erase(E->ev_pending.begin(), E->ev_pending.begin() + k);
  for (k = 0; k < E->dv_pending.size(); ++k) {
    auto& pr = E->dv_pending[k];
    if (wait) {
      HIPCHK(hipEventSynchronize(pr.second));
    } else if (hipEventQuery(pr.second) != hipSuccess) {
      break;
    }
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, pr.first, pr.second));
    E->dv_ms += ms;
    E->dv_windows += pr.windows;
    E->ev_pool.push_back(pr.first);
    E->ev_pool.push_back(pr.second);
  }
  E->dv_pending.erase(E->dv_pending.begin(), E->dv_pending.begin() + k);
  return 0;
}

// The sticky error word of k_sim (simulated time past 2^46 ns), as k_sim stores it into pinned host
// memory: exact after a stream synchronization, possibly one step late otherwise.
int check_sim_error(Eng* E) {
  const uint64_t herr = E->h_err ? __atomic_load_n(E->h_err, __ATOMIC_RELAXED) : 0;
  if (herr & kErrTimeOverflow) return E->fail(-EOVERFLOW, "simulated time exceeds 2^46 ns");
  if (herr & kErrHandoff)
    return E->fail(-EIO, "fused step: a source's previous window did not complete (hand-off timed out)");
  if (herr & kErrDeliverCap)
    return E->fail(-ENOSPC, "local delivery: a window's records exceed the delivery buffers (TGSIM_DELIVER_SLACK)");
  if (herr & kErrEmitPool)
    return E->fail(-ENOSPC, "sparse window: the sources that served more than their compact emit regions hold "
                            "overflowed the emit pool (TGSIM_EMIT_POOL, or TGSIM_EMIT_COMPACT=0)");
  if (E->h_xerr && __atomic_load_n(E->h_xerr, __ATOMIC_RELAXED))
    return E->fail(-ENOSPC, "exchange: a step's records for one rank exceed the slot capacity");
  return 0;
}

// Every reader of device results goes through here: the step itself does not synchronize.
int sync_stream(Eng* E) {
  HIPCHK(hipStreamSynchronize(E->st));
  HIPCHK(hipStreamSynchronize(E->rt_st));
  HIPCHK(hipStreamSynchronize(E->dst_st));
  return harvest_timing(E, true);
}

// The timing wheel, allocated at the first dense window: sparse windows never park
// items (k_sim_sparse defers a source with parked items to k_sim_list, which takes them all back), so
// an engine that only runs sparse windows never pays its 64 KiB per source; a gossip flood never parks
// (its dense windows would send their sources through k_sim_list afterwards).  No memory for it: the
// dense windows run without parking (every far item stays in the heap array).
void ensure_wheel(Eng* E) {
  if (E->d_wheel.p || E->wheel_failed || E->gossip_on) return;
  if (E->d_wheel.ensure_exact(static_cast<size_t>(E->S) * kWheelB * kWheelCB) != hipSuccess ||
      E->d_wmeta.ensure_exact(E->S) != hipSuccess) {
    (void)hipGetLastError();
    E->d_wheel.release();
    E->d_wmeta.release();
    E->wheel_failed = true;
  }
}

// The step-independent part of k_sim's arguments (tables, state, statistics, keys).
SimArgs base_sim_args(Eng* E) {
  SimArgs a{};
  a.params = E->d_params.p;
  a.state = E->d_state.p;
  a.enabled = E->d_enabled.p;
  a.ip = E->d_ip.p;
  a.rules = E->d_rules.p;
  a.heap = E->d_heap.p;
  a.ring = E->d_ring.p;
  a.wheel = E->d_wheel.p;
  a.wmeta = E->d_wmeta.p;
  a.stats = E->d_stats.p;
  a.key0 = E->key0;
  a.key1 = E->key1;
  a.n_src = E->S;
  a.shard_begin = E->o.shard_begin;
  a.n_peers = E->N;
  a.queue_limit = E->o.queue_limit;
  a.any_disabled = E->n_disabled ? 1u : 0u;
  a.tick_ns = E->o.tick_ns;
  a.err_host = E->d_err_host;
  a.emit_r = kHeapCap;  // the classic emit layout unless run_sim picks the compact one
  return a;
}

// The next window's emit set: the current one becomes the newest being delivered.
void rotate_emit(Eng* E) {
  // (current, newest delivered, older) <- (older, current, newest delivered): window k + 1 writes the
  // set of window k - 2 (three sets) or k - 1 (two), whose delivery it waits for (ev_local)
  auto rot = [E](auto& cur, auto& alt, auto& alt2) {
    if (E->emit_sets == 3) {
      std::swap(cur, alt2);  // (alt2, alt, cur)
      std::swap(alt, alt2);  // (alt2, cur, alt)
    } else {
      std::swap(cur, alt);
    }
  };
  rot(E->d_emit, E->d_emit_alt, E->d_emit_alt2);
  rot(E->el, E->el_alt, E->el_alt2);
  rot(E->d_pidx, E->d_pidx_alt, E->d_pidx_alt2);
  rot(E->d_emit_n, E->d_emit_n_alt, E->d_emit_n_alt2);
  rot(E->d_lcnt, E->d_lcnt_alt, E->d_lcnt_alt2);
  rot(E->d_dbkt, E->d_dbkt_alt, E->d_dbkt_alt2);
  rot(E->d_sdoff, E->d_sdoff_alt, E->d_sdoff_alt2);
  rot(E->d_sdpos, E->d_sdpos_alt, E->d_sdpos_alt2);
  rot(E->d_sdblk, E->d_sdblk_alt, E->d_sdblk_alt2);
  rot(E->d_sdtot, E->d_sdtot_alt, E->d_sdtot_alt2);
  rot(E->ev_local, E->ev_local_alt, E->ev_local_alt2);
}

// The size of a gossip window generated ahead of it (tgsim_gen_gossip): waits for the published
// scan total; a window larger than its reserved buffer is written again into a larger one.
int resolve_gen(Eng* E, Eng::GenWindow& w) {
  if (!w.pending) return 0;
  int rc = wait_published(E, &E->h_pub[6], w.pub_seq, E->ev_gpub, "gossip generation (scan total)");
  if (rc) return rc;
  const uint64_t total = __atomic_load_n(&E->h_pub[4], __ATOMIC_ACQUIRE);
  const uint64_t late = __atomic_load_n(&E->h_pub[5], __ATOMIC_ACQUIRE);
  w.pending = false;
  if (late) {  // the write kernels of this window (and of any after it) wrote nothing: the flag is set
               // before them on the stream, so no peer's fwd/pend changed for it (drop_gen)
    E->gossip_late = true;
    return E->fail(-EINVAL, "gossip: a receipt precedes the window at tick %llu (lookahead shorter than the window)",
                   static_cast<unsigned long long>(w.g.win0));
  }
  if (total > w.in.cap) {  // the capped write skipped this window: write it into a larger buffer
    HIPCHK(hipStreamSynchronize(E->st));  // (the old buffer is freed)
    HIPCHK(w.in.ensure(total));
    launch_gossip(w.g, nullptr, 0, nullptr, w.off.p, w.in.p, 2, E->st);
    HIPCHK(hipGetLastError());
  }
  w.n = total;
  return 0;
}

// A window's buffers back to the free list, stamped with the simulate call that retired them (a
// fused group's: always-wait, since its group delivery is awaited only by the group two later).
constexpr uint64_t kRetiredByGroup = ~0ull >> 2;
int retire_gen(Eng* E, Eng::GenWindow&& w, bool by_group = false) {
  // the call retiring it is numbered sim_calls + 1 once its simulate kernel is enqueued (a call that
  // fails before that never counts, so the stamp can only run ahead: more waiting, never less)
  w.retired_call = by_group ? kRetiredByGroup : E->sim_calls + 1;
  E->gen_free.push_back(std::move(w));
  return 0;
}

// A free window for the next generation (the OLDEST retired one).  Its offsets were last read by the
// delivery and routing of the window they belonged to; those are waited for by the simulation of
// the window emit_sets later (through its emit set or, two later, its fused buffer set), which the
// simulate stream runs before this generation once emit_sets more simulate calls were made.
// Otherwise (a short rotation) the generation waits for the latest delivery and routing.  With the
// gossip driver's emit_sets + 1 windows in rotation (tgsim_gossip_init) that never happens, so the
// generation never waits for a lagging delivery (an event per window instead cost ~20 us of host
// time per step).
int take_gen(Eng* E, Eng::GenWindow* w) {
  if (E->gen_free.empty()) return 0;
  *w = std::move(E->gen_free.front());
  E->gen_free.erase(E->gen_free.begin());
  if (w->retired_call && E->sim_calls < w->retired_call + E->emit_sets) {
    HIPCHK(hipStreamWaitEvent(E->st, E->ev_dst, 0));
    HIPCHK(hipStreamWaitEvent(E->st, E->ev_rt, 0));
  }
  return 0;
}

// After a late receipt the late window gen_q[from] and every window queued after it are dropped
// (their buffers go back to gen_free); the valid windows before it stay queued and can still be
// stepped (include/tgsim.h); the error stays (gossip_late).
void drop_gen(Eng* E, size_t from = 0) {
  for (size_t i = from; i < E->gen_q.size(); ++i) {
    E->gen_q_ticks -= E->gen_q[i].ticks;
    (void)retire_gen(E, std::move(E->gen_q[i]));
  }
  E->gen_q.erase(E->gen_q.begin() + static_cast<std::ptrdiff_t>(std::min(from, E->gen_q.size())), E->gen_q.end());
}

// Sparse or dense kernels for a window of n_in packets (commit: this is the window being launched;
// the streak counter advances).  Sparse steps (few packets per source, or more sources than the
// order kernel ranks): open queues run in the register-only k_sim_sparse, the rest in k_sim_list;
// dense steps: k_sim in heavy-first order.  The results are the same either way.
bool sparse_choice(Eng* E, uint64_t n_in, bool commit) {
  if (E->sparse_mode >= 0) return E->sparse_mode == 1;
  // dense traffic (C3, C5 at 100k peers; k_sim_sparse would defer every source with more than
  // 64 packets anyway): the LDS queue, in heavy-first order when ranked
  if (n_in >= 64ull * E->S) return false;
  // up to 64 packets per source (gossip, even at the flood's peak of ~20): the register-only
  // kernel wins unless the queues are too long for registers and it defers most sources to
  // k_sim_list (2 waves/SIMD).  The worklist size of the last sparse step (copied to pinned memory
  // behind it, read without waiting) decides; every 64th such step runs sparse again to re-measure
  if (E->next_sparse >= 0 && E->next_sparse_n == n_in) {
    const bool sp = E->next_sparse == 1;
    if (commit) {  // the choice made ahead (tgsim_sim_capacity) commits like a fresh one
      E->next_sparse = -1;
      E->dense_streak = sp ? 0 : E->dense_streak + 1;
    }
    return sp;
  }
  const uint32_t deferred = __atomic_load_n(E->h_work, __ATOMIC_RELAXED);
  const bool many = E->sparse_seen && static_cast<uint64_t>(E->dense_div) * deferred > E->S;
  const bool sp = !many || E->dense_streak + 1 >= 64;
  if (commit) {
    E->dense_streak = sp ? 0 : E->dense_streak + 1;
    E->next_sparse = -1;
  } else {
    E->next_sparse = sp ? 1 : 0;
    E->next_sparse_n = n_in;
  }
  return sp;
}

// The compact emit layout: a sparse window whose classic regions (the netem limit per source) would
// exceed kExactBoundBytes (24 GB per emit set at 1M peers) keeps emit_r records per source beyond 2
// per offered packet and a pool for the few sources that serve more.
bool compact_layout(Eng* E, uint64_t n_in, bool sparse) {
  return sparse && E->emit_compact &&
         (E->emit_compact == 2 ||
          (2 * n_in + static_cast<uint64_t>(kHeapCap) * E->S) * sizeof(tgsim_delivery) > kExactBoundBytes);
}
uint64_t emit_records(Eng* E, uint64_t n_in, bool compact) {  // the emit buffer of one window
  return compact ? 2 * n_in + static_cast<uint64_t>(E->emit_r + E->emit_pool) * E->S
                 : 2 * n_in + static_cast<uint64_t>(kHeapCap) * E->S;
}

// Records per destination bucket of a window (log2): room for about twice the window's offered
// packets per destination (a gossip window's records are about its offered packets), 8 to 64.
uint32_t bucket_log(uint64_t n_in, uint32_t n_dst) {
  const uint64_t want = 2 * n_in / std::max<uint32_t>(1, n_dst) + 4;
  uint32_t l = kBktLogMin;
  while (l < kBktLogMax && (1ull << l) < want) ++l;
  return l;
}

int run_sim(Eng* E, uint32_t n_ticks, bool local_hist = false) {
  int erc = check_sim_error(E);
  if (erc) return erc;
  erc = harvest_timing(E, false);
  if (erc) return erc;
  if (!E->gen_q.empty()) {
    if (!E->staged.empty()) return E->fail(-EBUSY, "host packets and generated traffic in one step");
    Eng::GenWindow& w = E->gen_q.front();
    int grc = resolve_gen(E, w);
    if (grc) {
      if (E->gossip_late) drop_gen(E);
      return grc;
    }
    if (n_ticks != w.ticks)
      return E->fail(-EINVAL, "generated window spans %u ticks, step is %u", w.ticks, n_ticks);
    std::swap(E->d_off, w.off);
    std::swap(E->d_in, w.in);
    E->n_in = w.n;
    E->gen_q_ticks -= w.ticks;
    int frc = retire_gen(E, std::move(w));  // the previous window's offsets: routing/delivery may read them
    E->gen_q.erase(E->gen_q.begin());
    if (frc) return frc;
    E->perm.clear();
  } else {
    int rc = stage_host_input(E, n_ticks);
    if (rc) return rc;
  }
  int rc = flush_config(E);
  if (rc) return rc;
  const bool sparse = sparse_choice(E, E->n_in, true);
  if (!sparse) ensure_wheel(E);
  const bool compact = compact_layout(E, E->n_in, sparse);
  const uint64_t emit_cap = emit_records(E, E->n_in, compact);
  HIPCHK(E->d_verdict.ensure(E->n_in ? E->n_in : 1));
  // the local delivery or routing two steps back read this emit pair
  HIPCHK(hipStreamWaitEvent(E->st, E->ev_local, 0));
  HIPCHK(E->d_emit.ensure(emit_cap));
  HIPCHK(E->d_emit_n.ensure(E->S));
  SimArgs a = base_sim_args(E);
  a.off = E->d_off.p;
  a.in = E->d_in.p;
  a.verdict = E->d_verdict.p;
  a.emit = E->d_emit.p;
  a.emit_n = E->d_emit_n.p;
  E->el = EmitRead{E->d_emit.p, nullptr, nullptr, kHeapCap};
  if (compact) {  // regions of 2 n_s + emit_r records, then the pool
    HIPCHK(E->d_pidx.ensure(E->S));
    a.emit_r = E->emit_r;
    a.emit_pool = E->d_emit.p + 2 * E->n_in + static_cast<uint64_t>(E->emit_r) * E->S;
    a.emit_pool_idx = E->d_pidx.p;
    a.emit_pool_cap = static_cast<uint32_t>(std::min<uint64_t>(static_cast<uint64_t>(E->emit_pool) * E->S, 0xFFFFFFFFull));
    E->el = EmitRead{E->d_emit.p, a.emit_pool, E->d_pidx.p, E->emit_r};
  }
  a.t0_ns = E->now_tick * E->o.tick_ns;
  a.horizon_ns = (E->now_tick + n_ticks) * E->o.tick_ns + E->o.lookahead_ns;
  const uint32_t n_wg = (E->S + kSpw - 1) / kSpw;
  const bool ordered = kSpw == 1 && E->S <= kOrderMaxSources;
  a.order = ordered && E->order_valid ? E->d_order.p : nullptr;
  a.stamps = nullptr;
  if (E->stamps_on) {
    HIPCHK(E->d_stamps.ensure(static_cast<size_t>(n_wg) * kStampSlots));
    a.stamps = E->d_stamps.p;
    E->n_stamp_wg = n_wg;
  }
  a.dst_cnt = nullptr;
  a.err_host = E->d_err_host;
  if (local_hist) {
    if (E->d_lcnt.cap < E->N) {
      HIPCHK(E->d_lcnt.ensure(E->N));
      HIPCHK(hipMemsetAsync(E->d_lcnt.p, 0, sizeof(uint64_t) * E->d_lcnt.cap, E->st));
    }
    a.dst_cnt = reinterpret_cast<unsigned long long*>(E->d_lcnt.p);
    // sparse windows: each record's destination slot from its histogram increment, so the scatter
    // takes no cursor atomic (TGSIM_DST_SLOT=0: the cursors, for A/B)
    a.dst_slot = sparse && E->dst_slot ? 1u : 0u;
    E->el.slot = a.dst_slot;
    // and, where nothing but the local delivery reads the records (no metrics, receipts folded in at
    // emission), straight into the destinations' buckets (TGSIM_DST_BKT=0: the emit records only)
    if (a.dst_slot && E->dst_bkt && !E->metrics_on) {
      HIPCHK(E->d_dbkt.ensure(static_cast<size_t>(E->N) << kBktLogMax));
      a.dst_bkt = E->d_dbkt.p;
      a.bkt_log = bucket_log(E->n_in, E->N);
      E->el.bkt = a.dst_bkt;
      E->el.bkt_log = a.bkt_log;
    }
  }
  if (E->gossip_on) {  // receipts at emission for the destinations of this shard
    a.g_first = E->d_gfirst.p;
    a.g_pend = E->d_gpend.p;
    a.g_fwd = E->d_gfwd.p;
    a.g_floods = E->gossip.n_floods;
    a.g_degree = E->gossip.degree;
  }
  a.worklist = nullptr;
  if (sparse) {
    // [0] the worklist's count, [1] k_sim_multi's, [2] emit-pool records claimed, [3] unused, the
    // worklist's sources, 8 words of TGSIM_DEFER_STATS, then k_sim_multi's sources
    if (E->d_work.cap < 2 * static_cast<size_t>(E->S) + 4 + 8) {
      HIPCHK(E->d_work.ensure(2 * static_cast<size_t>(E->S) + 4 + 8));
      HIPCHK(hipMemsetAsync(E->d_work.p, 0, sizeof(uint32_t) * E->d_work.cap, E->st));
    }
    a.worklist = E->d_work.p + 4;
    a.order = nullptr;  // (stamps, when on, are indexed by source: n_wg = S)
  }
  // the simulate kernels' span (bench: roofline): timing events cost the windows they bracket (a
  // timestamped marker per launch), so TGSIM_SIM_TIMING can sample every k-th window
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  const bool timed = E->sim_every && E->sim_count++ % E->sim_every == 0;
  if (timed) {
    HIPCHK(take_event(E, &ev0));
    HIPCHK(take_event(E, &ev1));
    HIPCHK(hipEventRecord(ev0, E->st));
  }
  if (sparse) {
    // the worklist counters start zeroed (at allocation, then by the kernel behind the last sparse
    // step, which also publishes them to pinned memory: no fill or copy on the stream per window)
    launch_sim_sparse(a, E->st, E->dm_work, __atomic_load_n(E->h_work, __ATOMIC_RELAXED));
    E->rotated = true;
  }
  else launch_sim(a, n_wg, E->st);
  HIPCHK(hipGetLastError());
  E->sim_calls++;  // behind the wait for this emit pair's last reader (ev_local): take_gen's count
  E->ev_sim_t = nullptr;
  if (timed) {
    HIPCHK(hipEventRecord(ev1, E->st));
    E->ev_pending.push_back({ev0, ev1, 1u});
    if (!E->metrics_on) E->ev_sim_t = ev1;  // (k_metrics_src follows k_sim on the stream)
  }
  if (sparse) {
    E->sparse_seen = true;
    E->sparse_windows++;
  }
  if (E->metrics_on) {
    MetricsArgs m;
    m.off = E->d_off.p;
    m.in = E->d_in.p;
    m.verdict = E->d_verdict.p;
    m.emit = E->el;
    m.emit_n = E->d_emit_n.p;
    m.state = E->d_state.p;
    m.n_src = E->S;
    m.src = E->d_msrc.p;
    m.hist = E->d_mhist.p;
    launch_metrics_src(m, E->st);
    HIPCHK(hipGetLastError());
  }
  // (no heavy-first order kernel behind a single window: on the simulate stream it delayed the next
  // window by its launch and ~9 us, more than the order saved -- sub-capacity storm 1.38 against
  // 1.51 G pkt/s, profiles/r06/ab_order/; the fused groups of tgsim_step_n keep theirs, once per group)
  (void)ordered;
  E->n_verdict = E->n_in;
  E->last_perm.swap(E->perm);
  E->perm.clear();
  E->now_tick += n_ticks;
  return 0;
}

int finish_sim_timing(Eng* E) {
  int rc = sync_stream(E);
  if (rc) return rc;
  return check_sim_error(E);
}

// The point on the simulate stream right behind the last window's k_sim: its timing event when it has
// one (each marker on the stream delays the next window's launch), else a marker of its own.
hipEvent_t sim_done_event(Eng* E) {
  if (E->ev_sim_t) return E->ev_sim_t;
  (void)hipEventRecord(E->ev_sim, E->st);
  return E->ev_sim;
}

// Groups the step's scheduled records by destination shard into `out` on the routing stream, after
// the step's k_sim and beside the next one (which writes the other emit pair): per-(rank, source)
// counts -> scan -> ordered scatter; the per-rank edges go to pinned host memory behind ev_route, so
// the host can launch the next step before it reads them (route_finish).
int route_launch(Eng* E, uint32_t n_ranks, const uint32_t* bounds, tgsim_delivery* out, size_t out_cap,
                 uint64_t slot_cap = 0, hipEvent_t routed = nullptr) {
  hipStream_t rs = E->rt_st;
  HIPCHK(hipStreamWaitEvent(rs, sim_done_event(E), 0));  // this step's k_sim
  RouteArgsHost h;
  memset(&h, 0, sizeof h);
  h.emit = E->el;
  h.emit_n = E->d_emit_n.p;
  h.off = E->d_off.p;
  h.n_src = E->S;
  h.n_ranks = n_ranks;
  for (uint32_t i = 0; i <= n_ranks && i < 9; ++i) h.bounds[i] = bounds[i];
  const uint64_t m = static_cast<uint64_t>(n_ranks) * E->S;
  HIPCHK(E->d_rcnt.ensure(m));
  HIPCHK(E->d_rpos.ensure(m + 1));
  HIPCHK(E->d_rblk.ensure((m + 1023) / 1024 + 1));
  HIPCHK(E->d_rtot.ensure(1));
  h.cnt = E->d_rcnt.p;
  h.pos = E->d_rpos.p;
  h.out = out;
  h.out_cap = out_cap;
  h.slot_cap = slot_cap;
  launch_route(h, 0, rs);
  HIPCHK(hipGetLastError());
  launch_scan(E->d_rcnt.p, E->d_rpos.p, m, E->d_rblk.p, E->d_rtot.p, rs);
  HIPCHK(hipGetLastError());
  launch_route(h, 1, rs);
  HIPCHK(hipGetLastError());
  // per-rank totals: pos[r * S] .. pos[(r + 1) * S], published to the slot's pinned words
  const uint32_t k = (E->route_head + E->route_n) % Eng::kRouteSlots;
  E->route_seq[k] = ++E->route_next_seq;
  if (!E->d_rsend.p) {
    HIPCHK(E->d_rsend.ensure(16 * Eng::kRouteSlots));
    HIPCHK(hipMemsetAsync(E->d_rsend.p, 0, sizeof(uint64_t) * 16 * Eng::kRouteSlots, rs));
  }
  launch_route_edges(E->d_rpos.p, E->S, n_ranks, E->h_edges + 16 * k, E->route_seq[k], rs, out, slot_cap, E->d_xerr,
                     0, E->d_rsend.p + 16 * k);
  HIPCHK(hipGetLastError());
  if (routed) HIPCHK(hipEventRecord(routed, rs));
  HIPCHK(hipEventRecord(E->ev_route[k], rs));
  HIPCHK(hipEventRecord(E->ev_rt, rs));
  HIPCHK(hipEventRecord(E->ev_local, rs));  // the last reader of this emit pair
  rotate_emit(E);
  E->route_ranks[k] = n_ranks;
  E->route_cap[k] = out_cap;
  E->route_n++;
  return 0;
}

// Spins until the device publishes `want` into the pinned word (kernels release it at system
// scope); `ev`, recorded after the publishing kernel, tells a fault from a slow step.
// The spin gives its core up only after a long wait (~ms): a yield on a loaded host handed the core
// away for a scheduler slice, ~0.9 ms added to every window of the closed gossip loop (1M peers:
// 3.3 against 5.6 G pkt/s in two runs of profiles/r06/ab_nofence/).
int wait_published(Eng* E, const uint64_t* word, uint64_t want, hipEvent_t ev, const char* what) {
  for (uint32_t it = 1;; ++it) {
    if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == want) return 0;
    spin_pause();
    if ((it & 255) == 0) {
      const hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) {
        if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == want) return 0;
        return E->fail(-EIO, "%s: the device finished without publishing its result", what);
      }
      if (q != hipErrorNotReady) HIPCHK(q);
      if (it > kSpinBeforeYield) std::this_thread::yield();
    }
  }
}

// Waits for the oldest launched step's records and edges (and, with wait_deliveries, for the
// asynchronous deliveries enqueued so far, whose input buffers the caller's next exchange may
// overwrite); per-rank counts into `counts`.
int route_finish(Eng* E, uint64_t* counts, bool wait_deliveries = true) {
  if (!E->route_n) return E->fail(-EINVAL, "no routed step pending");
  const uint32_t k = E->route_head;
  E->route_head = (k + 1) % Eng::kRouteSlots;
  E->route_n--;
  int rc = wait_published(E, &E->h_edges[16 * k + 15], E->route_seq[k], E->ev_route[k], "route (per-rank edges)");
  if (rc) return rc;
  if (wait_deliveries) HIPCHK(hipEventSynchronize(E->ev_dst));
  const uint32_t n_ranks = E->route_ranks[k];
  const uint64_t* edges = E->h_edges + 16 * k;
  for (uint32_t r = 0; r < n_ranks; ++r) counts[r] = edges[r + 1] - edges[r];
  if (edges[n_ranks] > E->route_cap[k])
    return E->fail(-ENOSPC, "route: %llu records exceed capacity %zu",
                   static_cast<unsigned long long>(edges[n_ranks]), E->route_cap[k]);
  rc = harvest_timing(E, false);
  if (rc) return rc;
  return check_sim_error(E);
}

int route(Eng* E, uint32_t n_ranks, const uint32_t* bounds, tgsim_delivery* out, size_t out_cap,
          uint64_t* counts) {
  int rc = route_launch(E, n_ranks, bounds, out, out_cap);
  if (rc) return rc;
  return route_finish(E, counts);
}

GossipArgs gossip_args(Eng* E, uint64_t win0, uint32_t n_ticks) {
  GossipArgs g;
  g.first = E->d_gfirst.p;
  g.fwd = E->d_gfwd.p;
  g.pend = E->d_gpend.p;
  g.nbr = E->d_gnbr.cap ? E->d_gnbr.p : nullptr;
  g.err = E->d_gerr.p;
  g.k0 = E->key0 ^ 0x3C6EF372u;
  g.k1 = E->key1 ^ 0xA54FF53Au;
  g.n_src = E->S;
  g.shard_begin = E->o.shard_begin;
  g.n_peers = E->N;
  g.n_floods = E->gossip.n_floods;
  g.degree = E->gossip.degree;
  g.msg_len = E->gossip.msg_len;
  g.n_ticks = n_ticks;
  g.tick_ns = E->o.tick_ns;
  g.win0 = win0;
  return g;
}

// Output of a delivery sort of n records: the drain buffer (grown, undrained tail compacted to the
// front) or, with TGSIM_OPT_DISCARD_DELIVERIES, a scratch buffer.
int delivery_out(Eng* E, uint64_t n, tgsim_delivery** out, hipStream_t sq) {
  if (E->o.flags & TGSIM_OPT_DISCARD_DELIVERIES) {
    HIPCHK(E->d_sorted.ensure(n ? n : 1));
    *out = E->d_sorted.p;
    return 0;
  }
  const uint64_t need = E->drain_head + E->drain_n + n;
  if (need > E->d_drain.cap) {
    DevBuf<tgsim_delivery> nb;
    HIPCHK(nb.ensure(E->drain_n + n));
    if (E->drain_n)
      HIPCHK(hipMemcpyAsync(nb.p, E->d_drain.p + E->drain_head, sizeof(tgsim_delivery) * E->drain_n,
                            hipMemcpyDeviceToDevice, sq));
    HIPCHK(hipStreamSynchronize(sq));
    E->d_drain.release();
    E->d_drain = nb;
    E->drain_head = 0;
  }
  *out = E->d_drain.p + E->drain_head + E->drain_n;
  E->drain_n += n;
  return 0;
}

// Records received by this shard (tgsim_deliver*, or the routed records of tgsim_step on a
// partial shard): histogram -> scan -> scatter -> per-destination order, on the delivery stream so
// that it overlaps the next step's k_sim.  It waits for the simulate stream's work so far (the
// records come from tgsim_step_sim, which completed them before returning), only for `wait` (the
// producer of d_in, e.g. the collective).
// check: read the record count back and reject records addressed to other shards.
// n_win > 1: the slotted input of a fused group (chunk c = source rank * n_win + window): the
// records are sorted per (window, destination) segment, so the output is the windows' deliveries
// in window order, in single-wave workgroups (beside the next group's k_sim_fused).
int deliver(Eng* E, const tgsim_delivery* in, uint64_t n, hipEvent_t wait, bool check, uint64_t slot = 0,
            uint32_t n_win = 1) {
  const uint32_t nd = E->S;  // destinations owned by this shard
  const uint64_t nseg = static_cast<uint64_t>(n_win) * nd;
  hipStream_t sq = E->dst_st;
  if (wait) HIPCHK(hipStreamWaitEvent(sq, wait, 0));
  hipEvent_t dv0 = nullptr, dv1 = nullptr;  // the delivery's span on its stream (bench: roofline.delivery)
  const bool timed = E->dv_every && E->dv_count++ % E->dv_every == 0;
  if (timed) {
    HIPCHK(take_event(E, &dv0));
    HIPCHK(take_event(E, &dv1));
    HIPCHK(hipEventRecord(dv0, sq));
  }
  if (E->d_dcnt.cap < nseg) {
    HIPCHK(E->d_dcnt.ensure(nseg));
    HIPCHK(hipMemsetAsync(E->d_dcnt.p, 0, sizeof(uint64_t) * E->d_dcnt.cap, sq));
  }
  HIPCHK(E->d_dpos.ensure(nseg));
  if (E->gossip_on) {  // receipts of the gossip workload (order-free: earliest tick wins), straight
                       // from the inbound records on the simulate stream, where the next window's
                       // generation runs: it waits for the records' arrival, not for any sort; records
                       // of this shard's own sources were folded in at emission
    if (E->S != E->N) {
      if (wait) HIPCHK(hipStreamWaitEvent(E->st, wait, 0));
      launch_gossip_recv_in(gossip_args(E, 0, 0), in, n, slot, true, E->st);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(E->ev_recv, E->st));
  }
  // slotted input: chunk by chunk over the counts in the headers, the grid sized for what a chunk
  // of this window can hold (2 records per offered packet), not for its capacity
  const uint64_t n_chunks = slot ? n / (slot + 1) : 0, hint = std::max<uint64_t>(2 * E->n_in, 65536);
  if (slot) launch_dst_slot(in, n_chunks, slot, hint, E->o.shard_begin, nd, E->d_dcnt.p, nullptr, sq, n_win);
  else launch_dst_hist(in, n, E->o.shard_begin, nd, E->d_dcnt.p, sq, slot, n_win);
  HIPCHK(hipGetLastError());
  int rc = 0;
  if (n_win > 1) {
    HIPCHK(E->d_doff.ensure(nseg + 1));
    HIPCHK(E->d_dblk.ensure((nseg + 1023) / 1024 + 1));
    HIPCHK(E->d_dtot.ensure(1));
    launch_scan_w(E->d_dcnt.p, E->d_doff.p, nseg, E->d_dblk.p, E->d_dtot.p, sq, E->d_dpos.p);
    HIPCHK(hipGetLastError());
  } else if (!check) {  // nothing on the host needs the count
    HIPCHK(E->d_doff.ensure(nd + 1));
    HIPCHK(E->d_dblk.ensure((nd + 1023) / 1024 + 1));
    HIPCHK(E->d_dtot.ensure(1));
    launch_scan(E->d_dcnt.p, E->d_doff.p, nd, E->d_dblk.p, E->d_dtot.p, sq, E->d_dpos.p, E->d_dcnt.p);
    HIPCHK(hipGetLastError());
  } else {
    uint64_t total = 0;
    rc = scan_counts(E, E->d_dcnt, E->d_doff, E->d_dblk, E->d_dtot, nd, &total, E->d_dpos.p, sq, nullptr, nullptr, true);
    if (rc) return rc;
    if (total != n) return E->fail(-EINVAL, "deliver: %llu of %llu records address other shards",
                                   static_cast<unsigned long long>(n - total), static_cast<unsigned long long>(n));
  }
  HIPCHK(E->d_scatter.ensure(n ? n : 1));
  if (slot) launch_dst_slot(in, n_chunks, slot, hint, E->o.shard_begin, nd, E->d_dpos.p, E->d_scatter.p, sq, n_win);
  else launch_dst_scatter(in, n, E->o.shard_begin, nd, E->d_dpos.p, E->d_scatter.p, sq, slot, n_win);
  HIPCHK(hipGetLastError());
  if (slot && !(E->o.flags & TGSIM_OPT_DISCARD_DELIVERIES)) {  // the drain needs the record count
    HIPCHK(hipMemcpyAsync(&E->h_dtot, E->d_dtot.p, sizeof(uint64_t), hipMemcpyDeviceToHost, sq));
    HIPCHK(hipStreamSynchronize(sq));
    n = E->h_dtot;
  }
  if (!E->gossip_on) HIPCHK(hipEventRecord(E->ev_recv, sq));
  tgsim_delivery* dst = nullptr;
  rc = delivery_out(E, n, &dst, sq);
  if (rc) return rc;
  if (n_win > 1) launch_dst_sort_w1(E->d_scatter.p, E->d_doff.p, E->d_dcnt.p, static_cast<uint32_t>(nseg), dst, sq);
  // (the scan cleared d_dcnt; slotted input: the hint is what the window's chunks can hold, not
  // their capacity, so that a gossip window's few records per destination take the flattened sort --
  // routed 1M-peer share at one rank: k_dst_sort_wide took 0.11 ms of a 0.38-ms window)
  else launch_dst_sort(E->d_scatter.p, E->d_doff.p, nullptr, nd, dst, sq, slot ? std::min(n, hint) : n, E->o.shard_begin);
  HIPCHK(hipGetLastError());
  if (E->metrics_on) {
    launch_metrics_dst(dst, E->d_doff.p, nd, E->d_mdst.p, E->d_mhist.p, sq);
    HIPCHK(hipGetLastError());
  }
  if (timed) {
    HIPCHK(hipEventRecord(dv1, sq));
    E->dv_pending.push_back({dv0, dv1, n_win});
  }
  HIPCHK(hipEventRecord(E->ev_dst, sq));
  return 0;
}

// The local delivery of one window on the delivery stream (after its k_sim): scan of the
// per-destination histogram -> scatter straight from the emit regions -> per-destination order.
int deliver_local_from(Eng* E, const EmitRead& emit, uint32_t* emit_n, uint64_t* lcnt,
                       const uint64_t* off, uint64_t n_in, hipEvent_t released) {
  const uint32_t nd = E->N;
  hipStream_t sq = E->dst_st;
  hipEvent_t dv0 = nullptr, dv1 = nullptr;  // the delivery's span on its stream (bench: roofline.delivery)
  const bool timed = E->dv_every && E->dv_count++ % E->dv_every == 0;
  if (timed) {
    HIPCHK(take_event(E, &dv0));
    HIPCHK(take_event(E, &dv1));
    HIPCHK(hipEventRecord(dv0, sq));
  }
  // a bucketed window: the scan outputs of its emit set (see Eng::d_sdoff), else the shared ones
  DevBuf<uint64_t>& doff = emit.bkt ? E->d_sdoff : E->d_doff;
  DevBuf<uint64_t>& dpos = emit.bkt ? E->d_sdpos : E->d_dpos;
  DevBuf<uint64_t>& dblk = emit.bkt ? E->d_sdblk : E->d_dblk;
  DevBuf<uint64_t>& dtot = emit.bkt ? E->d_sdtot : E->d_dtot;
  HIPCHK(doff.ensure(nd + 1));
  HIPCHK(dpos.ensure(nd));
  HIPCHK(dblk.ensure((nd + 1023) / 1024 + 1));
  HIPCHK(dtot.ensure(1));
  // single-wave workgroups for a dense window's delivery: it runs beside the next window's k_sim, whose
  // waves fill every CU's LDS and leave no room for a 4- or 16-wave block, so a 1,024-thread scan
  // waited for that k_sim to drain and the next k_sim for it (ev_local): 118 against ~97 us per
  // sub-capacity window (profiles/r06/open/).  Sparse (bucketed, lane-per-source) windows keep theirs.
  const bool single_wave = !emit.bkt && E->S < 65536;  // (C5's 100,000: the 4-wave forms, A/B'd there)
  if (single_wave) launch_scan_w(lcnt, doff.p, nd, dblk.p, dtot.p, sq, dpos.p, true);  // (clears lcnt)
  else launch_scan(lcnt, doff.p, nd, dblk.p, dtot.p, sq, dpos.p, lcnt);
  HIPCHK(hipGetLastError());
  const bool need_n = !(E->o.flags & TGSIM_OPT_DISCARD_DELIVERIES);
  // without the exact count (no host round trip): what the window's sources can emit, 2 per offered
  // packet plus the full netem limit per source.  Where that bound exceeds kExactBoundBytes (24 GB
  // of scatter and output buffers at 1M peers), deliver_slack queued items per source instead, and
  // k_deliver_guard checks the device's exact total: a window beyond it fails with -ENOSPC.  A
  // mid-run reshape (a faster link releasing a deep queue) reserves the full limit for the windows
  // after it; TGSIM_DELIVER_SLACK forces the bounded form (tests).
  const bool exact_fits = (2 * n_in + static_cast<uint64_t>(kHeapCap) * E->S) * sizeof(tgsim_delivery) <= kExactBoundBytes;
  const uint64_t slack =
      E->wide_windows || (exact_fits && !E->slack_forced) ? kHeapCap : std::min<uint64_t>(kHeapCap, E->deliver_slack);
  if (E->wide_windows) E->wide_windows--;
  uint64_t n = 2 * n_in + slack * E->S;
  if (need_n) {
    HIPCHK(hipMemcpyAsync(&E->h_dtot, dtot.p, sizeof(uint64_t), hipMemcpyDeviceToHost, sq));
    HIPCHK(hipStreamSynchronize(sq));
    n = E->h_dtot;
  }
  HIPCHK(E->d_scatter.ensure(n ? n : 1));
  const bool bounded = !need_n && slack < kHeapCap;
  EmitRead er = emit;
  if (bounded && emit.bkt) {  // the scatter and the sort check the total themselves (one dispatch fewer)
    er.guard_total = dtot.p;
    er.guard_cap = n;
  } else if (bounded) {
    launch_deliver_guard(dtot.p, n, emit_n, E->S, lcnt, doff.p, nd, E->d_err_host, sq);
    HIPCHK(hipGetLastError());
  }
  // (a bucketed window: only the records past their destination's bucket are in the emit records)
  launch_local_scatter(er, emit_n, off, E->S, 0, doff.p, dpos.p, E->d_scatter.p, sq, n_in, E->gossip_on, single_wave);
  HIPCHK(hipGetLastError());
  // the emit set and its histogram are free once scattered: the window two later may write them
  // while this one's per-destination sort still runs (the sort reads only the scatter buffer) --
  // unless the sort reads the window's buckets (released behind it, below)
  if (!emit.bkt) HIPCHK(hipEventRecord(released, sq));
  if (!E->gossip_on) HIPCHK(hipEventRecord(E->ev_recv, sq));
  tgsim_delivery* dst = nullptr;
  int rc = delivery_out(E, n, &dst, sq);
  if (rc) return rc;
  if (emit.bkt) {
    launch_dst_sort_bkt(emit.bkt, emit.bkt_log, E->d_scatter.p, doff.p, nd, dst, sq, er.guard_total, er.guard_cap,
                        E->d_err_host);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(released, sq));
  } else {
    launch_dst_sort(E->d_scatter.p, doff.p, nullptr, nd, dst, sq, need_n ? n : n_in, 0, single_wave);
  }
  HIPCHK(hipGetLastError());
  if (E->metrics_on) {
    launch_metrics_dst(dst, doff.p, nd, E->d_mdst.p, E->d_mhist.p, sq);
    HIPCHK(hipGetLastError());
  }
  if (timed) {
    HIPCHK(hipEventRecord(dv1, sq));
    E->dv_pending.push_back({dv0, dv1, 1u});
  }
  return 0;
}

// Single shard: k_sim counted every emitted record per destination, so the step needs no host
// round trip: scan -> scatter straight from the emit regions -> per-destination order, on the
// delivery stream beside the next step's k_sim (which writes the other emit pair).  Only the drain
// bookkeeping needs the record count on the host.
int deliver_local(Eng* E) {
  hipStream_t sq = E->dst_st;
  HIPCHK(hipStreamWaitEvent(sq, sim_done_event(E), 0));  // this step's k_sim
  if (E->gossip_on)  // receipts of the gossip workload: folded into k_sim at emission; the next
                     // window's generation waits for nothing on the delivery side
    HIPCHK(hipEventRecord(E->ev_recv, E->st));

  int rc = deliver_local_from(E, E->el, E->d_emit_n.p, E->d_lcnt.p, E->d_off.p, E->n_in, E->ev_local);
  if (rc) return rc;
  HIPCHK(hipEventRecord(E->ev_dst, sq));
  rotate_emit(E);
  return 0;
}

// tgsim_step_n's fused path: can the next g windows run in one k_sim_fused launch?  Generated
// dense windows on an engine that owns every peer, no host packets, no per-window diagnostics.
bool fusable(Eng* E, uint32_t n_ticks, uint32_t g, bool routed = false) {
  if (g < 2 || (E->S != E->N && !routed) || !E->staged.empty() || E->gen_q.size() < g || E->metrics_on ||
      E->gossip_on || E->sparse_mode == 1 || kSpw != 1)
    return false;
  for (uint32_t i = 0; i < g; ++i)
    if (E->gen_q[i].ticks != n_ticks || E->gen_q[i].n < 64ull * E->S) return false;  // sparse windows
  return true;
}

// g consecutive windows in one k_sim_fused launch, then the g local deliveries on the delivery
// stream (beside the next group's launch, which writes the other parity's buffer sets).
struct GroupRoute {  // a sharded group: the windows' records routed into slotted chunks
  uint32_t n_ranks;
  const uint32_t* bounds;
  tgsim_delivery* out;  // n_ranks x g chunks of (slot_cap + 1) records, rank-major
  uint64_t slot_cap;
  hipEvent_t routed;
};

int step_fused(Eng* E, uint32_t n_ticks, uint32_t g, const GroupRoute* gr = nullptr) {
  int rc = check_sim_error(E);
  if (rc) return rc;
  rc = harvest_timing(E, false);
  if (rc) return rc;
  rc = flush_config(E);  // effective from the first window, as for g tgsim_step calls
  if (rc) return rc;
  const uint32_t p = E->fgrp;
  Eng::GenWindow win[kFuseMax];
  for (uint32_t i = 0; i < g; ++i) win[i] = std::move(E->gen_q[i]);
  E->gen_q.erase(E->gen_q.begin(), E->gen_q.begin() + g);
  E->gen_q_ticks -= static_cast<uint64_t>(g) * n_ticks;
  HIPCHK(hipStreamWaitEvent(E->st, E->ev_fgrp[p], 0));  // the deliveries that last read set p
  if (E->rotated) {  // the fused kernels' bounded loads read every queue from slot 0
    launch_unrotate(E->d_heap.p, E->d_state.p, E->S, E->st);
    HIPCHK(hipGetLastError());
    E->rotated = false;
  }
  if (E->d_done.cap < E->S) {
    HIPCHK(E->d_done.ensure(E->S));
    HIPCHK(hipMemsetAsync(E->d_done.p, 0, sizeof(uint32_t) * E->d_done.cap, E->st));
    HIPCHK(E->d_ticket.ensure(1));
    HIPCHK(hipMemsetAsync(E->d_ticket.p, 0, sizeof(uint32_t), E->st));
    E->step_no = E->ticket_no = 0;
  }
  ensure_wheel(E);
  SimArgs a = base_sim_args(E);
  const bool ordered = E->S <= kOrderMaxSources;
  a.order = ordered && E->order_valid ? E->d_order.p : nullptr;
  FusedArgs f{};
  const uint64_t nseg = static_cast<uint64_t>(g) * E->N;  // (window, destination) segments
  for (auto& lc : E->f_lcnt)
    if (lc.cap < static_cast<uint64_t>(kFuseMax) * E->N) {
      HIPCHK(lc.ensure(static_cast<uint64_t>(kFuseMax) * E->N));
      HIPCHK(hipMemsetAsync(lc.p, 0, sizeof(uint64_t) * lc.cap, E->st));
    }
  uint64_t rec_bound = 0, n_max = 0;  // records the group's windows can emit; largest window
  for (uint32_t i = 0; i < g; ++i) {
    rec_bound += 2 * win[i].n + static_cast<uint64_t>(kHeapCap) * E->S;
    n_max = std::max(n_max, win[i].n);
  }
  // every buffer set of both parities sized at once (the first group pays the allocations, not a
  // later one in the middle of a run)
  const uint32_t n_sets = std::max(static_cast<uint32_t>(E->fuse_max), g);
  for (auto& grp : E->fset)
    for (uint32_t i = 0; i < n_sets; ++i) {
      HIPCHK(grp[i].emit.ensure(2 * n_max + static_cast<uint64_t>(kHeapCap) * E->S));
      HIPCHK(grp[i].emit_n.ensure(E->S));
    }
  HIPCHK(E->d_verdict.ensure(n_max ? n_max : 1));
  for (uint32_t i = 0; i + 1 < n_sets; ++i) HIPCHK(E->f_verdict[i].ensure(n_max ? n_max : 1));
  if (!gr) {  // the group delivery's scratch, for the largest group
    const uint64_t segs = static_cast<uint64_t>(E->fuse_max) * E->N;
    const uint64_t recs = static_cast<uint64_t>(E->fuse_max) * (2 * n_max + static_cast<uint64_t>(kHeapCap) * E->S);
    HIPCHK(E->d_doff.ensure(segs + 1));
    HIPCHK(E->d_dpos.ensure(segs));
    HIPCHK(E->d_dblk.ensure((segs + 1023) / 1024 + 1));
    HIPCHK(E->d_scatter.ensure(recs));
    if (E->o.flags & TGSIM_OPT_DISCARD_DELIVERIES) HIPCHK(E->d_sorted.ensure(recs));
  }
  for (uint32_t i = 0; i < g; ++i) {
    Eng::LocalSet& ls = E->fset[p][i];
    DevBuf<uint8_t>& vb = i + 1 == g ? E->d_verdict : E->f_verdict[i];
    const uint64_t t0 = (E->now_tick + static_cast<uint64_t>(i) * n_ticks) * E->o.tick_ns;
    f.w[i] = {win[i].off.p, win[i].in.p, vb.p, ls.emit.p, ls.emit_n.p,
              gr ? nullptr : reinterpret_cast<unsigned long long*>(E->f_lcnt[p].p + static_cast<uint64_t>(i) * E->N),
              t0, t0 + n_ticks * E->o.tick_ns + E->o.lookahead_ns};
  }
  a.stamps = nullptr;
  if (E->stamps_on) {  // diagnostics: one stamp row per (window, dispatch position), window-major
    HIPCHK(E->d_stamps.ensure(static_cast<size_t>(g) * E->S * kStampSlots));
    a.stamps = E->d_stamps.p;
    E->n_stamp_wg = static_cast<uint64_t>(g) * E->S;
  }
  f.n_win = g;
  f.prio_n = a.order ? E->prio_heavy : 0;
  f.step_base = E->step_no;
  f.ticket_base = E->ticket_no;
  f.ticket = E->d_ticket.p;
  f.done = E->d_done.p;
  hipEvent_t ev0, ev1;
  HIPCHK(take_event(E, &ev0));
  HIPCHK(take_event(E, &ev1));
  HIPCHK(hipEventRecord(ev0, E->st));
  if (!E->fused_wgs) {
    E->fused_wgs = sim_fused_resident();
  }
  // a sharded group's exchange (RCCL) and deliveries need CU slots while the next group simulates:
  // there a persistent grid holds kRoutedGridPct of the resident workgroups (engine_persist_routed)
  f.persistent = gr ? (E->routed_pct ? 1u : 0u) : 1u;
  const uint32_t wgs = gr && E->routed_pct ? std::max(1u, E->fused_wgs * std::min(E->routed_pct, 100u) / 100u)
                                           : E->fused_wgs;
  launch_sim_fused(a, f, wgs, E->st);
  HIPCHK(hipGetLastError());
  E->sim_calls++;  // behind the wait for set p's last readers (ev_fgrp): take_gen's count
  HIPCHK(hipEventRecord(ev1, E->st));
  E->ev_pending.push_back({ev0, ev1, g});
  E->step_no += g;
  // every workgroup of the persistent grid claims until a claim fails: the counter advances by the
  // tickets (g per source window-major, one source-major) plus one failed claim per workgroup
  const uint32_t tickets = g * E->S;
  E->ticket_no += tickets + (f.persistent ? std::min(wgs, tickets) : 0u);
  E->fused_windows += g;
  if (ordered) {  // the next launch's dispatch order: the last window's HTB records, heaviest first
    HIPCHK(E->d_order.ensure(E->S));
    launch_order(E->fset[p][g - 1].emit_n.p, E->S, E->d_order.p, E->st);
    HIPCHK(hipGetLastError());
    E->order_valid = true;
  }
  if (gr) {  // sharded: each window's records into its (rank, window) chunks, on the routing stream
    hipStream_t rs = E->rt_st;
    HIPCHK(hipEventRecord(E->ev_sim, E->st));
    HIPCHK(hipStreamWaitEvent(rs, E->ev_sim, 0));
    const uint64_t m = static_cast<uint64_t>(gr->n_ranks) * E->S;
    HIPCHK(E->d_rcnt.ensure(m));
    HIPCHK(E->d_rpos.ensure(m + 1));
    HIPCHK(E->d_rblk.ensure((m + 1023) / 1024 + 1));
    HIPCHK(E->d_rtot.ensure(1));
    const uint32_t k = (E->route_head + E->route_n) % Eng::kRouteSlots;
    E->route_seq[k] = ++E->route_next_seq;
    for (uint32_t i = 0; i < g; ++i) {
      RouteArgsHost h;
      memset(&h, 0, sizeof h);
      h.emit = EmitRead{E->fset[p][i].emit.p, nullptr, nullptr, kHeapCap};  // fused windows: classic layout
      h.emit_n = E->fset[p][i].emit_n.p;
      h.off = win[i].off.p;
      h.n_src = E->S;
      h.n_ranks = gr->n_ranks;
      for (uint32_t r = 0; r <= gr->n_ranks && r < 9; ++r) h.bounds[r] = gr->bounds[r];
      h.cnt = E->d_rcnt.p;
      h.pos = E->d_rpos.p;
      h.out = gr->out + static_cast<uint64_t>(i) * (gr->slot_cap + 1);
      h.out_cap = static_cast<uint64_t>(gr->n_ranks) * g * (gr->slot_cap + 1);
      h.slot_cap = gr->slot_cap;
      h.chunk_stride = static_cast<uint64_t>(g) * (gr->slot_cap + 1);
      h.waves_per_block = 1;  // beside the next group's k_sim_fused (see k_scan_w1)
      launch_route(h, 0, rs);
      HIPCHK(hipGetLastError());
      launch_scan_w(E->d_rcnt.p, E->d_rpos.p, m, E->d_rblk.p, E->d_rtot.p, rs, nullptr);
      HIPCHK(hipGetLastError());
      launch_route(h, 1, rs);
      HIPCHK(hipGetLastError());
      launch_route_edges(E->d_rpos.p, E->S, gr->n_ranks, E->h_edges + 16 * k, E->route_seq[k], rs, h.out,
                         gr->slot_cap, E->d_xerr, h.chunk_stride);
      HIPCHK(hipGetLastError());
    }
    if (gr->routed) HIPCHK(hipEventRecord(gr->routed, rs));
    HIPCHK(hipEventRecord(E->ev_route[k], rs));
    HIPCHK(hipEventRecord(E->ev_rt, rs));
    HIPCHK(hipEventRecord(E->ev_fgrp[p], rs));  // the last reader of buffer set p
    E->route_ranks[k] = gr->n_ranks;
    E->route_cap[k] = static_cast<size_t>(gr->n_ranks) * g * (gr->slot_cap + 1);
    E->route_n++;
  } else {
    // the group's deliveries, beside the next launch: one scan over the (window, destination)
    // counts, one scatter of every window's emit regions, one sort per segment; the sorted output is
    // window 0's deliveries, then window 1's, ... (the drain order of g tgsim_step calls)
    hipStream_t sq = E->dst_st;
    HIPCHK(hipEventRecord(E->ev_sim, E->st));
    HIPCHK(hipStreamWaitEvent(sq, E->ev_sim, 0));
    HIPCHK(E->d_doff.ensure(nseg + 1));
    HIPCHK(E->d_dpos.ensure(nseg));
    HIPCHK(E->d_dblk.ensure((nseg + 1023) / 1024 + 1));
    HIPCHK(E->d_dtot.ensure(1));
    launch_scan_w(E->f_lcnt[p].p, E->d_doff.p, nseg, E->d_dblk.p, E->d_dtot.p, sq, E->d_dpos.p);
    HIPCHK(hipGetLastError());
    uint64_t n_rec = rec_bound;
    if (!(E->o.flags & TGSIM_OPT_DISCARD_DELIVERIES)) {
      HIPCHK(hipMemcpyAsync(&E->h_dtot, E->d_dtot.p, sizeof(uint64_t), hipMemcpyDeviceToHost, sq));
      HIPCHK(hipStreamSynchronize(sq));
      n_rec = E->h_dtot;
    }
    HIPCHK(E->d_scatter.ensure(n_rec ? n_rec : 1));
    GroupDeliver gd{};
    for (uint32_t i = 0; i < g; ++i) {
      gd.emit[i] = E->fset[p][i].emit.p;
      gd.emit_n[i] = E->fset[p][i].emit_n.p;
      gd.off[i] = win[i].off.p;
    }
    gd.n_src = E->S;
    gd.n_dst = E->N;
    gd.pos = E->d_dpos.p;
    gd.out = E->d_scatter.p;
    launch_local_scatter_group(gd, g, sq);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(E->ev_recv, sq));
    tgsim_delivery* dst = nullptr;
    rc = delivery_out(E, n_rec, &dst, sq);
    if (rc) return rc;
    launch_dst_sort_w1(E->d_scatter.p, E->d_doff.p, E->f_lcnt[p].p, static_cast<uint32_t>(nseg), dst, sq);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(E->ev_fgrp[p], sq));
    HIPCHK(hipEventRecord(E->ev_dst, E->dst_st));
  }
  E->fgrp = p ^ 1;
  // the last window's input stays the engine's current input (as after tgsim_step); the replaced
  // buffers and the other windows go back to the free list (a generation waits for ev_dst first)
  std::swap(E->d_off, win[g - 1].off);
  std::swap(E->d_in, win[g - 1].in);
  E->n_in = win[g - 1].n;
  E->n_verdict = E->n_in;
  for (uint32_t i = 0; i < g; ++i) {
    rc = retire_gen(E, std::move(win[i]), true);
    if (rc) return rc;
  }
  E->perm.clear();
  E->last_perm.clear();
  E->now_tick += static_cast<uint64_t>(g) * n_ticks;
  return 0;
}

Eng* as_eng(void* e) { return static_cast<Eng*>(e); }

}  // namespace

namespace tgsim {
CommSlot* engine_comm_slot(void* e) { return e ? &as_eng(e)->comm : nullptr; }
int engine_device(void* e) { return as_eng(e)->dev; }
uint32_t engine_peers(void* e) { return as_eng(e)->N; }
void engine_shard(void* e, uint32_t* begin, uint32_t* end) {
  *begin = as_eng(e)->o.shard_begin;
  *end = as_eng(e)->o.shard_end;
}
int engine_fail(void* e, int code, const char* msg) { return as_eng(e)->fail(code, "%s", msg); }
void engine_persist_routed(void* e, uint32_t pct) { as_eng(e)->routed_pct = pct; }
const uint64_t* engine_route_counts_dev(void* e) {
  Eng* E = as_eng(e);
  return E->route_n && E->d_rsend.p ? E->d_rsend.p + 16 * E->route_head : nullptr;
}
int engine_route_max(void* e, uint64_t* out) {
  Eng* E = as_eng(e);
  *out = 0;
  if (!E->d_rsend.p) return 0;
  HIPCHK(hipStreamSynchronize(E->rt_st));
  uint64_t m[2 * Eng::kRouteSlots] = {};
  for (uint32_t k = 0; k < Eng::kRouteSlots; ++k)
    HIPCHK(hipMemcpy(&m[k], E->d_rsend.p + 16 * k + 8, sizeof(uint64_t), hipMemcpyDeviceToHost));
  for (uint32_t k = 0; k < Eng::kRouteSlots; ++k) *out = std::max(*out, m[k]);
  return 0;
}
int engine_record_routed(void* e, hipEvent_t ev) {
  Eng* E = as_eng(e);
  HIPCHK(hipEventRecord(ev, E->rt_st));
  return 0;
}
}  // namespace tgsim

namespace {


}  // namespace

// ================================================================================================
extern "C" {

uint32_t tgsim_abi_version(void) { return TGSIM_ABI_VERSION; }

int tgsim_create(const tgsim_opts* opts, void** out) {
  if (!opts || !out) return -EINVAL;
  *out = nullptr;
  if (opts->abi_version != TGSIM_ABI_VERSION) return -EPROTO;
  if (opts->n_peers == 0) return -EINVAL;
  Eng* E = new Eng();
  E->o = *opts;
  if (E->o.shard_begin == 0 && E->o.shard_end == 0) E->o.shard_end = E->o.n_peers;
  if (E->o.shard_begin >= E->o.shard_end || E->o.shard_end > E->o.n_peers) {
    delete E;
    return -EINVAL;
  }
  if (!E->o.tick_ns) E->o.tick_ns = 1000;
  if (!E->o.queue_limit) E->o.queue_limit = 1000;
  if (E->o.queue_limit > kHeapCap) {
    delete E;
    return -EINVAL;
  }
  if (!E->o.subnet_base) E->o.subnet_base = 16u << 24;
  E->N = E->o.n_peers;
  E->S = E->o.shard_end - E->o.shard_begin;
  E->key0 = static_cast<uint32_t>(E->o.seed);
  E->key1 = static_cast<uint32_t>(E->o.seed >> 32);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    delete E;
    return -ENODEV;  // no GPU: the engine has no CPU fallback by design
  }
  E->dev = E->o.device >= 0 ? E->o.device : 0;
  if (E->o.device < 0) (void)hipGetDevice(&E->dev);
  int rc = 0;
  auto bail = [&](int code) {
    tgsim_destroy(E);
    return code;
  };
  if ((rc = E->hip(hipSetDevice(E->dev), "hipSetDevice"))) return bail(rc);
  if ((rc = E->hip(hipStreamCreateWithFlags(&E->st, hipStreamNonBlocking), "stream"))) return bail(rc);
  // the delivery stream gets a priority of its own (so ROCclr puts it on a hardware queue of its
  // own, and the delivery of one step runs beside the next k_sim instead of behind it in one
  // queue): the lowest, since the delivery is off the critical path (next k_sim; the gossip loop's
  // generation) and at high priority its waves were dispatched first (A/B: storm +1.2 %, 1M-peer
  // gossip +3 % at low priority)
  int prio_lo = 0, prio_hi = 0;
  if ((rc = E->hip(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi), "stream"))) return bail(rc);
  if ((rc = E->hip(hipStreamCreateWithPriority(&E->dst_st, hipStreamNonBlocking, prio_lo), "stream")))
    return bail(rc);
  if ((rc = E->hip(hipStreamCreateWithPriority(&E->rt_st, hipStreamNonBlocking, prio_hi), "stream")))
    return bail(rc);
  if ((rc = E->hip(hipEventCreateWithFlags(&E->ev_rt, hipEventDisableTiming), "event"))) return bail(rc);
  if ((rc = E->hip(hipEventRecord(E->ev_rt, E->rt_st), "event"))) return bail(rc);
  if ((rc = E->hip(hipEventCreateWithFlags(&E->ev_dst, hipEventDisableTiming), "event"))) return bail(rc);
  if ((rc = E->hip(hipEventCreateWithFlags(&E->ev_sim, kEvSync), "event"))) return bail(rc);
  if ((rc = E->hip(hipEventRecord(E->ev_dst, E->dst_st), "event"))) return bail(rc);
  if ((rc = E->hip(hipEventCreateWithFlags(&E->ev_recv, kEvSync), "event"))) return bail(rc);
  if ((rc = E->hip(hipEventRecord(E->ev_recv, E->dst_st), "event"))) return bail(rc);
  for (hipEvent_t* ev : {&E->ev_local, &E->ev_local_alt, &E->ev_local_alt2}) {
    if ((rc = E->hip(hipEventCreateWithFlags(ev, kEvSync), "event"))) return bail(rc);
    if ((rc = E->hip(hipEventRecord(*ev, E->dst_st), "event"))) return bail(rc);
  }
  if ((rc = E->hip(hipHostMalloc(reinterpret_cast<void**>(&E->h_err), sizeof(uint64_t),
                                 hipHostMallocCoherent | hipHostMallocMapped), "pinned")))
    return bail(rc);
  *E->h_err = 0;
  if ((rc = E->hip(hipHostMalloc(reinterpret_cast<void**>(&E->h_xerr), sizeof(uint32_t),
                                 hipHostMallocCoherent | hipHostMallocMapped), "pinned")))
    return bail(rc);
  *E->h_xerr = 0;
  if ((rc = E->hip(hipHostMalloc(reinterpret_cast<void**>(&E->h_work), 2 * sizeof(uint32_t),
                                 hipHostMallocCoherent | hipHostMallocMapped), "pinned")))
    return bail(rc);
  E->h_work[0] = E->h_work[1] = 0;
  if ((rc = E->hip(hipHostGetDevicePointer(reinterpret_cast<void**>(&E->dm_work), E->h_work, 0), "pinned")))
    return bail(rc);
  if ((rc = E->hip(hipHostGetDevicePointer(reinterpret_cast<void**>(&E->d_xerr), E->h_xerr, 0), "pinned")))
    return bail(rc);
  if ((rc = E->hip(hipHostMalloc(reinterpret_cast<void**>(&E->h_gerr), sizeof(uint32_t)), "pinned"))) return bail(rc);
  *E->h_gerr = 0;
  if ((rc = E->hip(hipHostMalloc(reinterpret_cast<void**>(&E->h_pub), 8 * sizeof(uint64_t),
                                 hipHostMallocCoherent | hipHostMallocMapped), "pinned")))
    return bail(rc);
  memset(E->h_pub, 0, 8 * sizeof(uint64_t));
  if ((rc = E->hip(hipEventCreateWithFlags(&E->ev_gpub, hipEventDisableTiming), "event"))) return bail(rc);
  if ((rc = E->hip(hipHostGetDevicePointer(reinterpret_cast<void**>(&E->dm_pub), E->h_pub, 0), "pinned")))
    return bail(rc);
  if ((rc = E->hip(hipEventCreateWithFlags(&E->ev_pub, hipEventDisableTiming), "event"))) return bail(rc);
  if ((rc = E->hip(hipHostGetDevicePointer(reinterpret_cast<void**>(&E->d_err_host), E->h_err, 0), "pinned")))
    return bail(rc);

  if ((rc = E->hip(hipHostMalloc(reinterpret_cast<void**>(&E->h_edges), 16 * Eng::kRouteSlots * sizeof(uint64_t),
                                 hipHostMallocCoherent | hipHostMallocMapped),
                   "pinned")))
    return bail(rc);
  memset(E->h_edges, 0, 16 * Eng::kRouteSlots * sizeof(uint64_t));
  for (hipEvent_t& ev : E->ev_route)
    if ((rc = E->hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event"))) return bail(rc);
  *E->h_err = 0;
  E->stamps_on = getenv("TGSIM_STAMPS") != nullptr;
  if (const char* sp = getenv("TGSIM_SPARSE")) E->sparse_mode = atoi(sp) ? 1 : 0;
  if (const char* st = getenv("TGSIM_SIM_TIMING")) E->sim_every = static_cast<uint32_t>(std::max(0, atoi(st)));
  if (const char* dv = getenv("TGSIM_DV_TIMING")) E->dv_every = static_cast<uint32_t>(std::max(0, atoi(dv)));
  if (E->sim_every || E->dv_every) {  // the timing events, created here rather than in the step path
    E->ev_pool.resize(kEventPool);
    for (hipEvent_t& ev : E->ev_pool)
      if ((rc = E->hip(hipEventCreateWithFlags(&ev, kEvTiming), "event"))) {
        ev = nullptr;
        return bail(rc);
      }
  }
  if (const char* ec = getenv("TGSIM_EMIT_COMPACT")) E->emit_compact = std::min(std::max(atoi(ec), 0), 2);
  if (const char* ds = getenv("TGSIM_DST_SLOT")) E->dst_slot = atoi(ds) != 0;
  if (const char* db = getenv("TGSIM_DST_BKT")) E->dst_bkt = atoi(db) != 0;
  // (a shard of a multi-GPU run keeps two: its deliveries are not bucketed, and the 8-rank C4 test's
  // memory budget, VERDICT r04 item 7, has no room for a third)
  E->emit_sets = E->S == E->N ? 3u : 2u;
  if (const char* es = getenv("TGSIM_EMIT_SETS")) E->emit_sets = atoi(es) == 2 ? 2u : 3u;
  if (const char* er = getenv("TGSIM_EMIT_R")) E->emit_r = static_cast<uint32_t>(std::min(std::max(1, atoi(er)), 1024));
  if (const char* ep = getenv("TGSIM_EMIT_POOL")) E->emit_pool = static_cast<uint32_t>(std::min(std::max(0, atoi(ep)), 4096));
  if (const char* ds = getenv("TGSIM_DELIVER_SLACK")) {
    E->deliver_slack = strtoull(ds, nullptr, 10);
    E->slack_forced = true;
  }
  if (const char* fz = getenv("TGSIM_FUSE")) E->fuse_max = std::max(1, std::min(atoi(fz), static_cast<int>(kFuseMax)));
  for (hipEvent_t& ev : E->ev_fgrp) {
    if ((rc = E->hip(hipEventCreateWithFlags(&ev, kEvSync), "event"))) return bail(rc);
    if ((rc = E->hip(hipEventRecord(ev, E->dst_st), "event"))) return bail(rc);
  }
  E->enabled.assign(E->N, 1);  // containers start attached to the data network (local_docker.go:459)
  E->ip6_set.assign(E->N, 0);
  E->ip6.resize(E->N);
  E->k8s_init.assign(E->N, 0);
  E->gone.assign(E->N, 0);
  E->link_gen.assign(E->N, 0);
  E->ip.resize(E->N);
  for (uint32_t i = 0; i < E->N; ++i) E->ip[i] = E->o.subnet_base + 2 + i;
  E->src.resize(E->S);
  for (uint32_t s = 0; s < E->S; ++s) reset_source(E, s);
  E->patch_n = 0;  // the initial state needs no patch
  E->patch_gen++;
  E->any_patch = false;
  if ((rc = E->hip(E->d_params.ensure(E->S), "alloc params"))) return bail(rc);
  if ((rc = E->hip(E->d_state.ensure(E->S), "alloc state"))) return bail(rc);
  if ((rc = E->hip(E->d_enabled.ensure(E->N), "alloc enabled"))) return bail(rc);
  if ((rc = E->hip(E->d_ip.ensure(E->N), "alloc ip"))) return bail(rc);
  if ((rc = E->hip(E->d_heap.ensure(static_cast<size_t>(E->S) * kHeapCap), "alloc heap"))) return bail(rc);
  if ((rc = E->hip(E->d_ring.ensure(static_cast<size_t>(E->S) * kHeapCap), "alloc ring"))) return bail(rc);
  if ((rc = E->hip(E->d_gen_seq.ensure(E->S), "alloc gen_seq"))) return bail(rc);
  if ((rc = E->hip(E->d_stats.ensure(kStSlots * kStatCopies), "alloc stats"))) return bail(rc);
  // K7 sync counters: device table, pinned mirror and result/marker words, their own stream
  // (the sync stream is created at the first signal: HIP maps the streams of a process onto
  // GPU_MAX_HW_QUEUES hardware queues, and an idle fifth stream made the exchange share a queue
  // with the simulate stream)
  if ((rc = E->hip(hipEventCreateWithFlags(&E->ev_sig, hipEventDisableTiming), "event"))) return bail(rc);
  if ((rc = E->hip(E->d_sync.ensure(kStates), "alloc sync"))) return bail(rc);
  if ((rc = E->hip(hipMemset(E->d_sync.p, 0, sizeof(unsigned long long) * kStates), "memset"))) return bail(rc);
  if ((rc = E->hip(hipHostMalloc(reinterpret_cast<void**>(&E->h_mirror), sizeof(uint64_t) * kStates,
                                 hipHostMallocCoherent | hipHostMallocMapped), "pinned")))
    return bail(rc);
  memset(E->h_mirror, 0, sizeof(uint64_t) * kStates);
  if ((rc = E->hip(hipHostGetDevicePointer(reinterpret_cast<void**>(&E->dm_mirror), E->h_mirror, 0), "pinned")))
    return bail(rc);
  if ((rc = E->hip(hipHostMalloc(reinterpret_cast<void**>(&E->h_sig), 2 * sizeof(uint64_t),
                                 hipHostMallocCoherent | hipHostMallocMapped), "pinned")))
    return bail(rc);
  E->h_sig[0] = E->h_sig[1] = 0;
  if ((rc = E->hip(hipHostGetDevicePointer(reinterpret_cast<void**>(&E->dm_sig), E->h_sig, 0), "pinned")))
    return bail(rc);
  if ((rc = E->hip(E->d_off.ensure(E->S + 1), "alloc off"))) return bail(rc);
  if ((rc = E->hip(E->d_in.ensure(1), "alloc in"))) return bail(rc);
  if ((rc = E->hip(hipMemset(E->d_state.p, 0, sizeof(SrcState) * E->S), "memset"))) return bail(rc);
  if ((rc = E->hip(hipMemset(E->d_gen_seq.p, 0, sizeof(uint32_t) * E->S), "memset"))) return bail(rc);
  if ((rc = E->hip(hipMemset(E->d_stats.p, 0, sizeof(unsigned long long) * kStSlots * kStatCopies), "memset")))
    return bail(rc);
  E->metrics_on = (E->o.flags & TGSIM_OPT_METRICS) != 0;
  if (E->metrics_on) {
    const size_t ns = static_cast<size_t>(E->S) * kMetricSrcWords, nd = static_cast<size_t>(E->S) * kMetricDstWords;
    if ((rc = E->hip(E->d_msrc.ensure(ns), "alloc metrics"))) return bail(rc);
    if ((rc = E->hip(E->d_mdst.ensure(nd), "alloc metrics"))) return bail(rc);
    if ((rc = E->hip(E->d_mhist.ensure(2 * kMetricBins), "alloc metrics"))) return bail(rc);
    if ((rc = E->hip(hipMemset(E->d_msrc.p, 0, sizeof(unsigned long long) * ns), "memset"))) return bail(rc);
    if ((rc = E->hip(hipMemset(E->d_mdst.p, 0, sizeof(unsigned long long) * nd), "memset"))) return bail(rc);
    if ((rc = E->hip(hipMemset(E->d_mhist.p, 0, sizeof(unsigned long long) * 2 * kMetricBins), "memset")))
      return bail(rc);
  }
  E->peers_dirty = E->rules_dirty = E->params_dirty = true;
  if ((rc = flush_config(E))) return bail(rc);
  *out = E;
  return 0;
}

void tgsim_destroy(void* e) {
  Eng* E = as_eng(e);
  if (!E) return;
  (void)hipSetDevice(E->dev);
  if (E->st) (void)hipStreamSynchronize(E->st);
  if (E->dst_st) (void)hipStreamSynchronize(E->dst_st);
  if (E->rt_st) (void)hipStreamSynchronize(E->rt_st);
  if (E->sy_st) (void)hipStreamSynchronize(E->sy_st);
  // the exchange layer after the engine's streams (deliveries read its buffers), before their destruction
  if (E->comm.free_fn) E->comm.free_fn(E->comm.state);
  E->d_sync.release(); E->d_gone.release();
  if (E->h_mirror) (void)hipHostFree(E->h_mirror);
  for (int t = 0; t < 2; ++t) {
    if (E->h_patch[t]) (void)hipHostFree(E->h_patch[t]);
    if (E->ev_patch[t]) (void)hipEventDestroy(E->ev_patch[t]);
    E->d_patch_t[t].release();
  }
  if (E->ev_pcopy) (void)hipEventDestroy(E->ev_pcopy);
  {
  }
  if (E->h_sig) (void)hipHostFree(E->h_sig);
  if (E->ev_sig) (void)hipEventDestroy(E->ev_sig);
  if (E->sy_st) (void)hipStreamDestroy(E->sy_st);
  DevBuf<int> dummy;
  (void)dummy;
  E->d_params.release(); E->d_state.release(); E->d_enabled.release(); E->d_ip.release();
  E->d_rules.release(); E->d_heap.release(); E->d_ring.release(); E->d_wheel.release(); E->d_wmeta.release();
  E->d_gen_seq.release(); E->d_off.release(); E->d_cnt.release(); E->d_blk.release(); E->d_tot.release();
  E->d_in.release(); E->d_verdict.release(); E->d_emit.release(); E->d_emit_n.release(); E->d_emit_alt.release(); E->d_emit_n_alt.release(); E->d_lcnt.release(); E->d_lcnt_alt.release(); E->d_dbkt.release(); E->d_dbkt_alt.release(); E->d_sdoff.release(); E->d_sdpos.release(); E->d_sdblk.release(); E->d_sdtot.release(); E->d_sdoff_alt.release(); E->d_sdpos_alt.release(); E->d_sdblk_alt.release(); E->d_sdtot_alt.release(); E->d_sdoff_alt2.release(); E->d_sdpos_alt2.release(); E->d_sdblk_alt2.release(); E->d_sdtot_alt2.release(); E->d_emit_alt2.release(); E->d_emit_n_alt2.release(); E->d_lcnt_alt2.release(); E->d_dbkt_alt2.release(); E->d_pidx.release(); E->d_pidx_alt.release(); E->d_pidx_alt2.release(); E->d_rcnt.release(); E->d_rpos.release(); E->d_rblk.release(); E->d_rtot.release();
  E->d_bucket.release(); E->d_scatter.release(); E->d_sorted.release(); E->d_dcnt.release();
  E->d_doff.release(); E->d_dpos.release(); E->d_dblk.release(); E->d_dtot.release();
  E->d_drain.release(); E->d_gfirst.release(); E->d_gfwd.release(); E->d_gpend.release(); E->d_gnbr.release(); E->d_gerr.release(); E->d_stats.release(); E->d_stamps.release(); E->d_order.release();
  E->d_msrc.release(); E->d_mdst.release(); E->d_mhist.release(); E->d_work.release(); E->d_rsend.release();
  for (auto* q : {&E->gen_q, &E->gen_free})
    for (auto& w : *q) {
      w.off.release();
      w.in.release();
    }
  for (auto* pend : {&E->ev_pending, &E->dv_pending})
    for (auto& pr : *pend) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
  for (auto& grp : E->fset)
    for (auto& ls : grp) { ls.emit.release(); ls.emit_n.release(); }
  for (auto& v : E->f_lcnt) v.release();
  for (auto& v : E->f_verdict) v.release();
  E->d_done.release(); E->d_ticket.release();
  for (hipEvent_t ev : E->ev_fgrp)
    if (ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : E->ev_pool) (void)hipEventDestroy(ev);
  if (E->h_err) (void)hipHostFree(E->h_err);
  if (E->h_xerr) (void)hipHostFree(E->h_xerr);
  if (E->h_work) (void)hipHostFree(E->h_work);
  if (E->h_gerr) (void)hipHostFree(E->h_gerr);
  if (E->h_pub) (void)hipHostFree(E->h_pub);
  if (E->ev_gpub) (void)hipEventDestroy(E->ev_gpub);
  if (E->ev_pub) (void)hipEventDestroy(E->ev_pub);
  if (E->h_edges) (void)hipHostFree(E->h_edges);
  for (hipEvent_t ev : E->ev_route)
    if (ev) (void)hipEventDestroy(ev);
  if (E->ev_dst) (void)hipEventDestroy(E->ev_dst);
  if (E->ev_rt) (void)hipEventDestroy(E->ev_rt);
  if (E->ev_recv) (void)hipEventDestroy(E->ev_recv);
  if (E->ev_sim) (void)hipEventDestroy(E->ev_sim);
  if (E->ev_local) (void)hipEventDestroy(E->ev_local);
  if (E->ev_local_alt) (void)hipEventDestroy(E->ev_local_alt);
  if (E->ev_local_alt2) (void)hipEventDestroy(E->ev_local_alt2);
  if (E->dst_st) (void)hipStreamDestroy(E->dst_st);
  if (E->rt_st) (void)hipStreamDestroy(E->rt_st);
  if (E->st) (void)hipStreamDestroy(E->st);
  delete E;
}

const char* tgsim_last_error(const void* e) {
  return e ? static_cast<const Eng*>(e)->err.c_str() : "null engine";
}

// ConfigureNetwork with netlink replaced by staged state (applied at the next step): the docker
// sidecar's order of operations and errors, or the k8s one with TGSIM_OPT_K8S.
// The patch staging array (one slot per source at most per step), sized at the first configure call.
int ensure_patch_staging(Eng* E) {
  if (E->patch_stage.size() < E->S) E->patch_stage.resize(E->S);
  return 0;
}

int configure_one(Eng* E, uint32_t peer, const tgsim_config* cfg, const Compiled* pre) {
  if (peer >= E->N) return E->fail(-EINVAL, "peer %u out of range", peer);
  const int rc = (E->o.flags & TGSIM_OPT_K8S) ? configure_k8s(E, peer, cfg, pre) : configure_docker(E, peer, cfg, pre);
  if (owns(E, peer)) write_patch(E, peer - E->o.shard_begin);
  return rc;
}

int tgsim_configure(void* e, uint32_t peer, const tgsim_config* cfg) {
  Eng* E = as_eng(e);
  if (!E || !cfg) return -EINVAL;
  const int rc = ensure_patch_staging(E);
  if (rc) return rc;
  return configure_one(E, peer, cfg, nullptr);
}

int64_t tgsim_configure_batch(void* e, const uint32_t* peers, const tgsim_config* cfgs, size_t n, int32_t* rcs) {
  if (!e || (n && (!peers || !cfgs))) return -EINVAL;
  Eng* E = as_eng(e);
  if (E) {
    const int rc = ensure_patch_staging(E);
    if (rc) return rc;
  }
  int64_t failed = 0;
  for (size_t i = 0; i < n; ++i) {
    // a C5 epoch reshapes 10,000 of 100,000 sources: their host state (three lines each) and peer
    // entries are fetched a few calls ahead (the loop was bound by those misses)
    if (E && i + 8 < n && peers[i + 8] < E->N) {
      const uint32_t q = peers[i + 8];
      if (owns(E, q)) {
        const char* hp = reinterpret_cast<const char*>(&E->src[q - E->o.shard_begin]);
        __builtin_prefetch(hp);
        __builtin_prefetch(hp + 64);
        __builtin_prefetch(hp + 128);
      }
      __builtin_prefetch(&E->enabled[q]);
      __builtin_prefetch(&E->ip[q]);
    }
    const int rc = !E ? -EINVAL : configure_one(E, peers[i], &cfgs[i], nullptr);
    if (rcs) rcs[i] = rc;
    failed += rc != 0;
  }
  return failed;
}

int tgsim_submit(void* e, const tgsim_pkt* pkts, size_t n) {
  Eng* E = as_eng(e);
  if (!E || (!pkts && n)) return -EINVAL;
  if (!E->gen_q.empty()) return E->fail(-EBUSY, "generated traffic already pending for the next step");
  for (size_t i = 0; i < n; ++i) {
    if (pkts[i].src < E->o.shard_begin || pkts[i].src >= E->o.shard_end)
      return E->fail(-EINVAL, "packet %zu: src %u not owned by this shard", i, pkts[i].src);
    if (pkts[i].dst != TGSIM_EXTERNAL && pkts[i].dst >= E->N)
      return E->fail(-EINVAL, "packet %zu: dst %u out of range", i, pkts[i].dst);
  }
  const uint64_t base = E->staged.size();
  for (size_t i = 0; i < n; ++i) E->staged.push_back({pkts[i], base + i});
  return 0;
}

int tgsim_gen_storm(void* e, double lambda, uint32_t n_ticks) {
  Eng* E = as_eng(e);
  if (!E || !(lambda >= 0.0) || lambda > 4.0 || n_ticks == 0 || n_ticks > 65536) return -EINVAL;
  if (!E->staged.empty()) return E->fail(-EBUSY, "host packets already pending for the next step");
  HIPCHK(hipSetDevice(E->dev));
  GenArgsHost g;
  double p = std::exp(-lambda), F = p;
  for (int k = 0; k < 16; ++k) {
    const double t = F * 4294967296.0;
    g.tab[k] = t >= 4294967295.0 ? 0xFFFFFFFFu : static_cast<uint32_t>(t);
    p = p * lambda / static_cast<double>(k + 1);
    F = F + p;
  }
  g.k0 = E->key0 ^ 0x9E3779B9u;
  g.k1 = E->key1 ^ 0x7F4A7C15u;
  g.n_src = E->S;
  g.shard_begin = E->o.shard_begin;
  g.n_peers = E->N;
  g.n_ticks = n_ticks;
  g.now_tick = E->now_tick + E->gen_q_ticks;  // windows queue up back to back
  Eng::GenWindow w;  // a free window's offsets may still be read by a delivery or a routing
  int trc = take_gen(E, &w);
  if (trc) return trc;
  HIPCHK(E->d_cnt.ensure(E->S));
  launch_gen(g, E->d_cnt.p, nullptr, nullptr, nullptr, 0, E->st);
  HIPCHK(hipGetLastError());
  uint64_t total = 0;
  int rc = scan_counts(E, E->d_cnt, w.off, E->d_blk, E->d_tot, E->S, &total);
  if (rc) return rc;
  HIPCHK(w.in.ensure(total ? total : 1));
  launch_gen(g, nullptr, w.off.p, E->d_gen_seq.p, w.in.p, 1, E->st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(E->st));
  w.n = total;
  w.ticks = n_ticks;
  E->gen_q_ticks += n_ticks;
  E->gen_q.push_back(std::move(w));
  return 0;
}

// Gossip flood workload, see include/tgsim.h.
int tgsim_gossip_init(void* e, const tgsim_gossip* g) {
  Eng* E = as_eng(e);
  if (!E || !g || g->n_floods == 0 || g->n_floods > 64 || g->degree == 0 || g->degree > 64 ||
      g->msg_len == 0 || g->msg_len > 65535 || E->N < 2)
    return -EINVAL;
  if (g->start_tick < E->now_tick + E->gen_q_ticks) return E->fail(-EINVAL, "gossip: start tick in the past");
  HIPCHK(hipSetDevice(E->dev));
  E->gossip = *g;
  E->gossip_late = false;
  HIPCHK(E->d_gfirst.ensure(static_cast<size_t>(E->S) * 64));
  HIPCHK(E->d_gfwd.ensure(E->S));
  HIPCHK(E->d_gpend.ensure(E->S));
  HIPCHK(E->d_gerr.ensure(1));
  E->d_gnbr.release();  // the table of another degree, if any
  HIPCHK(E->d_gnbr.ensure(static_cast<size_t>(E->S) * g->degree));
  launch_gossip_nbr(gossip_args(E, 0, 0), E->d_gnbr.p, E->st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemsetAsync(E->d_gfirst.p, 0xFF, sizeof(uint32_t) * 64 * E->S, E->st));
  HIPCHK(hipMemsetAsync(E->d_gfwd.p, 0, sizeof(uint64_t) * E->S, E->st));
  HIPCHK(hipMemsetAsync(E->d_gpend.p, 0, sizeof(uint64_t) * E->S, E->st));
  HIPCHK(hipMemsetAsync(E->d_gerr.p, 0, sizeof(uint32_t), E->st));
  std::unordered_map<uint32_t, uint64_t> origin_pend;  // origin -> its floods (pending forwards)
  for (uint32_t f = 0; f < g->n_floods; ++f) {
    uint32_t r[4];
    philox_host(f, 0, 0x4F524947u, 0, E->key0 ^ 0x3C6EF372u, E->key1 ^ 0xA54FF53Au, r);
    const uint32_t origin = r[0] % E->N;
    if (origin < E->o.shard_begin || origin >= E->o.shard_end) continue;
    const uint32_t t = static_cast<uint32_t>(g->start_tick + static_cast<uint64_t>(f) * g->start_gap_ticks);
    HIPCHK(hipMemcpyAsync(E->d_gfirst.p + static_cast<uint64_t>(origin - E->o.shard_begin) * 64 + f, &t,
                          sizeof t, hipMemcpyHostToDevice, E->st));
    HIPCHK(hipStreamSynchronize(E->st));  // `t` lives on this stack frame
    origin_pend[origin - E->o.shard_begin] |= 1ull << f;
  }
  for (const auto& op : origin_pend) {
    HIPCHK(hipMemcpyAsync(E->d_gpend.p + op.first, &op.second, sizeof(uint64_t), hipMemcpyHostToDevice, E->st));
    HIPCHK(hipStreamSynchronize(E->st));
  }
  HIPCHK(hipStreamSynchronize(E->st));
  // a flood's windows grow geometrically while it spreads: reserve the window buffers (generated
  // input of two windows, the step's input and verdicts) for four forwards per peer and
  // out-neighbour (the 1M-peer flood's peak windows offer ~30 packets per peer), so no window of the
  // flood reallocates (each hipFree + hipMalloc stalls the closed loop for 0.3-0.5 ms)
  const size_t reserve = static_cast<size_t>(E->S) * g->degree * 4;  // the flood's peak: ~30 per peer
  while (E->gen_free.size() < E->emit_sets + 1) E->gen_free.emplace_back();  // in rotation (take_gen)
  for (auto& w : E->gen_free) {
    HIPCHK(w.off.ensure(E->S + 1));
    HIPCHK(w.in.ensure(reserve));
  }
  HIPCHK(E->d_in.ensure(reserve));
  HIPCHK(E->d_verdict.ensure(reserve));
  // the emit regions of both parities, for the same reserve (a hipFree + hipMalloc of several GB inside the flood stalls the loop)
  const uint64_t emit_cap = emit_records(E, reserve, compact_layout(E, reserve, true));
  for (auto* b : {&E->d_emit, &E->d_emit_alt, &E->d_emit_alt2})
    if (b != &E->d_emit_alt2 || E->emit_sets == 3) HIPCHK(b->ensure(emit_cap));
  // and the delivery's scatter buffer and (discarded deliveries) its output, which a window sizes by
  // its records' bound: grown inside the flood, each growth was a hipFree + hipMalloc on the host
  // with the device idle (0.3-0.7 ms gaps in the routed step's trace, profiles/r05/routed_trace/)
  HIPCHK(E->d_scatter.ensure(emit_cap));
  if (E->o.flags & TGSIM_OPT_DISCARD_DELIVERIES) HIPCHK(E->d_sorted.ensure(emit_cap));
  E->gossip_on = true;
  return 0;
}

int tgsim_gen_gossip(void* e, uint32_t n_ticks) {
  Eng* E = as_eng(e);
  if (!E || !E->gossip_on || n_ticks == 0 || n_ticks > 65536) return -EINVAL;
  if (!E->staged.empty()) return E->fail(-EBUSY, "host packets already pending for the next step");
  if (E->gossip_late)
    return E->fail(-EINVAL, "gossip: a receipt preceded an earlier window (tgsim_gossip_init starts a new flood)");
  HIPCHK(hipSetDevice(E->dev));
  for (size_t i = 0; i < E->gen_q.size(); ++i) {  // a window still unsized is sized (and written) before
                                                  // this one runs
    int rc = resolve_gen(E, E->gen_q[i]);
    if (rc) {
      if (E->gossip_late) drop_gen(E, i);  // the late window and any after it; the earlier ones stay
      return rc;
    }
  }
  // receipts are folded on the delivery stream (the sort of the same delivery may still run)
  HIPCHK(hipStreamWaitEvent(E->st, E->ev_recv, 0));
  const uint64_t win0 = E->now_tick + E->gen_q_ticks;
  const GossipArgs g = gossip_args(E, win0, n_ticks);
  Eng::GenWindow w;  // a free window's offsets may still be read by a routing or a delivery
  int trc = take_gen(E, &w);
  if (trc) return trc;
  HIPCHK(E->d_cnt.ensure(E->S));
  launch_gossip(g, nullptr, 0, E->d_cnt.p, nullptr, nullptr, 1, E->st);
  HIPCHK(hipGetLastError());
  // scan, then the forwards at once, without waiting for the total: the buffer is reserved for the
  // flood's peak, and a window larger than it writes nothing here (the kernel compares the device's
  // total with the capacity) and is written again once its size is known (resolve_gen, at the step)
  HIPCHK(w.off.ensure(E->S + 1));
  HIPCHK(E->d_blk.ensure((E->S + 1023) / 1024 + 1));
  HIPCHK(E->d_tot.ensure(1));
  launch_scan(E->d_cnt.p, w.off.p, E->S, E->d_blk.p, E->d_tot.p, E->st, nullptr);
  HIPCHK(hipGetLastError());
  launch_publish(E->d_tot.p, E->d_gerr.p, E->dm_pub + 4, ++E->pub_seq, E->st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(E->ev_gpub, E->st));
  HIPCHK(w.in.ensure(1));
  launch_gossip(g, nullptr, 0, nullptr, w.off.p, w.in.p, 2, E->st, w.in.cap, E->d_tot.p);
  HIPCHK(hipGetLastError());
  w.pending = true;
  w.pub_seq = E->pub_seq;
  w.g = g;
  w.n = 0;
  w.ticks = n_ticks;
  E->gen_q_ticks += n_ticks;
  E->gen_q.push_back(std::move(w));
  return 0;
}

int64_t tgsim_gossip_reached(void* e, uint64_t* out, size_t cap) {
  Eng* E = as_eng(e);
  if (!E || !E->gossip_on || (!out && cap)) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  int rc = sync_stream(E);
  if (rc) return rc;
  std::vector<uint64_t> fwd(E->S);
  HIPCHK(hipMemcpy(fwd.data(), E->d_gfwd.p, sizeof(uint64_t) * E->S, hipMemcpyDeviceToHost));
  for (uint32_t f = 0; f < E->gossip.n_floods && f < cap; ++f) {
    uint64_t c = 0;
    for (uint32_t s = 0; s < E->S; ++s) c += fwd[s] >> f & 1u;
    out[f] = c;
  }
  return E->gossip.n_floods;
}

int64_t tgsim_sim_capacity(void* e) {
  Eng* E = as_eng(e);
  if (!E) return -EINVAL;
  if (!E->gen_q.empty()) {
    int rc = resolve_gen(E, E->gen_q.front());
    if (rc) {
      if (E->gossip_late) drop_gen(E);
      return rc;
    }
  }
  const uint64_t n = !E->gen_q.empty() ? E->gen_q.front().n : E->staged.size();
  // the records the next window can emit in the layout it will use (the choice is kept for it)
  return static_cast<int64_t>(emit_records(E, n, compact_layout(E, n, sparse_choice(E, n, false))));
}

int tgsim_step_sim_launch(void* e, uint32_t n_ticks, uint32_t n_ranks, const uint32_t* bounds, void* d_out,
                          size_t out_cap) {
  Eng* E = as_eng(e);
  if (!E || n_ticks == 0 || n_ranks == 0 || n_ranks > 8 || !bounds || (!d_out && out_cap)) return -EINVAL;
  if (bounds[0] != 0 || bounds[n_ranks] != E->N) return E->fail(-EINVAL, "rank bounds must cover [0, n_peers)");
  if (E->route_n == Eng::kRouteSlots) return E->fail(-EBUSY, "two launched steps are not finished yet");
  HIPCHK(hipSetDevice(E->dev));
  int rc = run_sim(E, n_ticks);
  if (rc) return rc;
  return route_launch(E, n_ranks, bounds, static_cast<tgsim_delivery*>(d_out), out_cap);
}

int tgsim_step_sim_finish(void* e, uint64_t* counts) {
  Eng* E = as_eng(e);
  if (!E || !counts) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  return route_finish(E, counts);
}

int tgsim_step_sim_counts(void* e, uint64_t* counts) {
  Eng* E = as_eng(e);
  if (!E || !counts) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  return route_finish(E, counts, false);
}

int tgsim_step_sim_launch_slotted(void* e, uint32_t n_ticks, uint32_t n_ranks, const uint32_t* bounds, void* d_out,
                                  uint64_t slot_cap, void* routed_event) {
  Eng* E = as_eng(e);
  if (!E || n_ticks == 0 || n_ranks == 0 || n_ranks > 8 || !bounds || !d_out || slot_cap == 0) return -EINVAL;
  if (bounds[0] != 0 || bounds[n_ranks] != E->N) return E->fail(-EINVAL, "rank bounds must cover [0, n_peers)");
  if (E->route_n == Eng::kRouteSlots) return E->fail(-EBUSY, "two launched steps are not released yet");
  HIPCHK(hipSetDevice(E->dev));
  int rc = run_sim(E, n_ticks);
  if (rc) return rc;
  return route_launch(E, n_ranks, bounds, static_cast<tgsim_delivery*>(d_out), n_ranks * (slot_cap + 1), slot_cap,
                      static_cast<hipEvent_t>(routed_event));
}

int tgsim_step_sim_launch_slotted_n(void* e, uint32_t n_ticks, uint32_t n_win, uint32_t n_ranks,
                                    const uint32_t* bounds, void* d_out, uint64_t slot_cap, void* routed_event) {
  Eng* E = as_eng(e);
  if (!E || n_ticks == 0 || n_win == 0 || n_win > kFuseMax || n_ranks == 0 || n_ranks > 8 || !bounds || !d_out ||
      slot_cap == 0)
    return -EINVAL;
  if (n_win == 1)
    return tgsim_step_sim_launch_slotted(e, n_ticks, n_ranks, bounds, d_out, slot_cap, routed_event);
  if (bounds[0] != 0 || bounds[n_ranks] != E->N) return E->fail(-EINVAL, "rank bounds must cover [0, n_peers)");
  if (E->route_n == Eng::kRouteSlots) return E->fail(-EBUSY, "two launched steps are not released yet");
  HIPCHK(hipSetDevice(E->dev));
  if (!fusable(E, n_ticks, n_win, true))
    return E->fail(-EINVAL, "step_sim_launch_slotted_n: the next %u windows are not generated dense windows of %u ticks",
                   n_win, n_ticks);
  const GroupRoute gr{n_ranks, bounds, static_cast<tgsim_delivery*>(d_out), slot_cap, static_cast<hipEvent_t>(routed_event)};
  return step_fused(E, n_ticks, n_win, &gr);
}

int tgsim_deliver_slotted_n_async(void* e, const void* d_in, uint32_t n_ranks, uint32_t n_win, uint64_t slot_cap,
                                  void* wait_event) {
  Eng* E = as_eng(e);
  if (!E || !d_in || n_ranks == 0 || n_ranks > 8 || n_win == 0 || n_win > kFuseMax || slot_cap == 0) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  return deliver(E, static_cast<const tgsim_delivery*>(d_in), static_cast<uint64_t>(n_ranks) * n_win * (slot_cap + 1),
                 static_cast<hipEvent_t>(wait_event), false, slot_cap, n_win);
}

int tgsim_step_sim_release(void* e) {
  Eng* E = as_eng(e);
  if (!E) return -EINVAL;
  if (!E->route_n) return E->fail(-EINVAL, "no routed step pending");
  HIPCHK(hipSetDevice(E->dev));
  E->route_head = (E->route_head + 1) % Eng::kRouteSlots;
  E->route_n--;
  int rc = harvest_timing(E, false);
  if (rc) return rc;
  return check_sim_error(E);
}

int tgsim_deliver_slotted_async(void* e, const void* d_in, uint32_t n_ranks, uint64_t slot_cap, void* wait_event) {
  Eng* E = as_eng(e);
  if (!E || !d_in || n_ranks == 0 || n_ranks > 8 || slot_cap == 0) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  return deliver(E, static_cast<const tgsim_delivery*>(d_in), n_ranks * (slot_cap + 1),
                 static_cast<hipEvent_t>(wait_event), false, slot_cap);
}

int tgsim_delivery_event(void* e, void* event) {
  Eng* E = as_eng(e);
  if (!E || !event) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  HIPCHK(hipEventRecord(static_cast<hipEvent_t>(event), E->dst_st));
  return 0;
}

int tgsim_step_sim(void* e, uint32_t n_ticks, uint32_t n_ranks, const uint32_t* bounds, void* d_out,
                   size_t out_cap, uint64_t* counts) {
  if (!counts) return -EINVAL;
  if (as_eng(e) && as_eng(e)->route_n) return as_eng(e)->fail(-EBUSY, "launched steps are not finished yet");
  int rc = tgsim_step_sim_launch(e, n_ticks, n_ranks, bounds, d_out, out_cap);
  if (rc) return rc;
  return tgsim_step_sim_finish(e, counts);
}

int tgsim_deliver(void* e, const void* d_in, size_t n) {
  Eng* E = as_eng(e);
  if (!E || (!d_in && n)) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  int rc = deliver(E, static_cast<const tgsim_delivery*>(d_in), n, nullptr,
                   !(E->o.flags & TGSIM_OPT_DISCARD_DELIVERIES));
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(E->dst_st));
  return 0;
}

int tgsim_deliver_async(void* e, const void* d_in, size_t n, void* wait_event) {
  Eng* E = as_eng(e);
  if (!E || (!d_in && n)) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  return deliver(E, static_cast<const tgsim_delivery*>(d_in), n, static_cast<hipEvent_t>(wait_event), false);
}

int tgsim_wait_event(void* e, void* event) {
  Eng* E = as_eng(e);
  if (!E || !event) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  HIPCHK(hipStreamWaitEvent(E->st, static_cast<hipEvent_t>(event), 0));
  HIPCHK(hipStreamWaitEvent(E->rt_st, static_cast<hipEvent_t>(event), 0));  // routing writes the caller's buffer
  return 0;
}

int tgsim_sync(void* e) {
  Eng* E = as_eng(e);
  if (!E) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  int rc = sync_stream(E);
  if (rc) return rc;
  return check_sim_error(E);
}

int tgsim_step(void* e, uint32_t n_ticks) {
  Eng* E = as_eng(e);
  if (!E || n_ticks == 0) return -EINVAL;
  if (E->route_n) return E->fail(-EBUSY, "launched steps are not finished yet");
  HIPCHK(hipSetDevice(E->dev));
  if (E->S == E->N) {  // whole population on this engine: asynchronous local delivery
    int rc = run_sim(E, n_ticks, true);
    if (rc) return rc;
    return deliver_local(E);
  }
  int rc = run_sim(E, n_ticks);
  if (rc) return rc;
  // the window's emit layout (run_sim's choice, rotated by the routing below) bounds its records
  const uint64_t cap = emit_records(E, E->n_in, E->el.r != kHeapCap);
  HIPCHK(E->d_bucket.ensure(cap));
  const uint32_t bounds[2] = {0, E->N};
  uint64_t count = 0;
  rc = route(E, 1, bounds, E->d_bucket.p, E->d_bucket.cap, &count);
  if (rc) return rc;
  rc = deliver(E, E->d_bucket.p, count, nullptr, true);
  if (rc) return rc;
  return finish_sim_timing(E);
}

int tgsim_step_n(void* e, uint32_t n_ticks, uint32_t n_steps) {
  Eng* E = as_eng(e);
  if (!E || n_ticks == 0) return -EINVAL;
  if (E->route_n) return E->fail(-EBUSY, "launched steps are not finished yet");
  HIPCHK(hipSetDevice(E->dev));
  while (n_steps) {
    const uint32_t g = std::min(n_steps, static_cast<uint32_t>(E->fuse_max));
    int rc;
    if (fusable(E, n_ticks, g)) {
      rc = step_fused(E, n_ticks, g);
      n_steps -= g;
    } else {
      rc = tgsim_step(e, n_ticks);
      n_steps -= 1;
    }
    if (rc) return rc;
  }
  return 0;
}

int64_t tgsim_link_generation(void* e, uint32_t peer) {
  Eng* E = as_eng(e);
  if (!E || peer >= E->N) return -EINVAL;
  return E->link_gen[peer];
}

int64_t tgsim_drain(void* e, tgsim_delivery* out, size_t cap) {
  Eng* E = as_eng(e);
  if (!E || (!out && cap)) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  int rc = sync_stream(E);
  if (rc) return rc;
  // a window whose simulation failed (sticky error bits) hands out nothing
  if ((rc = check_sim_error(E))) return rc;
  const uint64_t n = std::min<uint64_t>(cap, E->drain_n);
  if (n) {
    HIPCHK(hipMemcpy(out, E->d_drain.p + E->drain_head, sizeof(tgsim_delivery) * n, hipMemcpyDeviceToHost));
  }
  E->drain_head += n;
  E->drain_n -= n;
  if (!E->drain_n) E->drain_head = 0;
  return static_cast<int64_t>(n);
}

int64_t tgsim_pending_deliveries(void* e) {
  Eng* E = as_eng(e);
  return E ? static_cast<int64_t>(E->drain_n) : -EINVAL;
}

int64_t tgsim_verdicts(void* e, uint8_t* out, size_t cap) {
  Eng* E = as_eng(e);
  if (!E || (!out && cap)) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  int rc = sync_stream(E);
  if (rc) return rc;
  // a window whose simulation failed (sticky error bits) hands out nothing
  if ((rc = check_sim_error(E))) return rc;
  if (cap >= E->n_verdict && E->n_verdict) {
    std::vector<uint8_t> tmp(E->n_verdict);
    HIPCHK(hipMemcpy(tmp.data(), E->d_verdict.p, E->n_verdict, hipMemcpyDeviceToHost));
    if (E->last_perm.empty()) {
      memcpy(out, tmp.data(), E->n_verdict);
    } else {
      for (uint64_t i = 0; i < E->n_verdict; ++i) out[E->last_perm[i]] = tmp[i];
    }
  }
  return static_cast<int64_t>(E->n_verdict);
}

int tgsim_stats(void* e, tgsim_stats_t* out) {
  Eng* E = as_eng(e);
  if (!E || !out) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  int rc = sync_stream(E);
  if (rc) return rc;
  std::vector<unsigned long long> all(static_cast<size_t>(kStSlots) * kStatCopies);
  HIPCHK(hipMemcpy(all.data(), E->d_stats.p, sizeof(unsigned long long) * all.size(), hipMemcpyDeviceToHost));
  unsigned long long s[kStSlots] = {};
  for (uint32_t c = 0; c < kStatCopies; ++c)
    for (uint32_t k = 0; k < kStSlots; ++k) s[k] += all[static_cast<size_t>(c) * kStSlots + k];
  memset(out, 0, sizeof *out);
  out->offered = s[kStOffered];
  out->scheduled = s[kStScheduled];
  out->cloned = s[kStCloned];
  out->corrupted = s[kStCorrupted];
  for (int i = 0; i < 8; ++i) out->by_verdict[i] = s[kStVerdict0 + i];
  out->bytes_scheduled = s[kStBytes];
  out->now_tick = E->now_tick;
  out->queue_state_bytes = s[kStQueue];
  out->flushed = s[kStFlushed];
  out->lost_in_flight = s[kStLost];
  return 0;
}

// The sync stream (high priority), created on first use.

// K7: SignalEntry on the device counter table (sync stream; see include/tgsim.h).
int tgsim_signal_async(void* e, uint32_t state, uint32_t n) {
  Eng* E = as_eng(e);
  if (!E || state >= kStates) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  HIPCHK(sync_stream_ready(E));
  launch_signal(E->d_sync.p, E->dm_mirror, state, n, E->dm_sig, E->dm_sig + 1, ++E->sig_seq, E->sy_st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(E->ev_sig, E->sy_st));
  return 0;
}

// Waits until every signal issued so far has landed in the pinned words (no device call).
static int signals_landed(Eng* E) {
  if (!E->sig_seq) return 0;
  return wait_published(E, &E->h_sig[1], E->sig_seq, E->ev_sig, "sync signal");
}

int64_t tgsim_signal(void* e, uint32_t state, uint32_t n) {
  Eng* E = as_eng(e);
  int rc = tgsim_signal_async(e, state, n);
  if (rc) return rc;
  rc = signals_landed(E);
  if (rc) return rc;
  return static_cast<int64_t>(__atomic_load_n(&E->h_sig[0], __ATOMIC_ACQUIRE));
}

int tgsim_sync_counters(void* e, void** d_table, uint32_t* n_states, void* event) {
  Eng* E = as_eng(e);
  if (!E || !d_table || !n_states) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  *d_table = E->d_sync.p;
  *n_states = kStates;
  HIPCHK(sync_stream_ready(E));
  if (event) HIPCHK(hipEventRecord(static_cast<hipEvent_t>(event), E->sy_st));
  return 0;
}

int64_t tgsim_metrics(void* e, uint32_t kind, uint64_t* out, size_t cap) {
  Eng* E = as_eng(e);
  if (!E || (!out && cap) || kind > TGSIM_METRICS_HIST) return -EINVAL;
  if (!E->metrics_on) return E->fail(-ENODATA, "engine created without TGSIM_OPT_METRICS");
  HIPCHK(hipSetDevice(E->dev));
  int rc = sync_stream(E);
  if (rc) return rc;
  const DevBuf<unsigned long long>& b = kind == TGSIM_METRICS_SRC ? E->d_msrc : kind == TGSIM_METRICS_DST ? E->d_mdst : E->d_mhist;
  const size_t n = kind == TGSIM_METRICS_SRC   ? static_cast<size_t>(E->S) * kMetricSrcWords
                   : kind == TGSIM_METRICS_DST ? static_cast<size_t>(E->S) * kMetricDstWords
                                               : 2 * kMetricBins;
  if (cap) HIPCHK(hipMemcpy(out, b.p, sizeof(uint64_t) * (cap < n ? cap : n), hipMemcpyDeviceToHost));
  return static_cast<int64_t>(n);
}

int tgsim_barrier_poll(void* e, uint32_t state, uint64_t target) {
  Eng* E = as_eng(e);
  if (!E || state >= kStates) return -EINVAL;
  const int rc = signals_landed(E);
  if (rc) return rc;
  return __atomic_load_n(&E->h_mirror[state], __ATOMIC_ACQUIRE) >= target ? 1 : 0;
}

double tgsim_sim_kernel_ms(void* e, uint64_t* n, int reset) {
  Eng* E = as_eng(e);
  if (!E) return -1;
  if (hipSetDevice(E->dev) != hipSuccess || sync_stream(E)) return -1;
  const double avg = E->sim_launches ? E->sim_ms / static_cast<double>(E->sim_launches) : 0.0;
  if (n) *n = E->sim_launches;
  if (reset) {
    E->sim_ms = 0;
    E->sim_launches = 0;
  }
  return avg;
}

double tgsim_delivery_kernel_ms(void* e, uint64_t* n, int reset) {
  Eng* E = as_eng(e);
  if (!E) return -1;
  if (hipSetDevice(E->dev) != hipSuccess || sync_stream(E)) return -1;
  const double avg = E->dv_windows ? E->dv_ms / static_cast<double>(E->dv_windows) : 0.0;
  if (n) *n = E->dv_windows;
  if (reset) {
    E->dv_ms = 0;
    E->dv_windows = 0;
  }
  return avg;
}

int64_t tgsim_debug_stamps(void* e, uint64_t* out, size_t cap) {
  Eng* E = as_eng(e);
  if (!E) return -EINVAL;
  const uint64_t n = E->stamps_on ? E->n_stamp_wg * kStampSlots : 0;
  if (out && cap >= n && n) {
    HIPCHK(hipSetDevice(E->dev));
    int rc = sync_stream(E);
    if (rc) return rc;
    HIPCHK(hipMemcpy(out, E->d_stamps.p, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
  }
  return static_cast<int64_t>(n);
}

int64_t tgsim_debug_carry_bytes(void* e) {
  Eng* E = as_eng(e);
  if (!E) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  int rc = sync_stream(E);
  if (rc) return rc;
  std::vector<unsigned long long> all(static_cast<size_t>(kStSlots) * kStatCopies);
  HIPCHK(hipMemcpy(all.data(), E->d_stats.p, sizeof(unsigned long long) * all.size(), hipMemcpyDeviceToHost));
  unsigned long long q = 0, skipped = 0;  // the per-window model minus what stayed in LDS
  for (uint32_t c = 0; c < kStatCopies; ++c) {
    q += all[static_cast<size_t>(c) * kStSlots + kStQueue];
    skipped += all[static_cast<size_t>(c) * kStSlots + kStCarrySkip];
  }
  return static_cast<int64_t>(q - skipped);
}

int64_t tgsim_debug_bucket_records(void* e) {
  Eng* E = as_eng(e);
  if (!E) return -EINVAL;
  HIPCHK(hipSetDevice(E->dev));
  int rc = sync_stream(E);
  if (rc) return rc;
  std::vector<unsigned long long> all(static_cast<size_t>(kStSlots) * kStatCopies);
  HIPCHK(hipMemcpy(all.data(), E->d_stats.p, sizeof(unsigned long long) * all.size(), hipMemcpyDeviceToHost));
  unsigned long long n = 0;
  for (uint32_t c = 0; c < kStatCopies; ++c) n += all[static_cast<size_t>(c) * kStSlots + kStBktRecs];
  return static_cast<int64_t>(n);
}

int64_t tgsim_debug_exec_faults(void) { return exec_faults(); }

int64_t tgsim_debug_sparse_windows(void* e) {
  Eng* E = as_eng(e);
  return E ? static_cast<int64_t>(E->sparse_windows) : -EINVAL;
}

int64_t tgsim_debug_fused_windows(void* e) {
  Eng* E = as_eng(e);
  return E ? static_cast<int64_t>(E->fused_windows) : -EINVAL;
}

void* tgsim_stream(void* e) {
  Eng* E = as_eng(e);
  return E ? static_cast<void*>(E->st) : nullptr;
}

// Host-only building blocks (no device needed): used by the CPU test-suite to check the
// configuration compiler against the oracle.
int tgsim_host_compile_shape(const tgsim_shape* s, uint64_t out[13]) {
  if (!s || !out) return -EINVAL;
  const Compiled c = compile_shape(*s);
  out[0] = c.p.lat_ns; out[1] = static_cast<uint64_t>(static_cast<int64_t>(c.p.sigma));
  out[2] = static_cast<uint32_t>((s->bandwidth_bps ? s->bandwidth_bps : UINT64_MAX) / 8);
  out[3] = c.p.mult; out[4] = c.p.shift_ext & 0xFF; out[5] = c.p.burst_ns;
  out[6] = c.p.thr_loss; out[7] = c.p.thr_dup; out[8] = c.thr_cor_new; out[9] = c.p.thr_reo;
  out[10] = c.rho_dup_new; out[11] = c.rho_cor_new; out[12] = c.rho_reo_new;
  return 0;
}

// rules: (prefix, len, action) triples already applied in order; writes up to cap intervals
// (lo, hi, act) and returns the count.
int64_t tgsim_host_compile_rules(const tgsim_rule* rules, size_t n, uint32_t* out, size_t cap) {
  std::map<uint64_t, uint8_t> m;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t key = (static_cast<uint64_t>(rules[i].prefix) << 8) | rules[i].len;
    if (rules[i].action == TGSIM_ACCEPT) m.erase(key);
    else m[key] = rules[i].action;
  }
  const std::vector<Interval> iv = compile_rules(m);
  for (size_t i = 0; i < iv.size() && i < cap; ++i) {
    out[3 * i] = iv[i].lo;
    out[3 * i + 1] = iv[i].hi;
    out[3 * i + 2] = iv[i].act;
  }
  return static_cast<int64_t>(iv.size());
}

}  // extern "C"
