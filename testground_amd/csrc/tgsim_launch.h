// tgsim_launch.h — host-callable launchers of the gfx950 kernels (tgsim_kernels.hip).
#pragma once
#include "tgsim_internal.h"

namespace tgsim {

struct GenArgsHost {
  uint32_t tab[16];
  uint32_t k0, k1, n_src, shard_begin, n_peers, n_ticks;
  uint64_t now_tick;
};

struct RouteArgsHost {
  EmitRead emit;
  const uint32_t* emit_n;
  const uint64_t* off;
  uint32_t n_src;
  uint32_t n_ranks;
  uint32_t bounds[9];
  uint64_t* cnt;        // [n_ranks][n_src]
  const uint64_t* pos;  // exclusive scan of cnt
  tgsim_delivery* out;
  uint64_t out_cap;
  uint64_t slot_cap;  // 0: flat; else per-rank chunks of a count header + slot_cap records
  uint64_t chunk_stride;      // slotted: records from one rank's chunk to the next (0: slot_cap + 1)
  uint32_t waves_per_block;   // 0 or 4: 256-thread blocks; 1: single-wave workgroups
};

void launch_sim(const SimArgs& a, uint32_t n_wg, hipStream_t st);
// f.n_win consecutive windows of every source in one persistent launch of n_wg workgroups
void launch_sim_fused(const SimArgs& a, const FusedArgs& f, uint32_t n_wg, hipStream_t st);
// workgroups of k_sim_fused resident on the device at once (its grid)
uint32_t sim_fused_resident();
// sparse step: k_sim_sparse over every source, then k_sim_list over the ones it deferred
// work_host: pinned words that receive the deferral counts (the counters are zeroed behind them)
void launch_sim_sparse(const SimArgs& a, hipStream_t st, uint32_t* work_host, uint32_t list_hint);
// no-op above kOrderMax (32768) sources
void launch_order(const uint32_t* weight, uint32_t n, uint32_t* order, hipStream_t st);
void launch_apply_cfg(const CfgPatch* p, uint32_t n, SrcParams* params, SrcState* state,
                      unsigned long long* stats, hipStream_t st);
// marks queued items towards gone[dst] != 0 dead (kDeadDst)
void launch_purge(uint4* heap, uint4* wheel, const WheelMeta* wmeta, const SrcState* state, uint32_t n_src,
                  const uint8_t* gone, hipStream_t st);
void launch_unrotate(uint4* heap, SrcState* state, uint32_t n_src, hipStream_t st);
// *v0 (and *v1) into pinned slot[0], slot[1], then seq into slot[2] (system-scope release)
void launch_publish(const uint64_t* v0, const uint32_t* v1, uint64_t* slot, uint64_t seq, hipStream_t st);
// K7: table[state] += n; new value -> mirror[state] and *result (pinned), then *marker = seq
void launch_signal(unsigned long long* table, uint64_t* mirror, uint32_t state, uint32_t n, uint64_t* result,
                   uint64_t* marker, uint64_t seq, hipStream_t st);
void launch_gen(const GenArgsHost& h, uint64_t* counts, const uint64_t* off, uint32_t* gen_seq,
                InRec* out, int phase, hipStream_t st);
// phase 0: fold delivered records into receipts; 1: per-source counts; 2: write the window.
void launch_gossip(const GossipArgs& g, const tgsim_delivery* recs, uint64_t n, uint64_t* counts,
                   const uint64_t* off, InRec* out, int phase, hipStream_t st, uint64_t out_cap = 0,
                   const uint64_t* total = nullptr);
// K8 metrics folds (opt-in): per source after k_sim, per destination after the delivery sort.
void launch_metrics_src(const MetricsArgs& m, hipStream_t st);
void launch_metrics_dst(const tgsim_delivery* recs, const uint64_t* off, uint32_t n_dst, unsigned long long* dst,
                        unsigned long long* hist, hipStream_t st);
// Receipts of n_dev[0] records (count read on the device).
void launch_gossip_nbr(const GossipArgs& g, uint32_t* nbr, hipStream_t st);
void launch_gossip_recv_dev(const GossipArgs& g, const tgsim_delivery* recs, const uint64_t* n_dev, hipStream_t st);
void launch_gossip_recv_in(const GossipArgs& g, const tgsim_delivery* recs, uint64_t n, uint64_t slot, bool skip_own,
                           hipStream_t st);
// Exclusive scan of in[0..n) into out[0..n] (out[n] = total, also stored at *total when non-null);
// pos (optional) receives a copy of out[0..n), the scatter cursors.
// clear: the input counts, zeroed as they are read (the histogram free for its next window), or null
void launch_scan(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* block_sums, uint64_t* total,
                 hipStream_t st, uint64_t* pos = nullptr, uint64_t* clear = nullptr);
void launch_route(const RouteArgsHost& h, int phase, hipStream_t st);
// edges[0..n_ranks] into slot[0..n_ranks] (pinned host memory), then seq into slot[15].
// slotted output (slot_cap != 0): also each rank chunk's count header in out, and *overflow = 1
// when a rank's count exceeds slot_cap.
void launch_route_edges(const uint64_t* pos, uint32_t n_src, uint32_t n_ranks, uint64_t* slot, uint64_t seq,
                        hipStream_t st, tgsim_delivery* out = nullptr, uint64_t slot_cap = 0,
                        uint32_t* overflow = nullptr, uint64_t chunk_stride = 0, uint64_t* dev_counts = nullptr);
// n (<= 64) device words to pinned host memory, then `seq` into host[n] (the word a host spins on).
void launch_publish_words(const uint64_t* src, uint32_t n, uint64_t* host, uint64_t seq, hipStream_t st);
// slot != 0: slotted input of n = chunks * (slot + 1) records (see launch_route_edges); with
// n_win > 1 chunk c holds window c % n_win, counted into cnt[(c % n_win) * n_dst + d] (a fused
// group: rank-major chunks, window-minor), in single-wave workgroups
// Slotted input (n_chunks chunks of a count header + up to `slot` records): histogram (out null) or
// scatter through pos (out given), grid-stride over the counts the headers announce.
void launch_dst_slot(const tgsim_delivery* in, uint64_t n_chunks, uint64_t slot, uint64_t slot_hint, uint32_t dst_begin,
                     uint32_t n_dst, uint64_t* cnt_or_pos, tgsim_delivery* out, hipStream_t st, uint32_t n_win);
void launch_dst_hist(const tgsim_delivery* in, uint64_t n, uint32_t dst_begin, uint32_t n_dst, uint64_t* cnt,
                     hipStream_t st, uint64_t slot = 0, uint32_t n_win = 1);
void launch_dst_scatter(const tgsim_delivery* in, uint64_t n, uint32_t dst_begin, uint32_t n_dst, uint64_t* pos,
                        tgsim_delivery* out, hipStream_t st, uint64_t slot = 0, uint32_t n_win = 1);
void launch_deliver_guard(const uint64_t* total, uint64_t cap, uint32_t* emit_n, uint32_t n_src, uint64_t* cnt,
                          uint64_t* off, uint32_t n_dst, uint64_t* err_host, hipStream_t st);
// pos: the destinations' cursors (= doff, the scanned segment starts, before the scatter); records that
// carry their destination slot (emit.slot) go to doff[d] + slot with no cursor atomic
// The per-destination order of a bucketed window (SimArgs::dst_bkt, 2^bkt_log records per bucket):
// the buckets and, for the destinations with more records, the scatter buffer (sc) behind them.
// total/cap/err_host: a bounded delivery's exact total against its buffers (null total: exact buffers).
void launch_dst_sort_bkt(const tgsim_delivery* bkt, uint32_t bkt_log, tgsim_delivery* sc, const uint64_t* doff,
                         uint32_t n_dst, tgsim_delivery* out, hipStream_t st, const uint64_t* total, uint64_t cap,
                         uint64_t* err_host);
void launch_local_scatter(const EmitRead& emit, const uint32_t* emit_n, const uint64_t* off, uint32_t n_src,
                          uint32_t dst_begin, const uint64_t* doff, uint64_t* pos, tgsim_delivery* out,
                          hipStream_t st, uint64_t n_hint, bool few_dst = false, bool single_wave = false);
// Orders each destination's records (segment d: off[d] .. off[d + 1]; dst_begin: the first
// destination's id) and resets cnt[] to zero for the next histogram, unless cnt is null (the scan
// cleared it: then sparse windows take the flattened sort).  (in, the scatter buffer, is
// overwritten for segments longer than 64.)  n_hint: about how many records.
void launch_dst_sort(tgsim_delivery* in, const uint64_t* off, uint64_t* cnt, uint32_t n_dst,
                     tgsim_delivery* out, hipStream_t st, uint64_t n_hint, uint32_t dst_begin = 0,
                     bool single_wave = false);
// The fused group's K5 (single-wave workgroups, see k_scan_w1): scan of n counts (clear: zeroed as
// read), scatter of the n_win windows' emit regions, one wavefront per (window, destination) segment.
// single_wave (above): the same single-wave form of a window's scatter and sort beside a running k_sim.
void launch_scan_w(uint64_t* in, uint64_t* out, uint64_t n, uint64_t* block_sums, uint64_t* total,
                   hipStream_t st, uint64_t* pos, bool clear = false);
void launch_local_scatter_group(const GroupDeliver& g, uint32_t n_win, hipStream_t st);
// TGSIM_CHECK builds: cross-lane helper calls whose source lanes were inactive (-ENOSYS otherwise)
int64_t exec_faults();
void launch_dst_sort_w1(tgsim_delivery* in, const uint64_t* off, uint64_t* cnt, uint32_t n_dst,
                        tgsim_delivery* out, hipStream_t st);

}  // namespace tgsim
