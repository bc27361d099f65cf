// tgsim_internal.h — device data layout of the engine (shared by host code and HIP kernels).
//
// HBM layout.  All per-source arrays are indexed by the shard-local source index
// s = src - shard_begin; per-peer tables are global (replicated on every shard).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tgsim.h"

namespace tgsim {

constexpr uint32_t kHeapCap = 1024;   // >= queue_limit (netem limit, max 1024)
constexpr uint32_t kWave = 64;        // lanes per wavefront
#ifndef TGSIM_SPW
#define TGSIM_SPW 1
#endif
constexpr uint32_t kSpw = TGSIM_SPW;
 // sources per simulate wavefront (LDS-resident queues)
constexpr uint32_t kAhead = kWave / kSpw;  // records per source staged per batch
constexpr uint64_t kEMask = (1ull << 46) - 1;  // eligibility time field of a queued item
constexpr uint32_t kStates = TGSIM_SYNC_STATES;  // sync states (K7 device counters)
// dst of a queued item whose destination disconnected or was re-addressed after it was queued
// (k_purge): HTB still serves it (it leaves the sender), nothing is delivered.  Never a real queued
// dst: TGSIM_EXTERNAL packets are filtered before the netem queue.
constexpr uint32_t kDeadDst = 0xFFFFFFFFu;

// Compiled netem + HTB parameters of one source (64 B, read once per step).
struct alignas(16) SrcParams {
  uint64_t lat_ns;     // netem latency (PSCHED ticks << 6)
  uint64_t burst_ns;   // HTB buffer (ticks << 6)
  int32_t sigma;       // tabledist sigma (s32)
  uint32_t mult;       // psched_ratecfg mult
  uint32_t shift_ext;  // bits 0..7 shift, bit 8 external traffic allowed
  uint32_t thr_loss, thr_dup, thr_cor, thr_reo;
  uint32_t rho_dup, rho_cor, rho_reo;
  uint32_t rule_off;   // first interval of this source's compiled FIB rules
  uint32_t rule_n;     // number of intervals
};
static_assert(sizeof(SrcParams) == 64, "SrcParams must stay 64 B");

// Mutable per-source state carried across steps (32 B).
struct alignas(16) SrcState {
  uint64_t tat;        // HTB theoretical arrival time (tokens >= 0 once now >= tat)
  uint32_t heap_n;     // queued, not yet eligible items (near + pool)
  uint32_t near_n;     // the first near_n of them: the sorted near region (the rest: the pool)
  uint32_t ring_n;
  uint32_t last_dup, last_cor, last_reo;  // get_crandom() correlation state
};
static_assert(sizeof(SrcState) == 32, "SrcState must stay 32 B");
// near_n packs the near region's length (bits 0..15) and the slot of the queue's first item in the
// source's kHeapCap-slot HBM array (bits 16..25; the items wrap around).  The slot is 0 in the
// compacted layout every writer but k_sim_sparse's FIFO path leaves; that path serves a prefix and
// appends behind the tail in place instead of moving the queue down (k_unrotate compacts it again
// before a fused launch, whose bounded loads assume slot 0).
__host__ __device__ inline uint32_t q_near(const SrcState& s) { return s.near_n & 0xFFFFu; }
__host__ __device__ inline uint32_t q_head(const SrcState& s) { return (s.near_n >> 16) & (kHeapCap - 1); }
// heap_n packs the items held in the source's heap array (bits 0..15) and the far items parked in
// its timing wheel (bits 16..31, DESIGN.md §4 "Timing wheel"); both count towards the netem limit.
__host__ __device__ inline uint32_t q_len(const SrcState& s) { return s.heap_n & 0xFFFFu; }
__host__ __device__ inline uint32_t q_parked(const SrcState& s) { return s.heap_n >> 16; }
__host__ __device__ inline uint32_t q_pack(uint32_t len, uint32_t parked) { return len | parked << 16; }
// ring_n packs the departure ring's length (bits 0..15) and the slot of its head in the source's
// kHeapCap-entry HBM ring (bits 16..25): the ring is circular in HBM, so a window reads only the head
// entries it may release and writes only the entries it appends (DESIGN.md §4 "Departure ring").
__host__ __device__ inline uint32_t r_len(const SrcState& s) { return s.ring_n & 0xFFFFu; }
__host__ __device__ inline uint32_t r_head(const SrcState& s) { return (s.ring_n >> 16) & (kHeapCap - 1); }
__host__ __device__ inline uint32_t r_pack(uint32_t len, uint32_t head) { return len | (head & (kHeapCap - 1)) << 16; }

// Timing wheel: a source's far netem items (eligible at or after the window's
// horizon) parked in HBM by eligibility time, so that a window reads only the buckets coming due
// and writes only the items it parks, instead of carrying the whole queue through LDS.  Bucket j of
// source s covers eligibility times [id << g, (id + 1) << g) for the one id = base + ((j - base) mod
// kWheelB) in [base, base + kWheelB); it holds up to kWheelCB items, unordered.  Parked items are
// queued items like any other (netem limit, flush, purge); they are only kept out of LDS.
constexpr uint32_t kWheelB = 64;   // buckets per source (one per lane)
constexpr uint32_t kWheelCB = 64;  // items per bucket (one per lane)
constexpr uint32_t kWheelGMin = 14, kWheelGMax = 40;  // bucket width 2^g ns (g >= 14: ids fit 32 bits)
struct alignas(16) WheelMeta {
  uint16_t cnt[kWheelB];  // items in each bucket (valid only while the state's q_parked() > 0)
  uint32_t base;          // lowest bucket id that may hold items
  uint32_t ctl;           // bits 0..7 g; bit 8 rebuild (the next window loads every bucket);
                          // bits 16..31 windows before another rebuild may be asked for
  uint32_t _pad[2];
};
static_assert(sizeof(WheelMeta) == 144, "WheelMeta");

// Offered packet as staged on the device (16 B, CSR by source, ordered by (tick, seq)).
struct alignas(16) InRec {
  uint32_t dst;
  uint32_t seq;
  uint32_t tick;      // relative to the step start
  uint32_t len;       // bytes (low 16 bits)
};

// Compiled FIB rule interval: every address in [lo, hi] resolves to `act` (Reject or Drop).
struct Interval {
  uint32_t lo, hi, act;
};

// Configuration delta scattered by the config-apply kernel (K9).
struct CfgPatch {
  uint32_t s;          // shard-local source
  uint32_t mask;       // bit0 last_dup, bit1 last_cor, bit2 last_reo, bit3 reset tat,
                       // bit4 flush the netem queue and departure ring (link removed)
  uint32_t last_dup, last_cor, last_reo, _pad;
  SrcParams p;
};

enum StatSlot {
  kStOffered = 0, kStScheduled, kStCloned, kStCorrupted, kStVerdict0,  // 4..11 verdicts
  kStBytes = 12, kStErr = 13, kStQueue = 14, kStLost = 15, kStFlushed = 16,
  kStCarrySkip = 17,  // modeled queue state bytes a source-major fused group kept in LDS (never moved)
  kStBktRecs = 18,    // records the simulate kernels wrote straight into destination buckets
  kStSlots = 20
};
// Counters are spread over kStatCopies copies (workgroup w adds into copy w % kStatCopies) so that
// a million one-source workgroups do not serialize on 16 addresses; readers sum the copies.  The
// error word lives in copy 0 only.
#ifndef TGSIM_STAT_COPIES
#define TGSIM_STAT_COPIES 2048
#endif
constexpr uint32_t kStatCopies = TGSIM_STAT_COPIES;  // 64 had ~16k adds per address and window at 1M
                                                     // sources: adds to one address serialize (~12 ns
                                                     // each), ~0.2 ms per window
constexpr uint32_t kErrTimeOverflow = 1u;

struct SimArgs {
  const SrcParams* params;
  SrcState* state;
  const uint8_t* enabled;   // per global peer
  const uint32_t* ip;       // per global peer
  const Interval* rules;
  const uint64_t* off;      // CSR offsets of the step's offered packets (S+1)
  const InRec* in;
  uint8_t* verdict;         // one byte per offered packet
  uint4* heap;              // [s][kHeapCap] eligibility heap, 16 B items
  uint64_t* ring;           // [s][kHeapCap] departure times, compacted (head at 0)
  tgsim_delivery* emit;     // per-source regions, base 2*off[s] + emit_r*s (EmitRead below)
  uint32_t* emit_n;         // records emitted per source this step
  unsigned long long* stats;
  uint32_t key0, key1;
  uint32_t n_src, shard_begin, n_peers, queue_limit;
  uint32_t any_disabled;    // 0: every peer is connected, the per-packet enabled[dst] gather is skipped
  uint64_t t0_ns, tick_ns, horizon_ns;
  const uint32_t* order;    // k_sim dispatch order (workgroup -> source), or null for identity
  uint64_t* stamps;         // diagnostics: kStampSlots s_memrealtime stamps per workgroup, or null
  unsigned long long* dst_cnt;  // single shard: per-destination histogram of the emitted records, or null
  uint64_t* err_host;       // pinned host word: the sticky error bits, or null
  // sparse steps: the sources k_sim_sparse left for k_sim_list; worklist[-4] their count,
  // worklist[-3] k_sim_multi's, worklist[-2] the emit-pool records claimed (zeroed before k_sim_sparse)
  uint32_t* worklist;
  // The rest of the emit layout (EmitRead): source s's first 2 n_s + emit_r records at its region; a
  // source with more (it served more than emit_r old queue items in the window) claims the rest from
  // emit_pool (worklist[-2] counts the records claimed, emit_pool_cap bounds them) and stores where
  // they start in emit_pool_idx[s].  emit_r = kHeapCap: the classic layout, which the netem limit
  // keeps every source inside (no pool; dense steps and fused windows always use it).
  tgsim_delivery* emit_pool;
  uint32_t* emit_pool_idx;
  // Gossip receipts folded into the simulate kernels (single shard, GossipArgs' tables), or null:
  // every emitted record is a receipt at its destination the moment its delivery time is known
  uint32_t* g_first;        // [s][64] earliest receipt tick
  uint64_t* g_pend;         // [s] received, not yet forwarded
  const uint64_t* g_fwd;    // [s] forwarded (stable during the step: written by k_gossip_write before it)
  uint32_t g_floods, g_degree;
  // Sparse windows of a single shard with dst_slot (below): the destinations' buckets, 2^bkt_log
  // records each.  A record whose destination slot is below that is written to
  // dst_bkt[(dst << bkt_log) + slot]
  // and never to its source's emit region (emit_n counts only the others); null: every record to the
  // emit region
  tgsim_delivery* dst_bkt;
  // dst_slot (sparse windows of a single shard): each record's arrival rank at its destination (the
  // value its dst_cnt increment returned) rides in its t_ns bits 46-63, so the local scatter places it
  // with no atomic (kSlotShift, EmitRead::slot)
  uint32_t emit_r : 24, bkt_log : 7, dst_slot : 1;  // bkt_log: log2 of a bucket's records (dst_bkt)
  uint32_t emit_pool_cap;
  // the timing wheel (WheelMeta): [s][kWheelB][kWheelCB] parked items and [s] bucket counts
  uint4* wheel;
  WheelMeta* wmeta;
  // (at exactly 256 B, kernarg windows k * 256, the scheduler had spilled 9 more SGPRs in k_sim_fused)
};
static_assert(sizeof(SimArgs) == 280, "SimArgs layout");
constexpr uint32_t kStampSlots = 32;  // 8 phase stamps + 24 profile counters (TGSIM_PROFILE)

// Fused launch of up to kFuseMax consecutive windows (k_sim_fused).  Window-major:
// ticket t -> window t / S of the (t % S)-th source in dispatch order, started once the source's
// window k - 1 has stored done[s] = step_base + k (the hand-off).  The windows differ only in these
// per-window fields.
constexpr uint32_t kFuseMax = 8;
struct FusedWindow {
  const uint64_t* off;
  const InRec* in;
  uint8_t* verdict;
  tgsim_delivery* emit;
  uint32_t* emit_n;
  unsigned long long* dst_cnt;
  uint64_t t0_ns, horizon_ns;
};
struct FusedArgs {
  FusedWindow w[kFuseMax];
  uint32_t n_win;
  uint32_t step_base;   // done[] value that window 0's predecessors have reached (window-major)
  uint32_t ticket_base; // *ticket before this launch (tickets are counted across launches)
  uint32_t* ticket;
  uint32_t* done;       // [S] last completed window of each source (wrapping step counter; window-major)
  uint32_t prio_n;      // tickets at dispatch positions below prio_n run at wave priority 3
  uint32_t persistent;  // 1: a grid of resident workgroups claims tickets until none is left; 0: one
                        // workgroup per ticket (the slots turn over, so an exchange can be dispatched)
};
constexpr uint32_t kErrHandoff = 2u;  // a window waited too long for its source's previous window
constexpr uint32_t kErrDeliverCap = 4u;  // a local delivery's records exceed its buffers (TGSIM_DELIVER_SLACK)
constexpr uint32_t kErrEmitPool = 8u;    // a sparse window's records overflowed the emit pool (TGSIM_EMIT_POOL)

// Where a window's records are, for the kernels that read them (scatter, routing, metrics,
// receipts): record i of source s is at base + 2*off[s] + r*s + i for i < cap_s = 2 n_s + r, else at
// pool + pool_idx[s] + (i - cap_s).  r = kHeapCap: the classic layout (no pool).
struct EmitRead {
  const tgsim_delivery* base;
  const tgsim_delivery* pool;
  const uint32_t* pool_idx;
  uint32_t r;
  uint32_t slot;  // the records carry their destination slot above kEMask in t_ns (SimArgs::dst_slot)
  // SimArgs::dst_bkt of the window, or null: the records with a slot below 2^bkt_log are there, not
  // in the emit records above (which hold only the others; the delivery reads both)
  const tgsim_delivery* bkt;
  uint32_t bkt_log, _pad;
  // a bounded local delivery of a bucketed window: the readers check the window's exact total (on the
  // device) against the buffers' bound themselves and write nothing past it (no k_deliver_guard)
  const uint64_t* guard_total;
  uint64_t guard_cap;
};
// A record's destination slot (its arrival rank among the window's records to that destination) in
// t_ns above the delivery time (< 2^46); kSlotNone: the rank did not fit, the scatter claims a place
// behind the first kSlotNone with a cursor atomic.
constexpr uint32_t kSlotShift = 46;
// Records per destination bucket (SimArgs::dst_bkt): 2^3 .. 2^6, chosen per window from its offered
// packets per destination
constexpr uint32_t kBktLogMin = 3, kBktLogMax = 6;
#if defined(TGSIM_CHECK) && !defined(TGSIM_CHECK_FULL_SLOTS)  // the check build sends every rank from
                                                                // 67 on through the cursor fallback
constexpr uint64_t kSlotNone = (1u << kBktLogMax) + 3;
#else
constexpr uint64_t kSlotNone = (1ull << (64 - kSlotShift)) - 1;
#endif
static_assert(kSlotNone >= (1u << kBktLogMax), "the fallback places records behind every bucket slot");
__host__ __device__ inline uint64_t slot_bits(unsigned long long rank) {
  return (uint64_t)(rank < kSlotNone ? rank : kSlotNone) << kSlotShift;
}
__host__ __device__ inline const tgsim_delivery* emit_rec(const EmitRead& e, uint32_t s, uint64_t o0, uint64_t o1,
                                                         uint32_t i, uint32_t pidx) {
  const uint64_t cap = 2 * (o1 - o0) + e.r;
  return i < cap ? e.base + 2 * o0 + (uint64_t)e.r * s + i : e.pool + pidx + (i - cap);
}
// Local delivery of a fused group: window w's emit regions, counts and CSR offsets; pos holds the
// scatter cursors of the g * n_dst (window, destination) segments.
struct GroupDeliver {
  const tgsim_delivery* emit[kFuseMax];
  const uint32_t* emit_n[kFuseMax];
  const uint64_t* off[kFuseMax];
  uint32_t n_src, n_dst;
  uint64_t* pos;
  tgsim_delivery* out;
};

// K8 metrics tables (include/tgsim.h TGSIM_METRICS_*).
constexpr uint32_t kMetricSrcWords = TGSIM_METRICS_SRC_WORDS, kMetricDstWords = TGSIM_METRICS_DST_WORDS;
constexpr uint32_t kMetricBins = TGSIM_METRICS_BINS;
struct MetricsArgs {
  const uint64_t* off;          // the step's CSR offsets (S+1)
  const InRec* in;
  const uint8_t* verdict;
  EmitRead emit;                // the step's records (per-source regions and pool)
  const uint32_t* emit_n;
  const SrcState* state;
  uint32_t n_src;
  unsigned long long* src;      // [S][kMetricSrcWords]
  unsigned long long* hist;     // [2][kMetricBins]
};

// Gossip workload state (C4) of one shard.
struct GossipArgs {
  uint32_t* first;          // [s][64] earliest receipt tick (0xFFFFFFFF: none)
  uint64_t* fwd;            // [s] floods already forwarded (or originated)
  uint64_t* pend;           // [s] floods received (or originated), not yet forwarded
  const uint32_t* nbr;      // [s][degree] out-neighbours (tabled at gossip_init), or null
  uint32_t* err;            // bit 0: a receipt precedes the generated window
  uint32_t k0, k1;          // neighbour hash key
  uint32_t n_src, shard_begin, n_peers;
  uint32_t n_floods, degree, msg_len, n_ticks;
  uint64_t tick_ns, win0;   // window start (absolute tick)
};

// Engine hooks of the RCCL exchange layer (tgsim_comm.cpp), which drives the engine through the
// public ABI and keeps its own state in the engine's comm slot (freed by tgsim_destroy).
struct CommSlot {
  void* state;
  void (*free_fn)(void*);
};
CommSlot* engine_comm_slot(void* engine);
int engine_device(void* engine);
uint32_t engine_peers(void* engine);
void engine_shard(void* engine, uint32_t* begin, uint32_t* end);
int engine_fail(void* engine, int code, const char* msg);
// Grid of a sharded fused group: 0 = one workgroup per ticket,
// else a persistent grid of pct % of the resident workgroups.
void engine_persist_routed(void* engine, uint32_t pct);
// Records `ev` on the routing stream after every routing enqueued so far (the exchange of a launched
// window waits for it on the device, not only for the host's view of the published edges).
int engine_record_routed(void* engine, hipEvent_t ev);
// Device address of the per-rank record counts of the oldest launched, unfinished routing (u64 per
// rank, written by its last routing kernel), or null.
const uint64_t* engine_route_counts_dev(void* engine);
// The largest per-rank count any routing has written so far (waits for the routing stream).
int engine_route_max(void* engine, uint64_t* out);

}  // namespace tgsim
