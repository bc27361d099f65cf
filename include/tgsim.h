/*
 * tgsim.h — C ABI of the MI355X network-emulation engine (libtgsim.so).
 *
 * This is the drop-in boundary for testground's per-packet enforcement of the sidecar's
 * network.Config.  In the reference the sidecar programs the Linux kernel (HTB + netem + FIB)
 * through netlink; every call below replaces one of those netlink/kernel interactions:
 *
 *   tgsim_configure   <- sidecar.Network.ConfigureNetwork       pkg/sidecar/instance.go:37-42
 *                        DockerNetwork.ConfigureNetwork         pkg/sidecar/docker_network.go:51-148
 *                          (network-name check :52-55, routing policy :57 -> route.go:102-117,
 *                           Enable=false disconnect :65-75, IP change :77-88,
 *                           link.Shape :139 -> link.go:155-183, link.AddRules :143 -> link.go:187-217)
 *   tgsim_submit/step <- the kernel data path the sidecar configured: FIB lookup of the
 *                        blackhole/prohibit routes (link.go:189-211), HTB class 1:2 token bucket
 *                        (link.go:118-128, :156-167), netem leaf 2:0 (link.go:131-141, :169-179)
 *   tgsim_drain       <- veth -> docker bridge -> peer delivery (pkg/runner/local_docker.go:706-721)
 *   tgsim_signal/
 *   tgsim_barrier     <- sync-service SignalEntry / SignalAndWait used by the handler
 *                        (pkg/sidecar/sidecar_handler.go:40-44, :75-80); the counters live in
 *                        device memory (K7), mirrored to pinned host memory for polling
 *   TGSIM_OPT_K8S     <- K8sNetwork.ConfigureNetwork instead of DockerNetwork's
 *                        (pkg/sidecar/k8s_network.go:114-256)
 *
 * A Go maintainer binds these with cgo.  Rules of the ABI:
 *   - plain C structs, caller-owned buffers, no exceptions across the boundary;
 *   - every int-returning call returns 0 (or a count) on success and a negative errno value on
 *     failure; tgsim_last_error() then describes the failure;
 *   - one engine handle owns its HIP stream and device memory and is NOT re-entrant: a host that
 *     calls from several goroutines/threads funnels the calls through one owner (the reference
 *     handler calls ConfigureNetwork sequentially per instance, concurrently across instances,
 *     sidecar_handler.go:26,:71 and pkg/docker/manager.go:166-177).
 *
 * Per-packet semantics (units, decision order, Philox keying, tie-breaks) are specified in
 * DESIGN.md §3 and restated independently by the CPU oracle in oracle/tgoracle.c.
 */
#ifndef TGSIM_H
#define TGSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TGSIM_ABI_VERSION 2u

/* Reserved destination id: traffic leaving the data network (the "external" routes that
 * RoutingPolicy AllowAll/DenyAll adds or removes, route.go:68-117). */
#define TGSIM_EXTERNAL 0xFFFFFFFFu

/* network.FilterAction (sdk-go; used at link.go:194-209). */
enum tgsim_filter { TGSIM_ACCEPT = 0, TGSIM_REJECT = 1, TGSIM_DROP = 2 };

/* network.RoutingPolicyType (route.go:106-112).  UNSET behaves as DenyAll (default case :110). */
enum tgsim_policy { TGSIM_POLICY_UNSET = 0, TGSIM_ALLOW_ALL = 1, TGSIM_DENY_ALL = 2 };

/* Per-packet verdict codes (low nibble: the offered packet; high nibble: its netem clone). */
enum tgsim_verdict {
    TGSIM_V_SCHEDULED = 0,    /* passed netem+HTB, delivered at tgsim_delivery.t_ns          */
    TGSIM_V_DISCONNECTED = 1, /* src or dst has Enable=false (docker_network.go:65-75)        */
    TGSIM_V_NO_ROUTE = 2,     /* external dst while routing policy != AllowAll (route.go:110) */
    TGSIM_V_BLACKHOLE = 3,    /* LinkRule Drop -> blackhole route, sender sees EINVAL         */
    TGSIM_V_PROHIBIT = 4,     /* LinkRule Reject -> prohibit route, sender sees EACCES        */
    TGSIM_V_LOSS = 5,         /* netem loss event                                             */
    TGSIM_V_QUEUE_FULL = 6,   /* netem limit (1000 packets) reached                           */
    TGSIM_V_EXTERNAL = 7,     /* external dst with AllowAll: leaves the data network unshaped */
    TGSIM_V_NONE = 15         /* (high nibble) no clone was made                              */
};

/* Delivery flags. */
#define TGSIM_FLAG_DUP 0x1u     /* this record is the netem clone of the offered packet */
#define TGSIM_FLAG_CORRUPT 0x2u /* netem corrupt event fired                          */

/* Engine flags (tgsim_opts.flags). */
#define TGSIM_OPT_KEEP_DELIVERIES 0x1u /* keep delivered records for tgsim_drain (default on via 0) */
#define TGSIM_OPT_DISCARD_DELIVERIES 0x2u /* bench: sort deliveries but do not accumulate them  */
#define TGSIM_OPT_METRICS 0x4u            /* per-instance counters and histograms (tgsim_metrics) */
/* K8sNetwork semantics (k8s_network.go:114-256) instead of DockerNetwork's (docker_network.go:51-148):
 * only network "default" (else "configured network is not `default`"); the first call re-creates
 * the data link (InitializeNetwork, :85-112); Shape -> AddRules -> routing policy, the policy only
 * on an enabled network (:246-254); connecting with an IPv6 address fails "ipv6 not supported"
 * (:161-163), after an address change has already disconnected the instance (:142-155). */
#define TGSIM_OPT_K8S 0x8u

typedef struct {
    uint32_t abi_version;  /* = TGSIM_ABI_VERSION                                          */
    uint32_t n_peers;      /* simulated instances in the whole run (all shards)            */
    uint32_t shard_begin;  /* sources owned by this engine: [shard_begin, shard_end)       */
    uint32_t shard_end;    /* 0/0 -> [0, n_peers)                                          */
    uint64_t seed;         /* Philox4x32-10 key                                            */
    uint64_t tick_ns;      /* simulation tick; 0 -> 1000 ns                                */
    uint32_t queue_limit;  /* netem limit; 0 -> 1000 (netlink default); max 1024          */
    uint32_t flags;        /* TGSIM_OPT_*                                                  */
    uint64_t lookahead_ns; /* HTB horizon beyond the step end (closed-loop drivers); 0 = none */
    uint32_t subnet_base;  /* data-network base address, host order; 0 -> 16.0.0.0          */
    int32_t device;        /* HIP device ordinal; -1 -> current device                       */
} tgsim_opts;

/* One LinkRule (network.LinkRule{LinkShape.Filter, Subnet}); only Filter is honoured, exactly as
 * in the reference (link.go:185-186). */
typedef struct {
    uint32_t prefix; /* IPv4 network address, host byte order */
    uint8_t len;     /* prefix length 0..32                    */
    uint8_t action;  /* enum tgsim_filter                      */
    uint16_t _pad;
} tgsim_rule;

/* network.LinkShape as the reference passes it to netlink (link.go:155-183). */
typedef struct {
    int64_t latency_ns;     /* time.Duration */
    int64_t jitter_ns;      /* time.Duration */
    uint64_t bandwidth_bps; /* bits/s; 0 = unlimited (link.go:156-159) */
    float loss, corrupt, corrupt_corr, reorder, reorder_corr, duplicate, duplicate_corr; /* percent */
    uint32_t _pad;
} tgsim_shape;

/* network.Config flattened (sdk-go; fields used at docker_network.go:52-143, k8s_network.go:114-254).
 * cfg.IPv4 / cfg.IPv6 are pointers in sdk-go (nil = keep the current address); has_ipv4 /
 * has_ipv6 carry that.  A changed address (docker_network.go:77-78) disconnects and reconnects the
 * instance: its netem/HTB qdiscs are re-created empty and packets still queued towards it at any
 * sender are lost (they leave the sender and find no port).  LinkRule subnets are IPv4 only: an
 * IPv6 rule subnet must be rejected by the binding, never truncated. */
typedef struct {
    const char* network;    /* must be "default" (else "unsupported network: %s") */
    uint8_t enable;
    uint8_t routing_policy; /* enum tgsim_policy */
    uint8_t has_ipv4;
    uint8_t has_ipv6;
    uint32_t ipv4;          /* host order; used when has_ipv4 */
    tgsim_shape shape;      /* cfg.Default */
    const tgsim_rule* rules;
    uint32_t n_rules;
    uint32_t _pad2;
    uint8_t ipv6[16];       /* network order; used when has_ipv6 */
} tgsim_config;

/* Offered packet, host -> engine (16 B). tick is relative to the engine's current time and must
 * be < the n_ticks of the next tgsim_step.  seq is the per-source sequence number that keys the
 * Philox stream together with (seed, src, dst). */
typedef struct {
    uint32_t src;
    uint32_t dst; /* peer id or TGSIM_EXTERNAL */
    uint32_t seq;
    uint16_t len; /* bytes on the wire */
    uint16_t tick;
} tgsim_pkt;

/* Delivered packet, engine -> host (24 B).  Drain order: (dst, t_ns, src, seq, clone first). */
typedef struct {
    uint64_t t_ns; /* delivery time (HTB departure) */
    uint32_t src;
    uint32_t dst;
    uint32_t seq;
    uint16_t len;
    uint16_t flags; /* TGSIM_FLAG_* */
} tgsim_delivery;

typedef struct {
    uint64_t offered;         /* offered packets processed (originals)            */
    uint64_t scheduled;       /* records given a delivery time (clones included)  */
    uint64_t cloned;          /* netem duplicates created                        */
    uint64_t corrupted;       /* corrupt events on scheduled records             */
    uint64_t by_verdict[8];   /* originals+clones per enum tgsim_verdict         */
    uint64_t bytes_scheduled; /* sum of len over scheduled records               */
    uint64_t now_tick;        /* engine time after the last step                 */
    uint64_t queue_state_bytes; /* netem queue state carried across steps: 16 B per
                                   queued item + 8 B per departing item, summed at
                                   every step start and end (the HBM round trip)   */
    uint64_t flushed;         /* queued/departing items lost when their sender's data
                                 link was removed (disconnect, re-addressing)       */
    uint64_t lost_in_flight;  /* records served by HTB whose destination had been
                                 disconnected or re-addressed after they were
                                 queued (no delivery)                               */
} tgsim_stats_t;

/* Closed-loop gossip flood workload, generated and consumed on the device.
 * Flood f (0 <= f < n_floods) starts at tick start_tick + f * start_gap_ticks at its origin peer;
 * every peer forwards a flood once, on its first receipt, to its `degree` out-neighbours
 * (a fixed hash of (seed, peer, k)), one msg_len-byte packet each, seq = f * degree + k, offered
 * at the tick after the receipt's delivery time.  Corrupted deliveries are not receipts. */
typedef struct {
    uint32_t n_floods;         /* 1..64                                                      */
    uint32_t degree;           /* out-neighbours per peer, 1..64                             */
    uint32_t msg_len;          /* bytes per message, 1..65535                                */
    uint32_t start_gap_ticks;  /* ticks between flood starts                                 */
    uint64_t start_tick;       /* absolute tick of flood 0 (>= the engine's next window)     */
} tgsim_gossip;

/* ---- lifecycle ---------------------------------------------------------------------------- */
int tgsim_create(const tgsim_opts* opts, void** out_engine);
void tgsim_destroy(void* engine);
const char* tgsim_last_error(const void* engine);
uint32_t tgsim_abi_version(void);

/* ---- configuration (replaces netlink: Shape / AddRules / routing policy / connect) --------- */
/* Applies cfg to instance `peer` at the engine's current time (effective for packets offered in
 * the next step).  Follows DockerNetwork.ConfigureNetwork's order of operations.  Every shard of a
 * multi-GPU run must receive every call (peer tables are replicated). */
int tgsim_configure(void* engine, uint32_t peer, const tgsim_config* cfg);
/* n tgsim_configure calls in order (cfgs[i] to peers[i]): the Go host funnels the per-instance
 * ConfigureNetwork calls into one engine goroutine, which drains its queue in one batch.
 * rcs[i] (optional) receives each call's return code; returns the number of failed calls. */
int64_t tgsim_configure_batch(void* engine, const uint32_t* peers, const tgsim_config* cfgs, size_t n,
                              int32_t* rcs);
/* How many times `peer`'s data link has been removed so far: a disconnect (Enable=false,
 * docker_network.go:65-75) or a re-addressing reconnect (:77-88; k8s_network.go:130-155).  A caller
 * that holds state about packets in flight (the packet bridge) compares it before and after a
 * tgsim_configure: a changed value means every packet queued by the peer, or towards it, is gone
 * (tgsim_stats_t.flushed / lost_in_flight) and will never be delivered. */
int64_t tgsim_link_generation(void* engine, uint32_t peer);

/* ---- data path ---------------------------------------------------------------------------- */
int tgsim_submit(void* engine, const tgsim_pkt* pkts, size_t n);
/* Storm-style synthetic traffic generated on the device for the next step:
 * per source and tick Poisson(lambda) packets to a uniform destination != src, len U{64..1500}. */
int tgsim_gen_storm(void* engine, double lambda, uint32_t n_ticks);
/* Advances time by n_ticks: every offered packet of the window goes through filter -> netem ->
 * HTB; deliveries are routed to their destination and sorted.  Single-shard convenience.
 * On an engine that owns every peer the step is asynchronous on the engine's stream (with
 * TGSIM_OPT_DISCARD_DELIVERIES and no gossip driver it returns without a host round trip); every
 * call that reads results (drain, verdicts, stats, gossip_reached, sim_kernel_ms) synchronizes
 * first.  A simulated-time overflow (-EOVERFLOW) is then reported by the next step or reader. */
int tgsim_step(void* engine, uint32_t n_ticks);
/* n_steps consecutive tgsim_step(engine, n_ticks) calls, with identical results (verdicts then
 * refer to the last window).  Windows of generated traffic (tgsim_gen_storm) on an engine that owns
 * every peer run up to kFuseMax = 8 per launch (TGSIM_FUSE, default 8): a source's next window starts as soon as its previous one
 * is done, so one window's slowest sources overlap the next window's first ones (no launch tail or
 * gap between the windows of a group).  A source whose previous window does not complete in time
 * (a hardware fault) is reported as -EIO. */
int tgsim_step_n(void* engine, uint32_t n_ticks, uint32_t n_steps);

/* Multi-shard form of tgsim_step.  Phase 1 simulates the owned sources and writes the scheduled
 * records into d_out (DEVICE memory, caller-owned, capacity out_cap records) grouped by the
 * destination's shard; rank_bounds[0..n_ranks] are the peer boundaries of the shards and
 * rank_counts[0..n_ranks-1] receives the per-shard record counts (host memory).  Returns once
 * d_out is complete and every earlier delivery (tgsim_deliver_async) has finished. */
int tgsim_step_sim(void* engine, uint32_t n_ticks, uint32_t n_ranks, const uint32_t* rank_bounds,
                   void* d_out, size_t out_cap, uint64_t* rank_counts);
/* tgsim_step_sim in two halves, so a host can start the next step's simulation before it
 * exchanges this step's records: _launch enqueues the simulation and the routing into d_out and
 * returns; _finish waits for the oldest launched step (and for earlier asynchronous deliveries)
 * and fills its counts.  Up to two launched steps may be pending (each with its own d_out), so the
 * simulate stream always has the next step queued; tgsim_step and tgsim_step_sim refuse (-EBUSY)
 * while any is.  Records beyond out_cap are dropped and reported as -ENOSPC by _finish. */
int tgsim_step_sim_launch(void* engine, uint32_t n_ticks, uint32_t n_ranks, const uint32_t* rank_bounds,
                          void* d_out, size_t out_cap);
int tgsim_step_sim_finish(void* engine, uint64_t* rank_counts);
/* tgsim_step_sim_finish without the wait for earlier asynchronous deliveries: the caller orders
 * the reuse of a delivery's input buffer on the device instead (tgsim_delivery_event), so the host
 * never blocks on the delivery stream. */
int tgsim_step_sim_counts(void* engine, uint64_t* rank_counts);
/* Slotted form of the pipelined step, for an exchange with fixed per-rank sizes (no count
 * exchange, so the host never waits for the device): d_out holds n_ranks chunks of
 * (slot_cap + 1) records; chunk r starts with a header record whose t_ns is the number of records
 * for rank r that follow it.  routed_event (a hipEvent_t, may be null) is recorded when d_out is
 * complete; the exchange waits for it on the device.  A rank whose records exceed slot_cap sets a
 * sticky error: the next step launch, release or reader fails with -ENOSPC.  _release retires the
 * oldest launched step without waiting for it. */
int tgsim_step_sim_launch_slotted(void* engine, uint32_t n_ticks, uint32_t n_ranks, const uint32_t* rank_bounds,
                                  void* d_out, uint64_t slot_cap, void* routed_event);
int tgsim_step_sim_release(void* engine);
/* Fused form of the slotted step (n_win generated windows in one launch, tgsim_step_n): d_out holds
 * n_ranks x n_win chunks of (slot_cap + 1) records, rank-major (chunk r * n_win + w: window w's
 * records for rank r behind its count header), so one all-to-all moves the whole group; counts as
 * ONE launched step for _release.  -EINVAL when the next n_win windows are not fusable. */
int tgsim_step_sim_launch_slotted_n(void* engine, uint32_t n_ticks, uint32_t n_win, uint32_t n_ranks,
                                    const uint32_t* rank_bounds, void* d_out, uint64_t slot_cap, void* routed_event);
/* tgsim_deliver_slotted_async of a fused group's exchange output (n_ranks x n_win chunks, source-rank
 * major): the windows' deliveries are appended in window order. */
int tgsim_deliver_slotted_n_async(void* engine, const void* d_in, uint32_t n_ranks, uint32_t n_win, uint64_t slot_cap,
                                  void* wait_event);
/* Phase 2: sorts the records addressed to this shard (DEVICE memory, n records) into the
 * delivery order and appends them to the drain buffer. */
int tgsim_deliver(void* engine, const void* d_in, size_t n);
/* Asynchronous phase 2: enqueues the delivery on the engine's delivery stream and returns.  The
 * stream first waits for wait_event (a hipEvent_t recorded after the producer of d_in, e.g. the
 * all-to-all; may be null), so the delivery of one step overlaps the next step's simulation.  d_in
 * must stay valid until tgsim_sync (or any reader) returns; no count check. */
int tgsim_deliver_async(void* engine, const void* d_in, size_t n, void* wait_event);
/* tgsim_deliver_async of a slotted exchange's output: n_ranks chunks of (slot_cap + 1) records,
 * each a count header and the records (the layout tgsim_step_sim_launch_slotted writes). */
int tgsim_deliver_slotted_async(void* engine, const void* d_in, uint32_t n_ranks, uint64_t slot_cap, void* wait_event);
/* Makes the engine's simulate stream wait for a hipEvent_t of another stream (e.g. the collective
 * that still reads the d_out buffer the next tgsim_step_sim will overwrite). */
int tgsim_wait_event(void* engine, void* event);
/* Records a hipEvent_t on the engine's delivery stream after every delivery enqueued so far (a
 * stream about to overwrite a delivery's input buffer waits for it). */
int tgsim_delivery_event(void* engine, void* event);
/* Waits for all of the engine's device work; reports a pending -EOVERFLOW. */
int tgsim_sync(void* engine);
/* Upper bound of records phase 1 can emit for the next step (for sizing d_out). */
int64_t tgsim_sim_capacity(void* engine);

/* Copies up to cap delivered records (oldest step first) and removes them; returns the count. */
int64_t tgsim_drain(void* engine, tgsim_delivery* out, size_t cap);
int64_t tgsim_pending_deliveries(void* engine);
/* Per-packet verdict bytes of the last step, in submit order (host packets) or generation order. */
int64_t tgsim_verdicts(void* engine, uint8_t* out, size_t cap);
int tgsim_stats(void* engine, tgsim_stats_t* out);

/* ---- RCCL exchange owned by the engine ---------------------------------- */
/* Replaces the cross-host delivery of the reference (weave CNI between k8s nodes,
 * pkg/sidecar/k8s_network.go:266-314): peers are partitioned over one engine per GPU (one process
 * per GPU), and scheduled records reach their destination's engine over RCCL (xGMI).  The engine
 * owns the communicator, its exchange stream and every buffer; a host only calls these functions
 * (INTEGRATION.md shows the Go loop).  librccl.so.1 is loaded on first use. */
#define TGSIM_COMM_ID_BYTES 128
/* A fresh communicator id (ncclGetUniqueId, 128 bytes into out_id).  One rank creates it and the
 * host hands it to every rank (the Go runner: through the sync service). */
int tgsim_comm_id(void* out_id);
/* Joins `engine` to the run's exchange as `rank` of `nranks` (<= 8) engines, one per GPU.  The
 * shards (tgsim_opts shard_begin/shard_end) must be contiguous in rank order and cover every peer;
 * they are gathered here.  Collective: every rank calls it with the same id. */
int tgsim_comm_init(void* engine, const void* id, int rank, int nranks);
/* One window on every rank (collective): simulate the owned sources, route the scheduled records
 * by destination shard, exchange the per-rank counts and then the records (grouped send/recv; the
 * own shard's records never leave the GPU), deliver them beside the next window's simulation.  The
 * host waits for this window's routing (one pinned-word poll) and for the count exchange: the
 * closed-loop form (gossip forwards, epoch reshaping) of tgsim_step. */
int tgsim_comm_step(void* engine, uint32_t n_ticks);
/* tgsim_comm_step in two halves: _launch enqueues the window's simulation and routing and returns,
 * so the host can stage the next window's ConfigureNetwork calls (they take effect at the next
 * launch) while the window simulates; _finish exchanges and delivers it. */
int tgsim_comm_launch(void* engine, uint32_t n_ticks);
int tgsim_comm_finish(void* engine);
/* n_steps pre-generated windows (tgsim_gen_storm) with the simulation two launches ahead of the
 * exchange, in groups of up to `fuse` (<= 8) windows per launch and per exchange, each rank's
 * records in fixed chunks of slot_cap records behind a count header (0: the largest per-rank count
 * of the earlier tgsim_comm_step windows, max over ranks, x 1.25 + 4096; without such windows the
 * bound of what one window can emit).  The host never waits for
 * the device.  A chunk that would overflow fails the run with -ENOSPC (nothing is lost silently). */
int tgsim_comm_run(void* engine, uint32_t n_ticks, uint32_t n_steps, uint32_t fuse, uint64_t slot_cap);
/* SignalAndWait over the shards (sync-service Barrier, sidecar_handler.go:40-44): the counts of
 * `state` are summed over the ranks by an all-reduce of the device counter tables; returns 1 when
 * the sum >= target, else 0.  Collective. */
int tgsim_comm_barrier(void* engine, uint32_t state, uint64_t target);
/* Every host wait of tgsim_comm_{step,finish,run,barrier} on a peer rank is bounded by
 * TGSIM_COMM_TIMEOUT_MS (read at tgsim_comm_init; default 300000): a rank whose peer stopped gets
 * -ETIMEDOUT naming the window, and every later tgsim_comm_* call on that engine fails the same way;
 * tgsim_destroy then aborts the communicator (ncclCommAbort) instead of waiting on it; with an RCCL
 * that has no ncclCommAbort it leaves the communicator, its stream and buffers allocated (a message on
 * stderr) rather than wait forever. */
typedef struct {
    int32_t rank, nranks;
    uint64_t exchanged_records; /* records (slotted: record slots) this rank has sent, self included */
    uint64_t max_rank_count;    /* largest per-rank count a tgsim_comm_step window routed here */
    uint64_t slot_cap;          /* chunk capacity of the last tgsim_comm_run                    */
    uint32_t bounds[9];         /* rank r owns peers [bounds[r], bounds[r + 1])                 */
    uint32_t _pad;
} tgsim_comm_info_t;
int tgsim_comm_info(void* engine, tgsim_comm_info_t* out);

/* ---- gossip workload (C4) ------------------------------------------------------------------ */
/* Arms the gossip driver: resets the per-peer receipt state of this shard and schedules the
 * floods whose origin it owns.  Requires lookahead_ns >= the window of every later step and
 * <= the minimum netem delay, so that a window's receipts are known before the next window. */
int tgsim_gossip_init(void* engine, const tgsim_gossip* g);
/* Generates the next n_ticks window of gossip traffic on the device (origins + forwards of the
 * receipts delivered so far), like tgsim_gen_storm.  The generation runs ahead of the host, so a
 * receipt that precedes the window (lookahead shorter than the window) is reported with -EINVAL by
 * the step that consumes it (or tgsim_sim_capacity, or the next tgsim_gen_gossip): that window and
 * every window queued after it are dropped without changing any peer's forwarded floods, and the
 * error stays until tgsim_gossip_init. */
int tgsim_gen_gossip(void* engine, uint32_t n_ticks);
/* Per flood, the number of this shard's peers that have the flood (received or originated);
 * out[0..n_floods).  Returns n_floods. */
int64_t tgsim_gossip_reached(void* engine, uint64_t* out, size_t cap);

/* ---- sync counters (sync-service SignalEntry / Barrier) ------------------------------------ */
/* K7: TGSIM_SYNC_STATES u64 counters in device memory, incremented by a kernel on the engine's sync
 * stream (never behind a queued simulation) that also writes the new value into a pinned host
 * mirror, so polling a barrier reads host memory and never calls the device. */
#define TGSIM_SYNC_STATES 65536u
/* Increments state `state` by n and returns the new value (1-based sequence, SignalEntry). */
int64_t tgsim_signal(void* engine, uint32_t state, uint32_t n);
/* tgsim_signal without waiting for (or returning) the new value: bulk signals such as n instances
 * entering a barrier at once.  0 on success. */
int tgsim_signal_async(void* engine, uint32_t state, uint32_t n);
/* Returns 1 when the state's count >= target, 0 otherwise (after every signal issued so far). */
int tgsim_barrier_poll(void* engine, uint32_t state, uint64_t target);
/* The device counter table (TGSIM_SYNC_STATES u64, device memory) for a collective over the
 * shards (the sum over ranks is the global count); `event` (a hipEvent_t, may be null) is recorded
 * on the sync stream after every signal issued so far, for the collective's stream to wait on. */
int tgsim_sync_counters(void* engine, void** d_table, uint32_t* n_states, void* event);

/* ---- metrics (the plans' runenv counters/histograms, pkg/metrics viewer.go:46) ---- */
/* With TGSIM_OPT_METRICS, every step folds per-instance counters and log2 histograms on the
 * device (accumulated since create).  tgsim_metrics copies one table and returns its word count:
 *   TGSIM_METRICS_SRC  [instance of this shard][12]: offered packets, offered bytes, verdict
 *                      counts 0..7 (originals + clones), HTB records served, bytes served;
 *   TGSIM_METRICS_DST  [instance of this shard][2]: records and bytes delivered to it;
 *   TGSIM_METRICS_HIST [2][64]: per step, instances by netem backlog at the step end (ring +
 *                      queue), and by records delivered to them; bin b = floor(log2 x) + 1
 *                      (bin 0: none).
 * -ENODATA when the engine was created without TGSIM_OPT_METRICS. */
enum tgsim_metrics_kind { TGSIM_METRICS_SRC = 0, TGSIM_METRICS_DST = 1, TGSIM_METRICS_HIST = 2 };
#define TGSIM_METRICS_SRC_WORDS 12u
#define TGSIM_METRICS_DST_WORDS 2u
#define TGSIM_METRICS_BINS 64u
int64_t tgsim_metrics(void* engine, uint32_t kind, uint64_t* out, size_t cap);

/* ---- packet bridge: plan payloads through the simulated network ------- */
/* The payload bytes stay on the host; each datagram becomes a 16-B tgsim_pkt for the engine, and
 * every delivery the engine drains is handed back with its payload: twice for a netem duplicate,
 * with one bit flipped for a corrupted copy (the bit from a hash of (src, seq, clone)), never for
 * a lost, filtered or queue-full one.  Packet lengths seen by netem/HTB are payload + 28 B
 * (IPv4 + UDP headers).  Replaces the veth -> bridge hop of pkg/runner/local_docker.go:706-721 for
 * plans whose sockets are bridged (tgsim_udp_front below). */
typedef struct {
    uint64_t t_ns;  /* delivery time                                    */
    uint32_t src, dst, seq;
    uint16_t flags; /* TGSIM_FLAG_*                                     */
    uint16_t _pad;
    uint64_t off;   /* payload: data[off, off + len) of the recv buffer */
    uint32_t len;
    uint32_t _pad2;
} tgsim_msg;
/* The engine calls a bridge makes (NULL ops: this library's tgsim_* functions).  The CPU tests
 * drive the same bridge over the oracle's tgo_* functions. */
typedef struct {
    int (*submit)(void*, const tgsim_pkt*, size_t);
    int (*step)(void*, uint32_t);
    int64_t (*verdicts)(void*, uint8_t*, size_t);
    int64_t (*drain)(void*, tgsim_delivery*, size_t);
} tgsim_engine_ops;
int tgsim_bridge_create(void* engine, const tgsim_engine_ops* ops, uint32_t n_peers, uint32_t window_ticks,
                        uint64_t now_tick, void** out_bridge);
void tgsim_bridge_destroy(void* bridge);
/* Queues n datagrams: src[i] -> dst[i] (TGSIM_EXTERNAL allowed) with payload data[off[i], off[i+1]),
 * offered at absolute tick ticks[i] (ticks NULL: the start of the next window).  seq_out (may be
 * NULL) receives each datagram's per-source sequence number.  Returns n or -errno. */
int64_t tgsim_bridge_send(void* bridge, size_t n, const uint32_t* src, const uint32_t* dst, const uint8_t* data,
                          const uint64_t* off, const uint64_t* ticks, uint32_t* seq_out);
/* One window: submits the datagrams due in it, steps the engine, resolves every verdict and queues
 * every delivery with its payload.  Returns the deliveries queued. */
int64_t tgsim_bridge_step(void* bridge);
/* Moves up to max queued deliveries of `peer` (UINT32_MAX: of every peer, by destination) and their
 * payloads (packed into data, cap bytes) to the caller, oldest first; returns the count. */
int64_t tgsim_bridge_recv(void* bridge, uint32_t peer, tgsim_msg* msgs, size_t max, uint8_t* data, size_t cap);
int64_t tgsim_bridge_pending(void* bridge, uint32_t peer); /* deliveries queued (UINT32_MAX: all) */
int64_t tgsim_bridge_in_flight(void* bridge);              /* datagrams sent, not yet resolved  */
/* peer's data link was removed by the last tgsim_configure (tgsim_link_generation changed): every
 * datagram already handed to the engine that was sent by peer or addressed to it is resolved as
 * lost, since the engine flushes or purges it without a delivery.  Datagrams not yet handed to the
 * engine (due in a later window) are kept.  Returns how many were resolved. */
int64_t tgsim_bridge_link_removed(void* bridge, uint32_t peer);
uint64_t tgsim_bridge_now_tick(void* bridge);              /* start of the next window          */
/* UDP front end: one socket on 127.0.0.1 receives every instance's datagrams (a 4-byte big-endian
 * destination header, then the payload) from the instance's registered address; pump() moves what
 * arrived into the bridge (recvmmsg), steps one window and sends each delivery to its destination's
 * address with a 4-byte big-endian source header (sendmmsg). */
int tgsim_udp_front_create(void* bridge, uint16_t port, void** out_front);
int tgsim_udp_front_port(void* front);
int tgsim_udp_front_register(void* front, uint32_t peer, uint32_t ipv4, uint16_t port);
/* Header-less mode for unmodified UDP code: the front end binds a socket at (ipv4, port) (port 0:
 * any) that stands for peer's data address.  A registered instance that sends a plain datagram to
 * it sends to `peer` (no destination header); every delivery from `peer` leaves from that socket,
 * so the receiver's recvfrom sees peer's data address as the source (no source header).  Any
 * 127.0.0.0/8 address works without privileges.  Returns the bound port or -errno.  (TUN/TAP
 * capture, which would carry TCP too, needs /dev/net/tun and CAP_NET_ADMIN: DESIGN.md §9.) */
int tgsim_udp_front_bind_peer(void* front, uint32_t peer, uint32_t ipv4, uint16_t port);
int64_t tgsim_udp_front_pump(void* front);
void tgsim_udp_front_destroy(void* front);

/* ---- device timing (bench instrumentation) ------------------------------------------------ */
/* Average device time (ms) of the simulate kernel over the steps since the last reset, measured
 * with HIP events on the engine's stream. */
double tgsim_sim_kernel_ms(void* engine, uint64_t* n_launches, int reset);
/* The same for the delivery (K5: per-destination histogram scan, scatter, per-destination sort),
 * from its first kernel to its sort on the delivery stream, per window delivered (a fused group's
 * delivery counts each of its windows).  The span includes the time its kernels wait for CU slots
 * beside the next window's simulate kernel. */
double tgsim_delivery_kernel_ms(void* engine, uint64_t* n_windows, int reset);
void* tgsim_stream(void* engine);
/* Diagnostics: with TGSIM_STAMPS set at create time, the simulate kernel records 24 words per
 * workgroup (s_memrealtime at its phase boundaries, batch count, HW_ID, queue sizes); copies them
 * for the last step and returns the word count (0 when disabled). */
int64_t tgsim_debug_stamps(void* engine, uint64_t* out, size_t cap);
/* Diagnostics: HBM bytes the simulate kernels actually moved carrying netem queues and departure
 * rings between windows since the engine was created (loads + stores).  tgsim_stats_t's
 * queue_state_bytes models one load and one store per window; a fused group (tgsim_step_n) keeps
 * each source's queue in LDS across its windows and moves it once per group. */
int64_t tgsim_debug_carry_bytes(void* engine);
/* Diagnostics: records the simulate kernels wrote straight into destination buckets (sparse windows
 * of an engine that owns every peer) since the engine was created.  The others went
 * through the emit regions and the scatter. */
int64_t tgsim_debug_bucket_records(void* engine);
/* Diagnostics: windows simulated by fused launches (tgsim_step_n) since the engine was created. */
int64_t tgsim_debug_fused_windows(void* engine);
/* Diagnostics: windows simulated by the sparse kernels (k_sim_sparse + k_sim_multi + k_sim_list) since
 * the engine was created; the others ran the dense k_sim (or were fused). */
int64_t tgsim_debug_sparse_windows(void* engine);
/* Diagnostics of a TGSIM_CHECK build of the engine (scripts/r05_check_build.sh): cross-lane reads whose
 * source lanes were inactive so far, process-wide.  -ENOSYS in the product build. */
int64_t tgsim_debug_exec_faults(void);

#ifdef __cplusplus
}
#endif

#endif /* TGSIM_H */
