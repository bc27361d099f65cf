/*
 * tgoracle.h — CPU golden model of the per-packet network.Config enforcement path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the checker for the HIP engine (libtgsim.so): only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The product path
 * never calls it and fails loudly when its own HIP extension is missing.
 *
 * Parity status: the reference path is Go (pkg/sidecar) driving Linux HTB/netem/FIB through
 * vishvananda/netlink v1.1.0; none of it is buildable or runnable here (no Go toolchain, no tc,
 * no kernel sources).  The reference's own tests pin only coarse behaviour (ping-pong RTT windows
 * plans/network/pingpong.go:185,:195; splitbrain reachability plans/splitbrain/main.go:50-58;
 * config pass-through pkg/sidecar/sidecar_test.go:36,:59,:91-92).  The oracle is pinned by those
 * known answers (tests/test_oracle.py) and by Philox4x32-10 known-answer vectors; netem/HTB
 * arithmetic beyond them is "parity unpinned" against the reference and is a restatement of the
 * published netlink/kernel algorithms.
 *
 * The API mirrors include/tgsim.h function for function (tgo_* for tgsim_*) so one test driver can
 * feed identical inputs to both and compare the outputs bit for bit.
 */
#ifndef TGORACLE_H
#define TGORACLE_H

#include "../include/tgsim.h"

#ifdef __cplusplus
extern "C" {
#endif

int tgo_create(const tgsim_opts* opts, void** out);
void tgo_destroy(void* o);
const char* tgo_last_error(const void* o);
int tgo_configure(void* o, uint32_t peer, const tgsim_config* cfg);
int64_t tgo_configure_batch(void* o, const uint32_t* peers, const tgsim_config* cfgs, size_t n, int32_t* rcs);
int64_t tgo_link_generation(void* o, uint32_t peer);
int tgo_submit(void* o, const tgsim_pkt* pkts, size_t n);
int tgo_gen_storm(void* o, double lambda, uint32_t n_ticks);
int tgo_step(void* o, uint32_t n_ticks);
int tgo_step_n(void* o, uint32_t n_ticks, uint32_t n_steps);
int tgo_step_sim(void* o, uint32_t n_ticks, uint32_t n_ranks, const uint32_t* bounds, void* out, size_t cap,
                 uint64_t* counts);
int tgo_step_sim_launch(void* o, uint32_t n_ticks, uint32_t n_ranks, const uint32_t* bounds, void* out, size_t cap);
int tgo_step_sim_finish(void* o, uint64_t* counts);
int tgo_deliver(void* o, const void* in, size_t n);
int tgo_deliver_async(void* o, const void* in, size_t n, void* wait_event);
int tgo_wait_event(void* o, void* event);
int tgo_sync(void* o);
int64_t tgo_sim_capacity(void* o);
int64_t tgo_pending_deliveries(void* o);
int64_t tgo_drain(void* o, tgsim_delivery* out, size_t cap);
int64_t tgo_verdicts(void* o, uint8_t* out, size_t cap);
int tgo_stats(void* o, tgsim_stats_t* out);
int64_t tgo_signal(void* o, uint32_t state, uint32_t n);
int tgo_barrier_poll(void* o, uint32_t state, uint64_t target);
int tgo_signal_async(void* o, uint32_t state, uint32_t n);
int tgo_sync_counters(void* o, void** table, uint32_t* n_states, void* event);
int tgo_gossip_init(void* o, const tgsim_gossip* g);
int tgo_gen_gossip(void* o, uint32_t n_ticks);
int64_t tgo_gossip_reached(void* o, uint64_t* out, size_t cap);
int64_t tgo_metrics(void* o, uint32_t kind, uint64_t* out, size_t cap);

/* Building blocks exposed for known-answer tests. */
void tgo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint32_t tgo_percentage2u32(float pct);
uint32_t tgo_to_microseconds(int64_t ns);
uint32_t tgo_time2tick(uint32_t us);
/* Compiled per-instance shape: out[0]=latency_ns out[1]=jitter_ns(sigma) out[2]=rate_Bps
 * out[3]=mult out[4]=shift out[5]=burst_ns out[6..9]=thr loss,dup,corrupt,reorder
 * out[10..12]=rho dup,corrupt,reorder. */
void tgo_compile_shape(const tgsim_shape* s, uint64_t out[13]);
void tgo_poisson_table(double lambda, uint32_t out[16]);
/* Offered records produced by tgo_gen_storm for the pending step (internal CSR order). */
int64_t tgo_offered(void* o, tgsim_pkt* out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
