/*
 * tgoracle.c — CPU golden model (TEST INFRASTRUCTURE ONLY; see tgoracle.h for the contract).
 *
 * A deliberately plain, single-threaded restatement of the per-packet step, written from the
 * reference's call sites and the published netlink/kernel algorithms, NOT from the HIP engine:
 *
 *   unit conversion      pkg/sidecar/link.go:143-151 (toMicroseconds); netlink v1.1.0
 *                        time2Tick / Percentage2u32 / NewNetem / NewHtbClass / Xmittime [ext]
 *   shape application    link.go:155-183 (HTB class rate, netem attrs; no LossCorr/DelayCorr)
 *   rule semantics       link.go:187-217 (Accept deletes, Reject=prohibit, Drop=blackhole,
 *                        cumulative across configs, rule LinkShape ignored)
 *   routing policy       route.go:102-117 (AllowAll enables external routes, anything else denies)
 *   order of operations  docker_network.go:51-148 (docker), k8s_network.go:114-256 (TGSIM_OPT_K8S)
 *   link removal         NetworkDisconnect / CNI DelNetworkList drop the link with its qdiscs
 *                        (docker_network.go:65-75, :84-87; k8s_network.go:134, :151): queued
 *                        items are lost, packets queued towards the instance find no port
 *   per-packet enqueue   Linux sch_netem.c netem_enqueue (dup -> loss -> clone -> corrupt ->
 *                        limit -> reorder/delay), tabledist uniform branch, get_crandom [ext]
 *   token bucket         Linux sch_htb.c class tokens + psched_ratecfg_precompute/l2t_ns [ext]
 *
 * Every decision is keyed by Philox4x32-10(key = seed, ctr = (src, dst, seq, draw)), so results
 * do not depend on evaluation order, sharding or step partitioning.
 */
#include "tgoracle.h"

#include <errno.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11; constants as Random123 / rocrand_philox4x32_10.h:62-65) */
void tgo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* ------------------------------------------------------------------------------------------ */
/* Go float->uint32 conversion on amd64: truncate to int64, keep the low 32 bits; NaN/Inf/out of
 * range yield the "integer indefinite" 0x8000000000000000, whose low 32 bits are 0. */
static uint32_t go_f64_to_u32(double x) {
    if (!(x > -9.2233720368547758e18 && x < 9.2233720368547758e18)) return 0;
    return (uint32_t)(int64_t)x;
}

/* netlink Percentage2u32: float32 arithmetic on math.MaxUint32 (rounds to 2^32 as float32). */
uint32_t tgo_percentage2u32(float pct) {
    if (pct == 100.0f) return 0xFFFFFFFFu;
    volatile float q = pct / 100.0f;
    volatile float v = 4294967296.0f * q;
    return go_f64_to_u32((double)v);
}

/* link.go:143-151: Duration.Microseconds() truncates toward zero, clamp at MaxUint32, uint32(). */
uint32_t tgo_to_microseconds(int64_t ns) {
    int64_t us = ns / 1000;
    if (us > (int64_t)0xFFFFFFFFu) us = 0xFFFFFFFFu;
    return (uint32_t)us;
}

/* netlink time2Tick with /proc/net/psched = 3e8 40 f4240 3b9aca00: tickInUsec = 1000/64. */
uint32_t tgo_time2tick(uint32_t us) { return go_f64_to_u32((double)us * 15.625); }

/* psched_ratecfg_precompute (net/sched/sch_generic.c). */
static void ratecfg(uint64_t rate_bps_bytes, uint32_t* mult, uint32_t* shift) {
    *mult = 1;
    *shift = 0;
    if (rate_bps_bytes > 0) {
        uint64_t factor = 1000000000ull;
        for (;;) {
            *mult = (uint32_t)(factor / rate_bps_bytes);
            if ((*mult & (1u << 31)) || (factor & (1ull << 63))) break;
            factor <<= 1;
            (*shift)++;
        }
    }
}

typedef struct {
    uint64_t lat_ns;
    int32_t sigma;
    uint64_t rate_Bps;
    uint32_t mult, shift;
    uint64_t burst_ns;
    uint32_t thr_loss, thr_dup, thr_cor, thr_reo;
    uint32_t rho_dup, rho_cor, rho_reo;
    int cor_set, dup_corr_set, reo_set;
} cshape;

static void compile_shape(const tgsim_shape* s, cshape* c) {
    memset(c, 0, sizeof *c);
    /* netem (link.go:169-179 -> netlink NewNetem) */
    uint32_t lat_us = tgo_to_microseconds(s->latency_ns);
    uint32_t jit_us = tgo_to_microseconds(s->jitter_ns);
    uint32_t lat_t = tgo_time2tick(lat_us);
    uint32_t jit_t = lat_t > 0 ? tgo_time2tick(jit_us) : jit_us; /* "Jitter is only valid if latency is > 0" */
    c->lat_ns = (uint64_t)lat_t << 6;                             /* PSCHED_TICKS2NS */
    uint64_t jit_ns = (uint64_t)jit_t << 6;
    c->sigma = (int32_t)(uint32_t)jit_ns; /* tabledist(s64 mu, s32 sigma, ...) */
    if ((uint32_t)c->sigma == 0x80000000u) c->sigma = 0x7FFFFFFF; /* 2*(u32)sigma would be 0 */
    c->thr_loss = tgo_percentage2u32(s->loss);
    c->thr_dup = tgo_percentage2u32(s->duplicate);
    c->thr_reo = tgo_percentage2u32(s->reorder);
    c->thr_cor = tgo_percentage2u32(s->corrupt);
    c->rho_dup = c->thr_dup > 0 ? tgo_percentage2u32(s->duplicate_corr) : 0;
    c->rho_reo = tgo_percentage2u32(s->reorder_corr);
    c->rho_cor = tgo_percentage2u32(s->corrupt_corr);
    c->cor_set = c->thr_cor > 0;     /* TCA_NETEM_CORRUPT only when Probability > 0 */
    c->reo_set = c->thr_reo > 0;     /* TCA_NETEM_REORDER only when Probability > 0 (gap = 1) */
    c->dup_corr_set = c->rho_dup > 0; /* TCA_NETEM_CORR only when a correlation > 0 */
    /* HTB class (link.go:156-167 -> netlink NewHtbClass: rate/8, mtu 1600, hz 1e9) */
    uint64_t rate = s->bandwidth_bps ? s->bandwidth_bps : UINT64_MAX;
    uint64_t rate_B = rate / 8;
    uint32_t buf_bytes = go_f64_to_u32((double)rate_B / 1e9 + 1600.0);
    uint32_t buf_us = go_f64_to_u32(1000000.0 * ((double)buf_bytes / (double)rate_B));
    c->burst_ns = (uint64_t)tgo_time2tick(buf_us) << 6;
    c->rate_Bps = (uint32_t)rate_B; /* TcRateSpec.Rate is u32 in netlink v1.1.0 (no RATE64) */
    ratecfg(c->rate_Bps, &c->mult, &c->shift);
}

void tgo_compile_shape(const tgsim_shape* s, uint64_t out[13]) {
    cshape c;
    compile_shape(s, &c);
    out[0] = c.lat_ns; out[1] = (uint64_t)(int64_t)c.sigma; out[2] = c.rate_Bps; out[3] = c.mult;
    out[4] = c.shift; out[5] = c.burst_ns; out[6] = c.thr_loss; out[7] = c.thr_dup;
    out[8] = c.thr_cor; out[9] = c.thr_reo; out[10] = c.rho_dup; out[11] = c.rho_cor;
    out[12] = c.rho_reo;
}

/* Poisson(lambda) CDF as u32 thresholds (storm generator). */
void tgo_poisson_table(double lambda, uint32_t out[16]) {
    double p = exp(-lambda), F = p;
    for (int k = 0; k < 16; ++k) {
        double t = F * 4294967296.0;
        out[k] = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
        p = p * lambda / (double)(k + 1);
        F = F + p;
    }
}

/* ------------------------------------------------------------------------------------------ */
typedef struct {
    uint64_t e;
    uint32_t seq, dst;
    uint16_t len, flags;
} item;

typedef struct {
    uint32_t net;
    uint8_t len, action;
} rule;

typedef struct {
    /* netem/HTB parameters currently installed (kernel-side state, incl. persisting quirks) */
    uint64_t lat_ns, burst_ns;
    int32_t sigma;
    uint32_t mult, shift;
    uint32_t thr_loss, thr_dup, thr_cor, thr_reo;
    uint32_t rho_dup, rho_cor, rho_reo;
    uint32_t last_dup, last_cor, last_reo;
    uint32_t shape_epoch;
    int allow_ext;
    /* FIB rules of this instance */
    rule* rules;
    uint32_t n_rules, cap_rules;
    /* queue state */
    uint64_t tat;
    item* heap;
    uint32_t heap_n;
    uint64_t* ring;
    uint32_t ring_head, ring_n;
} source;

typedef struct {
    tgsim_pkt p;
    uint64_t idx;
} offered;

typedef struct {
    tgsim_opts o;
    char err[256];
    uint32_t nsrc;
    source* src;
    uint8_t* enabled;
    uint32_t* ip;
    uint8_t* ip6_set;   /* the link carries an IPv6 address (cfg.IPv6 was given at connect) */
    uint8_t (*ip6)[16];
    uint8_t* k8s_init;  /* K8sNetwork.initialized, per instance (k8s_network.go:119-125) */
    uint32_t* link_gen; /* data links removed per instance (tgsim_link_generation) */
    uint32_t key[2];
    uint64_t now_tick;
    offered* off;
    size_t n_off, cap_off;
    /* device-generated windows queued ahead of the steps that consume them (tgsim_gen_*) */
    /* late: a gossip window generated while a receipt already preceded it (no packets); reported
     * as the HIP engine reports it, by the call that resolves it: the step that consumes it,
     * tgsim_sim_capacity, or the next tgsim_gen_gossip (its generation runs ahead of the host) */
    struct genwin { offered* pk; size_t n, cap; uint32_t ticks; int late; uint32_t late_tick; uint64_t win0; } *gq;
    size_t gq_n, gq_cap;
    uint64_t gq_ticks;
    uint8_t* verdicts;
    size_t n_verdicts;
    tgsim_delivery* out; /* undrained deliveries */
    size_t n_out, cap_out, out_head;
    tgsim_delivery* step_out;
    size_t n_step, cap_step;
    tgsim_stats_t st;
    uint64_t counters[TGSIM_SYNC_STATES];
    uint32_t* gen_seq;
    /* gossip workload (C4): receipt tick per (local peer, flood), forwarded-flood bitmask */
    int gossip_on;
    int gossip_late; /* sticky until tgo_gossip_init: a receipt preceded a generated window */
    tgsim_gossip g;
    uint32_t* g_first;
    uint64_t* g_fwd;
    /* K8 metrics (TGSIM_OPT_METRICS): per-instance tables and the two log2 histograms */
    int metrics_on;
    uint64_t* m_src; /* [nsrc][TGSIM_METRICS_SRC_WORDS] */
    uint64_t* m_dst; /* [nsrc][TGSIM_METRICS_DST_WORDS] */
    uint64_t m_hist[2 * TGSIM_METRICS_BINS];
    /* split step_sim: counts of a launched, not yet finished step */
    uint64_t pend_counts[2][8];
    uint32_t pend_ranks[2], pend_head, pend_n;
} oracle;

#define HCAP 1024u

static int fail(oracle* o, int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(o->err, sizeof o->err, fmt, ap);
    va_end(ap);
    return code;
}

static void* grow(void* p, size_t* cap, size_t need, size_t elem) {
    if (need <= *cap) return p;
    size_t nc = *cap ? *cap : 64;
    while (nc < need) nc *= 2;
    void* q = realloc(p, nc * elem);
    if (!q) abort();
    *cap = nc;
    return q;
}

/* Appends a new generated window of n_ticks starting at now_tick + gq_ticks. */
static struct genwin* gen_window(oracle* o, uint32_t n_ticks) {
    o->gq = grow(o->gq, &o->gq_cap, o->gq_n + 1, sizeof *o->gq);
    struct genwin* w = &o->gq[o->gq_n++];
    memset(w, 0, sizeof *w);
    w->ticks = n_ticks;
    return w;
}

/* The late window gq[i] is reported: it and every window queued after it are dropped (the ones
 * before it stay queued and can still be stepped), and the error stays until gossip_init. */
static int gen_report_late(oracle* o, size_t i) {
    const uint32_t t = o->gq[i].late_tick;
    const unsigned long long a = (unsigned long long)o->gq[i].win0;
    for (size_t k = i; k < o->gq_n; ++k) {
        free(o->gq[k].pk);
        o->gq_ticks -= o->gq[k].ticks;
    }
    o->gq_n = i;
    o->gossip_late = 1;
    return fail(o, -EINVAL, "gossip: a receipt at tick %u precedes the window at %llu", t, a);
}

static void gen_push(struct genwin* w, const tgsim_pkt* k) {
    w->pk = grow(w->pk, &w->cap, w->n + 1, sizeof(offered));
    w->pk[w->n].p = *k;
    w->pk[w->n].idx = w->n;
    w->n++;
}

static void reset_netem(oracle* o, uint32_t s) {
    source* S = &o->src[s];
    S->lat_ns = 0; S->burst_ns = 0; S->sigma = 0;
    S->thr_loss = S->thr_dup = S->thr_cor = S->thr_reo = 0;
    S->rho_dup = S->rho_cor = S->rho_reo = 0;
    S->last_dup = S->last_cor = S->last_reo = 0;
    /* HTB class created with Rate MaxUint64 (link.go:98-105) */
    tgsim_shape z;
    memset(&z, 0, sizeof z);
    cshape c;
    compile_shape(&z, &c);
    S->mult = c.mult; S->shift = c.shift; S->burst_ns = c.burst_ns;
    S->tat = 0;
}

int tgo_create(const tgsim_opts* opts, void** out) {
    if (!opts || !out) return -EINVAL;
    if (opts->abi_version != TGSIM_ABI_VERSION) return -EPROTO;
    if (opts->n_peers == 0) return -EINVAL;
    oracle* o = (oracle*)calloc(1, sizeof *o);
    o->o = *opts;
    if (o->o.shard_begin == 0 && o->o.shard_end == 0) o->o.shard_end = o->o.n_peers;
    if (o->o.shard_begin >= o->o.shard_end || o->o.shard_end > o->o.n_peers) {
        free(o);
        return -EINVAL;
    }
    if (!o->o.tick_ns) o->o.tick_ns = 1000;
    if (!o->o.queue_limit) o->o.queue_limit = 1000;
    if (o->o.queue_limit > HCAP) {
        free(o);
        return -EINVAL;
    }
    if (!o->o.subnet_base) o->o.subnet_base = 16u << 24;
    o->key[0] = (uint32_t)o->o.seed;
    o->key[1] = (uint32_t)(o->o.seed >> 32);
    o->nsrc = o->o.shard_end - o->o.shard_begin;
    o->src = (source*)calloc(o->nsrc, sizeof(source));
    o->enabled = (uint8_t*)malloc(o->o.n_peers);
    memset(o->enabled, 1, o->o.n_peers); /* containers start attached (local_docker.go:459) */
    o->ip = (uint32_t*)malloc(sizeof(uint32_t) * o->o.n_peers);
    o->ip6_set = (uint8_t*)calloc(o->o.n_peers, 1);
    o->ip6 = calloc(o->o.n_peers, 16);
    o->k8s_init = (uint8_t*)calloc(o->o.n_peers, 1);
    o->link_gen = (uint32_t*)calloc(o->o.n_peers, sizeof(uint32_t));
    for (uint32_t i = 0; i < o->o.n_peers; ++i) o->ip[i] = o->o.subnet_base + 2 + i;
    o->gen_seq = (uint32_t*)calloc(o->nsrc, sizeof(uint32_t));
    o->metrics_on = (o->o.flags & TGSIM_OPT_METRICS) != 0;
    if (o->metrics_on) {
        o->m_src = (uint64_t*)calloc((size_t)o->nsrc * TGSIM_METRICS_SRC_WORDS, sizeof(uint64_t));
        o->m_dst = (uint64_t*)calloc((size_t)o->nsrc * TGSIM_METRICS_DST_WORDS, sizeof(uint64_t));
    }
    for (uint32_t s = 0; s < o->nsrc; ++s) {
        o->src[s].heap = (item*)malloc(sizeof(item) * HCAP);
        o->src[s].ring = (uint64_t*)malloc(sizeof(uint64_t) * HCAP);
        reset_netem(o, s);
    }
    *out = o;
    return 0;
}

void tgo_destroy(void* p) {
    oracle* o = (oracle*)p;
    if (!o) return;
    for (uint32_t s = 0; s < o->nsrc; ++s) {
        free(o->src[s].heap);
        free(o->src[s].ring);
        free(o->src[s].rules);
    }
    for (size_t i = 0; i < o->gq_n; ++i) free(o->gq[i].pk);
    free(o->gq);
    free(o->src); free(o->enabled); free(o->ip); free(o->off); free(o->verdicts);
    free(o->ip6_set); free(o->ip6); free(o->k8s_init); free(o->link_gen);
    free(o->out); free(o->step_out); free(o->gen_seq); free(o->g_first); free(o->g_fwd);
    free(o->m_src); free(o->m_dst);
    free(o);
}

const char* tgo_last_error(const void* p) { return p ? ((const oracle*)p)->err : "null engine"; }

/* link.go:187-217 */
static int add_rules(oracle* o, source* S, const tgsim_rule* rules, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) {
        const tgsim_rule* r = &rules[i];
        int bad = r->len > 32;
        uint32_t mask = (!bad && r->len) ? (0xFFFFFFFFu << (32 - r->len)) : 0;
        bad = bad || (r->prefix & ~mask) != 0; /* fib_table_insert/delete reject host bits */
        if (r->action == TGSIM_ACCEPT) {         /* RouteDel blackhole + prohibit, errors ignored */
            if (bad) continue;
            for (uint32_t j = 0; j < S->n_rules;) {
                if (S->rules[j].net == r->prefix && S->rules[j].len == r->len) {
                    S->rules[j] = S->rules[--S->n_rules];
                } else {
                    ++j;
                }
            }
            continue;
        }
        if (r->action != TGSIM_REJECT && r->action != TGSIM_DROP)
            return fail(o, -EINVAL, "invalid filter action %u", r->action);
        if (bad) return fail(o, -EINVAL, "invalid argument");
        uint32_t j;
        for (j = 0; j < S->n_rules; ++j)
            if (S->rules[j].net == r->prefix && S->rules[j].len == r->len) break;
        if (j == S->n_rules) { /* RouteReplace creates */
            size_t cap = S->cap_rules;
            S->rules = (rule*)grow(S->rules, &cap, (size_t)S->n_rules + 1, sizeof(rule));
            S->cap_rules = (uint32_t)cap;
            S->rules[S->n_rules].net = r->prefix;
            S->rules[S->n_rules].len = r->len;
            S->n_rules++;
        }
        S->rules[j].action = r->action;
    }
    return 0;
}

#define DEAD_DST 0xFFFFFFFFu /* queued item whose destination link went away (never a real queued dst) */

/* The instance's data link is removed: its HTB/netem qdiscs die with what they hold, and every
 * packet still waiting in some sender's netem queue towards it will leave into a missing port. */
static void link_down(oracle* o, uint32_t peer) {
    o->enabled[peer] = 0;
    o->link_gen[peer]++;
    if (peer >= o->o.shard_begin && peer < o->o.shard_end) {
        source* S = &o->src[peer - o->o.shard_begin];
        o->st.flushed += S->heap_n + S->ring_n;
        S->heap_n = 0;
        S->ring_n = 0;
        S->ring_head = 0;
    }
    for (uint32_t s = 0; s < o->nsrc; ++s)
        for (uint32_t k = 0; k < o->src[s].heap_n; ++k)
            if (o->src[s].heap[k].dst == peer) o->src[s].heap[k].dst = DEAD_DST;
}

/* A new data link: NetworkConnect / CNI AddNetworkList with the requested addresses, then
 * NewNetlinkLink's fresh HTB class and netem qdisc. */
static void link_up(oracle* o, uint32_t peer, const tgsim_config* cfg) {
    o->enabled[peer] = 1;
    if (cfg->has_ipv4) o->ip[peer] = cfg->ipv4;
    o->ip6_set[peer] = cfg->has_ipv6 != 0;
    if (cfg->has_ipv6) memcpy(o->ip6[peer], cfg->ipv6, 16);
    if (peer >= o->o.shard_begin && peer < o->o.shard_end) {
        uint32_t s = peer - o->o.shard_begin;
        source* S = &o->src[s];
        o->st.flushed += S->heap_n + S->ring_n;
        S->heap_n = 0;
        S->ring_n = 0;
        S->ring_head = 0;
        reset_netem(o, s);
    }
}

/* link.Shape (link.go:155-183) with netem_change's handling of absent attributes. */
static void shape_link(oracle* o, uint32_t peer, const tgsim_shape* shape) {
    source* S = &o->src[peer - o->o.shard_begin];
    cshape c;
    compile_shape(shape, &c);
    S->shape_epoch++;
    uint32_t ctr[4] = {peer, 0xFFFFFFFEu, S->shape_epoch, 3}, rnd[4]; /* init_crandom: last = random */
    tgo_philox4x32_10(ctr, o->key, rnd);
    S->lat_ns = c.lat_ns;
    S->sigma = c.sigma;
    S->thr_loss = c.thr_loss;
    S->thr_dup = c.thr_dup;
    if (c.dup_corr_set) { S->rho_dup = c.rho_dup; S->last_dup = rnd[0]; }
    if (c.cor_set) { S->thr_cor = c.thr_cor; S->rho_cor = c.rho_cor; S->last_cor = rnd[1]; }
    if (c.reo_set) { S->rho_reo = c.rho_reo; S->last_reo = rnd[2]; }
    S->thr_reo = c.thr_reo; /* gap = 0 disables reordering whatever q->reorder holds */
    S->mult = c.mult;
    S->shift = c.shift;
    S->burst_ns = c.burst_ns;
}

static int owned_peer(const oracle* o, uint32_t peer) { return peer >= o->o.shard_begin && peer < o->o.shard_end; }

static void routing_policy(oracle* o, uint32_t peer, uint8_t policy) { /* route.go:102-117 */
    if (owned_peer(o, peer)) o->src[peer - o->o.shard_begin].allow_ext = policy == TGSIM_ALLOW_ALL;
}

static int ipv4_differs(const oracle* o, uint32_t peer, const tgsim_config* cfg) {
    return cfg->has_ipv4 && cfg->ipv4 != o->ip[peer];
}

int64_t tgo_link_generation(void* p, uint32_t peer) {
    oracle* o = (oracle*)p;
    if (!o || peer >= o->o.n_peers) return -EINVAL;
    return o->link_gen[peer];
}

int tgo_configure(void* p, uint32_t peer, const tgsim_config* cfg) {
    oracle* o = (oracle*)p;
    if (!o || !cfg) return -EINVAL;
    if (peer >= o->o.n_peers) return fail(o, -EINVAL, "peer %u out of range", peer);
    const char* net = cfg->network ? cfg->network : "";
    int online;
    if (!(o->o.flags & TGSIM_OPT_K8S)) {
        /* DockerNetwork.ConfigureNetwork, docker_network.go:51-148 */
        if (strcmp(net, "default") != 0) return fail(o, -EINVAL, "unsupported network: %s", net);
        routing_policy(o, peer, cfg->routing_policy); /* :57 */
        online = o->enabled[peer];
        if (!cfg->enable) { /* :65-75 */
            if (online) link_down(o, peer);
            return 0;
        }
        int v6 = cfg->has_ipv6 && (!o->ip6_set[peer] || memcmp(o->ip6[peer], cfg->ipv6, 16) != 0);
        if (online && (v6 || ipv4_differs(o, peer, cfg))) { /* :77-88 */
            link_down(o, peer);
            online = 0;
        }
        if (!online) link_up(o, peer, cfg); /* :90-137 */
        if (!owned_peer(o, peer)) return 0;
        shape_link(o, peer, &cfg->shape);                                                /* :139 */
        return add_rules(o, &o->src[peer - o->o.shard_begin], cfg->rules, cfg->n_rules); /* :143 */
    }
    /* K8sNetwork.ConfigureNetwork, k8s_network.go:114-256 */
    if (strcmp(net, "default") != 0) return fail(o, -EINVAL, "configured network is not `default`");
    if (!o->k8s_init[peer]) { /* :119-125, InitializeNetwork removes the pod's original address */
        o->k8s_init[peer] = 1;
        if (o->enabled[peer]) link_down(o, peer);
    }
    online = o->enabled[peer];
    if (!cfg->enable) { /* :130-140 */
        if (online) link_down(o, peer);
        return 0;
    }
    if (online && (cfg->has_ipv6 || ipv4_differs(o, peer, cfg))) { /* :142-155, links hold no IPv6 */
        link_down(o, peer);
        online = 0;
    }
    if (!online) {
        if (cfg->has_ipv6) return fail(o, -EAFNOSUPPORT, "ipv6 not supported"); /* :161-163 */
        link_up(o, peer, cfg);
    }
    if (owned_peer(o, peer)) {
        shape_link(o, peer, &cfg->shape); /* :246-248 */
        int rc = add_rules(o, &o->src[peer - o->o.shard_begin], cfg->rules, cfg->n_rules); /* :249-251 */
        if (rc) return rc;
    }
    routing_policy(o, peer, cfg->routing_policy); /* :252-254 */
    return 0;
}

int tgo_submit(void* p, const tgsim_pkt* pkts, size_t n) {
    oracle* o = (oracle*)p;
    if (!o || (!pkts && n)) return -EINVAL;
    if (o->gq_n) return fail(o, -EBUSY, "generated traffic already pending for the next step");
    for (size_t i = 0; i < n; ++i) {
        const tgsim_pkt* k = &pkts[i];
        if (k->src < o->o.shard_begin || k->src >= o->o.shard_end)
            return fail(o, -EINVAL, "packet %zu: src %u not owned by this shard", i, k->src);
        if (k->dst != TGSIM_EXTERNAL && k->dst >= o->o.n_peers)
            return fail(o, -EINVAL, "packet %zu: dst %u out of range", i, k->dst);
    }
    o->off = (offered*)grow(o->off, &o->cap_off, o->n_off + n, sizeof(offered));
    for (size_t i = 0; i < n; ++i) {
        o->off[o->n_off].p = pkts[i];
        o->off[o->n_off].idx = o->n_off;
        o->n_off++;
    }
    return 0;
}

int64_t tgo_configure_batch(void* p, const uint32_t* peers, const tgsim_config* cfgs, size_t n, int32_t* rcs) {
    if (!p || (n && (!peers || !cfgs))) return -EINVAL;
    int64_t failed = 0;
    for (size_t i = 0; i < n; ++i) {
        int rc = tgo_configure(p, peers[i], &cfgs[i]);
        if (rcs) rcs[i] = rc;
        failed += rc != 0;
    }
    return failed;
}

/* Storm generator restatement: per (src, tick) Poisson count, uniform dst != src,
 * len 64 + u mod 1437. */
int tgo_gen_storm(void* p, double lambda, uint32_t n_ticks) {
    oracle* o = (oracle*)p;
    if (!o || !(lambda >= 0.0) || lambda > 4.0 || n_ticks > 65536) return -EINVAL;
    uint32_t tab[16];
    tgo_poisson_table(lambda, tab);
    uint32_t gk[2] = {o->key[0] ^ 0x9E3779B9u, o->key[1] ^ 0x7F4A7C15u};
    uint32_t N = o->o.n_peers;
    if (n_ticks == 0) return -EINVAL;
    if (o->n_off) return fail(o, -EBUSY, "host packets already pending for the next step");
    const uint64_t base = o->now_tick + o->gq_ticks;
    struct genwin* w = gen_window(o, n_ticks);
    o->gq_ticks += n_ticks;
    if (N < 2) return 0;
    for (uint32_t s = 0; s < o->nsrc; ++s) {
        uint32_t src = o->o.shard_begin + s;
        for (uint32_t t = 0; t < n_ticks; ++t) {
            uint32_t abs_t = (uint32_t)(base + t);
            uint32_t ctr[4] = {src, abs_t, 0x53544F52u, 0}, r[4];
            tgo_philox4x32_10(ctr, gk, r);
            uint32_t cnt = 0;
            while (cnt < 16 && r[0] >= tab[cnt]) cnt++;
            for (uint32_t j = 0; j < cnt; ++j) {
                uint32_t c2[4] = {src, abs_t, 0x53544F52u, j + 1}, q[4];
                tgo_philox4x32_10(c2, gk, q);
                uint32_t d = q[0] % (N - 1);
                if (d >= src) d++;
                tgsim_pkt k;
                k.src = src; k.dst = d; k.seq = o->gen_seq[s]++;
                k.len = (uint16_t)(64 + q[1] % 1437u); k.tick = (uint16_t)t;
                gen_push(w, &k);
            }
        }
    }
    return 0;
}

int64_t tgo_offered(void* p, tgsim_pkt* out, size_t cap) {
    oracle* o = (oracle*)p;
    const offered* src = o->n_off || !o->gq_n ? o->off : o->gq[0].pk;  /* next step's input */
    size_t m = o->n_off || !o->gq_n ? o->n_off : o->gq[0].n;
    size_t n = m < cap ? m : cap;
    for (size_t i = 0; i < n; ++i) out[i] = src[i].p;
    return (int64_t)m;
}

/* ------------------------------------------------------------------------------------------ */
static int item_lt(const item* a, const item* b) {
    if (a->e != b->e) return a->e < b->e;
    if (a->seq != b->seq) return a->seq < b->seq;
    return (a->flags & TGSIM_FLAG_DUP) && !(b->flags & TGSIM_FLAG_DUP); /* clone enqueued first */
}

static void heap_push(source* S, item it) {
    uint32_t i = S->heap_n++;
    while (i > 0) {
        uint32_t p = (i - 1) / 2;
        if (!item_lt(&it, &S->heap[p])) break;
        S->heap[i] = S->heap[p];
        i = p;
    }
    S->heap[i] = it;
}

static item heap_pop(source* S) {
    item top = S->heap[0];
    item last = S->heap[--S->heap_n];
    uint32_t i = 0, n = S->heap_n;
    for (;;) {
        uint32_t c = 2 * i + 1;
        if (c >= n) break;
        if (c + 1 < n && item_lt(&S->heap[c + 1], &S->heap[c])) c++;
        if (!item_lt(&S->heap[c], &last)) break;
        S->heap[i] = S->heap[c];
        i = c;
    }
    if (n) S->heap[i] = last;
    return top;
}

/* HTB class 1:2 serving the netem leaf in eligibility order (sch_htb.c tokens in ns). */
static void htb_until(oracle* o, uint32_t s, uint64_t horizon) {
    source* S = &o->src[s];
    while (S->heap_n && S->heap[0].e < horizon) {
        item it = heap_pop(S);
        uint64_t d = it.e > S->tat ? it.e : S->tat;
        uint64_t floor_ = it.e > S->burst_ns ? it.e - S->burst_ns : 0;
        uint64_t base = S->tat > floor_ ? S->tat : floor_;
        S->tat = base + (((uint64_t)it.len * S->mult) >> S->shift);
        S->ring[(S->ring_head + S->ring_n) % HCAP] = d;
        S->ring_n++;
        if (it.dst == DEAD_DST) { /* leaves the sender, finds no port */
            o->st.lost_in_flight++;
            continue;
        }
        o->step_out = (tgsim_delivery*)grow(o->step_out, &o->cap_step, o->n_step + 1, sizeof(tgsim_delivery));
        tgsim_delivery* r = &o->step_out[o->n_step++];
        r->t_ns = d;
        r->src = o->o.shard_begin + s;
        r->dst = it.dst;
        r->seq = it.seq;
        r->len = it.len;
        r->flags = it.flags;
        o->st.scheduled++;
        o->st.bytes_scheduled += it.len;
        if (it.flags & TGSIM_FLAG_CORRUPT) o->st.corrupted++;
    }
}

static uint32_t crandom(uint32_t raw, uint32_t rho, uint32_t* last) { /* get_crandom */
    if (rho == 0) return raw;
    uint64_t r = (uint64_t)rho + 1;
    uint32_t a = (uint32_t)(((uint64_t)raw * ((1ull << 32) - r) + (uint64_t)(*last) * r) >> 32);
    *last = a;
    return a;
}

/* netem_enqueue from the queue-limit check on (dup/loss/corrupt already decided). */
static int enqueue(oracle* o, uint32_t s, uint64_t T, const tgsim_pkt* k, uint32_t reo_raw,
                   const uint32_t ctr_delay[4], int delay_word, uint16_t flags) {
    source* S = &o->src[s];
    htb_until(o, s, T);
    while (S->ring_n && S->ring[S->ring_head] < T) {
        S->ring_head = (S->ring_head + 1) % HCAP;
        S->ring_n--;
    }
    if (S->heap_n + S->ring_n >= o->o.queue_limit) return TGSIM_V_QUEUE_FULL;
    uint64_t e;
    int reordered = 0;
    if (S->thr_reo) {
        uint32_t v = crandom(reo_raw, S->rho_reo, &S->last_reo);
        reordered = !(S->thr_reo < v);
    }
    if (reordered) {
        e = T;
    } else if (S->sigma == 0) {
        e = T + S->lat_ns;
    } else {
        uint32_t r[4];
        tgo_philox4x32_10(ctr_delay, o->key, r);
        uint32_t m = 2u * (uint32_t)S->sigma;
        int64_t delay = (int64_t)(r[delay_word] % m) + (int64_t)S->lat_ns - (int64_t)S->sigma;
        e = delay > 0 ? T + (uint64_t)delay : T;
    }
    item it;
    it.e = e; it.seq = k->seq; it.dst = k->dst; it.len = k->len; it.flags = flags;
    heap_push(S, it);
    (void)o;
    return TGSIM_V_SCHEDULED;
}

static uint32_t lpm(const source* S, uint32_t ip) {
    int best = -1;
    uint32_t act = TGSIM_ACCEPT;
    for (uint32_t i = 0; i < S->n_rules; ++i) {
        const rule* r = &S->rules[i];
        uint32_t mask = r->len ? 0xFFFFFFFFu << (32 - r->len) : 0;
        if ((ip & mask) == r->net && (int)r->len > best) {
            best = r->len;
            act = r->action;
        }
    }
    return act;
}

static uint8_t process(oracle* o, uint32_t s, uint64_t T, const tgsim_pkt* k) {
    source* S = &o->src[s];
    o->st.offered++;
    if (!o->enabled[k->src] || (k->dst != TGSIM_EXTERNAL && !o->enabled[k->dst]))
        return 0xF0 | TGSIM_V_DISCONNECTED;
    if (k->dst == TGSIM_EXTERNAL) return 0xF0 | (S->allow_ext ? TGSIM_V_EXTERNAL : TGSIM_V_NO_ROUTE);
    if (S->n_rules) {
        uint32_t a = lpm(S, o->ip[k->dst]);
        if (a == TGSIM_DROP) return 0xF0 | TGSIM_V_BLACKHOLE;
        if (a == TGSIM_REJECT) return 0xF0 | TGSIM_V_PROHIBIT;
    }
    uint32_t c0[4] = {k->src, k->dst, k->seq, 0}, r0[4];
    tgo_philox4x32_10(c0, o->key, r0);
    int count = 1;
    if (S->thr_dup && S->thr_dup >= crandom(r0[0], S->rho_dup, &S->last_dup)) count++;
    if (S->thr_loss && S->thr_loss >= r0[1]) count--;
    if (count == 0) return 0xF0 | TGSIM_V_LOSS;
    uint8_t cv = TGSIM_V_NONE;
    if (count == 2) { /* clone re-enters the root qdisc with duplicate = 0 */
        o->st.cloned++;
        uint32_t c2[4] = {k->src, k->dst, k->seq, 2}, r2[4];
        tgo_philox4x32_10(c2, o->key, r2);
        if (S->thr_loss && S->thr_loss >= r2[0]) {
            cv = TGSIM_V_LOSS;
        } else {
            uint16_t fl = TGSIM_FLAG_DUP;
            if (S->thr_cor && S->thr_cor >= crandom(r2[1], S->rho_cor, &S->last_cor)) fl |= TGSIM_FLAG_CORRUPT;
            cv = (uint8_t)enqueue(o, s, T, k, r2[2], c2, 3, fl);
        }
    }
    uint16_t fl = 0;
    if (S->thr_cor && S->thr_cor >= crandom(r0[2], S->rho_cor, &S->last_cor)) fl |= TGSIM_FLAG_CORRUPT;
    uint32_t c1[4] = {k->src, k->dst, k->seq, 1};
    uint8_t ov = (uint8_t)enqueue(o, s, T, k, r0[3], c1, 0, fl);
    return (uint8_t)((cv << 4) | ov);
}

static int cmp_off(const void* a, const void* b) {
    const offered* x = (const offered*)a;
    const offered* y = (const offered*)b;
    if (x->p.src != y->p.src) return x->p.src < y->p.src ? -1 : 1;
    if (x->p.tick != y->p.tick) return x->p.tick < y->p.tick ? -1 : 1;
    if (x->p.seq != y->p.seq) return x->p.seq < y->p.seq ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

static int cmp_del(const void* a, const void* b) {
    const tgsim_delivery* x = (const tgsim_delivery*)a;
    const tgsim_delivery* y = (const tgsim_delivery*)b;
    if (x->dst != y->dst) return x->dst < y->dst ? -1 : 1;
    if (x->t_ns != y->t_ns) return x->t_ns < y->t_ns ? -1 : 1;
    if (x->src != y->src) return x->src < y->src ? -1 : 1;
    if (x->seq != y->seq) return x->seq < y->seq ? -1 : 1;
    int xd = (x->flags & TGSIM_FLAG_DUP) != 0, yd = (y->flags & TGSIM_FLAG_DUP) != 0;
    return yd - xd; /* clone first */
}

/* Runs the window's offered packets through filter -> netem -> HTB; leaves the scheduled records
 * of the step (unsorted) in o->step_out. */
static uint64_t queue_bytes(const oracle* o) {
    uint64_t b = 0;
    for (uint32_t s = 0; s < o->nsrc; ++s) b += 16ull * o->src[s].heap_n + 8ull * o->src[s].ring_n;
    return b;
}

/* Histogram bin of x: 0 for none, b for 2^(b-1) <= x < 2^b (include/tgsim.h TGSIM_METRICS_HIST). */
static uint32_t log2_bin(uint64_t x) {
    uint32_t b = 0;
    while (x) { b++; x >>= 1; }
    return b < TGSIM_METRICS_BINS ? b : TGSIM_METRICS_BINS - 1;
}

/* Per source after a step: offered packets/bytes and verdicts of the step's input, the HTB
 * records it served, and the backlog histogram (K8 metrics, include/tgsim.h). */
static void metrics_step(oracle* o) {
    for (size_t i = 0; i < o->n_off; ++i) {
        const tgsim_pkt* k = &o->off[i].p;
        uint64_t* row = o->m_src + (size_t)(k->src - o->o.shard_begin) * TGSIM_METRICS_SRC_WORDS;
        uint8_t v = o->verdicts[o->off[i].idx];
        row[0]++;
        row[1] += k->len;
        row[2 + (v & 15)]++;
        if ((v >> 4) < 8) row[2 + (v >> 4)]++;
    }
    for (size_t i = 0; i < o->n_step; ++i) {
        uint64_t* row = o->m_src + (size_t)(o->step_out[i].src - o->o.shard_begin) * TGSIM_METRICS_SRC_WORDS;
        row[10]++;
        row[11] += o->step_out[i].len;
    }
    for (uint32_t s = 0; s < o->nsrc; ++s) o->m_hist[log2_bin((uint64_t)o->src[s].heap_n + o->src[s].ring_n)]++;
}

int64_t tgo_metrics(void* p, uint32_t kind, uint64_t* out, size_t cap) {
    oracle* o = (oracle*)p;
    if (!o || (!out && cap) || kind > TGSIM_METRICS_HIST) return -EINVAL;
    if (!o->metrics_on) return fail(o, -ENODATA, "engine created without TGSIM_OPT_METRICS");
    const uint64_t* b = kind == TGSIM_METRICS_SRC ? o->m_src : kind == TGSIM_METRICS_DST ? o->m_dst : o->m_hist;
    size_t n = kind == TGSIM_METRICS_SRC   ? (size_t)o->nsrc * TGSIM_METRICS_SRC_WORDS
               : kind == TGSIM_METRICS_DST ? (size_t)o->nsrc * TGSIM_METRICS_DST_WORDS
                                           : 2 * TGSIM_METRICS_BINS;
    if (cap && n) memcpy(out, b, sizeof(uint64_t) * (cap < n ? cap : n));
    return (int64_t)n;
}

static int step_core(oracle* o, uint32_t n_ticks) {
    if (n_ticks == 0) return -EINVAL;
    if (o->gq_n) { /* the oldest generated window is this step's input */
        if (o->n_off) return fail(o, -EBUSY, "host packets and generated traffic in one step");
        if (o->gq[0].late) return gen_report_late(o, 0);
        if (o->gq[0].ticks != n_ticks)
            return fail(o, -EINVAL, "generated window spans %u ticks, step is %u", o->gq[0].ticks, n_ticks);
        free(o->off);
        o->off = o->gq[0].pk;
        o->n_off = o->gq[0].n;
        o->cap_off = o->gq[0].cap;
        o->gq_ticks -= n_ticks;
        if (o->gq_n > 1) memmove(o->gq, o->gq + 1, (o->gq_n - 1) * sizeof *o->gq);
        o->gq_n--;
    }
    for (size_t i = 0; i < o->n_off; ++i)
        if (o->off[i].p.tick >= n_ticks)
            return fail(o, -EINVAL, "packet %zu: tick %u beyond step of %u ticks", i, o->off[i].p.tick, n_ticks);
    if (o->n_off) qsort(o->off, o->n_off, sizeof(offered), cmp_off);
    o->st.queue_state_bytes += queue_bytes(o);
    free(o->verdicts);
    o->verdicts = (uint8_t*)malloc(o->n_off ? o->n_off : 1);
    o->n_verdicts = o->n_off;
    o->n_step = 0;
    uint64_t T0 = o->now_tick * o->o.tick_ns;
    for (size_t i = 0; i < o->n_off; ++i) {
        const tgsim_pkt* k = &o->off[i].p;
        uint32_t s = k->src - o->o.shard_begin;
        uint64_t T = T0 + (uint64_t)k->tick * o->o.tick_ns;
        uint8_t v = process(o, s, T, k);
        o->verdicts[o->off[i].idx] = v;
        o->st.by_verdict[v & 15]++;
        if ((v >> 4) != TGSIM_V_NONE) o->st.by_verdict[v >> 4]++;
    }
    uint64_t T1 = (o->now_tick + n_ticks) * o->o.tick_ns;
    for (uint32_t s = 0; s < o->nsrc; ++s) htb_until(o, s, T1 + o->o.lookahead_ns);
    o->st.queue_state_bytes += queue_bytes(o);
    if (o->metrics_on) metrics_step(o);
    o->n_off = 0;
    o->now_tick += n_ticks;
    o->st.now_tick = o->now_tick;
    return 0;
}

/* Sorts records into delivery order and appends them to the drain queue. */
static void gossip_receive(oracle* o, const tgsim_delivery* recs, size_t n);

static void deliver_records(oracle* o, const tgsim_delivery* recs, size_t n) {
    if (o->gossip_on) gossip_receive(o, recs, n);
    if (o->metrics_on) { /* per destination of this shard: records and bytes, histogram of counts */
        uint64_t* cnt = (uint64_t*)calloc(o->nsrc, sizeof(uint64_t));
        for (size_t i = 0; i < n; ++i) {
            uint32_t d = recs[i].dst - o->o.shard_begin;
            cnt[d]++;
            o->m_dst[(size_t)d * TGSIM_METRICS_DST_WORDS + 1] += recs[i].len;
        }
        for (uint32_t d = 0; d < o->nsrc; ++d) {
            o->m_dst[(size_t)d * TGSIM_METRICS_DST_WORDS] += cnt[d];
            o->m_hist[TGSIM_METRICS_BINS + log2_bin(cnt[d])]++;
        }
        free(cnt);
    }
    o->out = (tgsim_delivery*)grow(o->out, &o->cap_out, o->n_out + n, sizeof(tgsim_delivery));
    if (n) { /* (UBSan: no null pointers into memcpy/qsort, even for zero records) */
        memcpy(o->out + o->n_out, recs, n * sizeof(tgsim_delivery));
        qsort(o->out + o->n_out, n, sizeof(tgsim_delivery), cmp_del);
    }
    o->n_out += n;
}

int tgo_step(void* p, uint32_t n_ticks) {
    oracle* o = (oracle*)p;
    if (!o) return -EINVAL;
    if (o->pend_n) return fail(o, -EBUSY, "launched steps are not finished yet");
    int rc = step_core(o, n_ticks);
    if (rc) return rc;
    deliver_records(o, o->step_out, o->n_step);
    return 0;
}

/* tgsim_step_n (include/tgsim.h): n_steps windows in order; the engine fuses them into launches,
 * which changes no result, so the golden model simply steps n times. */
int tgo_step_n(void* p, uint32_t n_ticks, uint32_t n_steps) {
    for (uint32_t i = 0; i < n_steps; ++i) {
        int rc = tgo_step(p, n_ticks);
        if (rc) return rc;
    }
    return 0;
}

/* Multi-shard form: scheduled records grouped by the destination's shard into `out` (host
 * memory here), counts per shard in `counts`. */
static int step_sim_core(oracle* o, uint32_t n_ticks, uint32_t n_ranks, const uint32_t* bounds, void* out,
                         size_t cap, uint64_t* counts) {
    if (!o || !n_ranks || n_ranks > 8 || !bounds || !counts) return -EINVAL;
    if (bounds[0] != 0 || bounds[n_ranks] != o->o.n_peers) return fail(o, -EINVAL, "rank bounds must cover [0, n_peers)");
    int rc = step_core(o, n_ticks);
    if (rc) return rc;
    if (o->n_step > cap) return fail(o, -ENOSPC, "step_sim: %zu records exceed capacity %zu", o->n_step, cap);
    tgsim_delivery* dst = (tgsim_delivery*)out;
    size_t w = 0;
    for (uint32_t r = 0; r < n_ranks; ++r) {
        counts[r] = 0;
        for (size_t i = 0; i < o->n_step; ++i)
            if (o->step_out[i].dst >= bounds[r] && o->step_out[i].dst < bounds[r + 1]) {
                dst[w++] = o->step_out[i];
                counts[r]++;
            }
    }
    return 0;
}

int tgo_step_sim(void* p, uint32_t n_ticks, uint32_t n_ranks, const uint32_t* bounds, void* out,
                 size_t cap, uint64_t* counts) {
    oracle* o = (oracle*)p;
    if (o && o->pend_n) return fail(o, -EBUSY, "launched steps are not finished yet");
    return step_sim_core(o, n_ticks, n_ranks, bounds, out, cap, counts);
}

/* Split form (up to two launched steps pending): the oracle runs the whole step at launch and
 * keeps its counts for the matching finish. */
int tgo_step_sim_launch(void* p, uint32_t n_ticks, uint32_t n_ranks, const uint32_t* bounds, void* out,
                        size_t cap) {
    oracle* o = (oracle*)p;
    if (!o) return -EINVAL;
    if (o->pend_n == 2) return fail(o, -EBUSY, "two launched steps are not finished yet");
    const uint32_t k = (o->pend_head + o->pend_n) % 2;
    int rc = step_sim_core(o, n_ticks, n_ranks, bounds, out, cap, o->pend_counts[k]);
    if (rc) return rc;
    o->pend_ranks[k] = n_ranks;
    o->pend_n++;
    return 0;
}

int tgo_step_sim_finish(void* p, uint64_t* counts) {
    oracle* o = (oracle*)p;
    if (!o || !counts || !o->pend_n) return -EINVAL;
    const uint32_t k = o->pend_head;
    o->pend_head = (k + 1) % 2;
    o->pend_n--;
    for (uint32_t r = 0; r < o->pend_ranks[k]; ++r) counts[r] = o->pend_counts[k][r];
    return 0;
}

int tgo_deliver(void* p, const void* in, size_t n) {
    oracle* o = (oracle*)p;
    if (!o || (!in && n)) return -EINVAL;
    const tgsim_delivery* r = (const tgsim_delivery*)in;
    for (size_t i = 0; i < n; ++i)
        if (r[i].dst < o->o.shard_begin || r[i].dst >= o->o.shard_end)
            return fail(o, -EINVAL, "deliver: record %zu addresses dst %u outside this shard", i, r[i].dst);
    deliver_records(o, r, n);
    return 0;
}

/* Host memory, synchronous: the asynchronous forms of the engine are plain calls here. */
int tgo_deliver_async(void* p, const void* in, size_t n, void* wait_event) {
    (void)wait_event;
    return tgo_deliver(p, in, n);
}

int tgo_wait_event(void* p, void* event) {
    (void)event;
    return p ? 0 : -EINVAL;
}

int tgo_sync(void* p) { return p ? 0 : -EINVAL; }

int64_t tgo_sim_capacity(void* p) {
    oracle* o = (oracle*)p;
    if (o->gq_n && o->gq[0].late) return gen_report_late(o, 0);
    const size_t n = o->gq_n ? o->gq[0].n : o->n_off;
    return (int64_t)(2 * n + 1024ull * o->nsrc);
}

int64_t tgo_pending_deliveries(void* p) {
    oracle* o = (oracle*)p;
    return (int64_t)(o->n_out - o->out_head);
}

int64_t tgo_drain(void* p, tgsim_delivery* out, size_t cap) {
    oracle* o = (oracle*)p;
    size_t avail = o->n_out - o->out_head;
    size_t n = avail < cap ? avail : cap;
    if (n) memcpy(out, o->out + o->out_head, n * sizeof(tgsim_delivery));
    o->out_head += n;
    if (o->out_head == o->n_out) o->out_head = o->n_out = 0;
    return (int64_t)n;
}

int64_t tgo_verdicts(void* p, uint8_t* out, size_t cap) {
    oracle* o = (oracle*)p;
    size_t n = o->n_verdicts < cap ? o->n_verdicts : cap;
    if (n) memcpy(out, o->verdicts, n);
    return (int64_t)o->n_verdicts;
}

int tgo_stats(void* p, tgsim_stats_t* out) {
    *out = ((oracle*)p)->st;
    return 0;
}

int64_t tgo_signal(void* p, uint32_t state, uint32_t n) {
    oracle* o = (oracle*)p;
    if (!o || state >= TGSIM_SYNC_STATES) return -EINVAL;
    o->counters[state] += n;
    return (int64_t)o->counters[state];
}

int tgo_signal_async(void* p, uint32_t state, uint32_t n) {
    int64_t v = tgo_signal(p, state, n);
    return v < 0 ? (int)v : 0;
}

int tgo_barrier_poll(void* p, uint32_t state, uint64_t target) {
    oracle* o = (oracle*)p;
    if (!o || state >= TGSIM_SYNC_STATES) return -EINVAL;
    return o->counters[state] >= target;
}

/* Host memory here: the table the sharded barrier sums over the ranks. */
int tgo_sync_counters(void* p, void** table, uint32_t* n_states, void* event) {
    oracle* o = (oracle*)p;
    (void)event;
    if (!o || !table || !n_states) return -EINVAL;
    *table = o->counters;
    *n_states = TGSIM_SYNC_STATES;
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Gossip flood workload (include/tgsim.h tgsim_gossip).  A peer forwards flood
 * f once, at the tick after its earliest receipt, to its `degree` hashed out-neighbours. */
static uint32_t gossip_hash(const oracle* o, uint32_t a, uint32_t b, uint32_t tag) {
    uint32_t gk[2] = {o->key[0] ^ 0x3C6EF372u, o->key[1] ^ 0xA54FF53Au};
    uint32_t ctr[4] = {a, b, tag, 0}, r[4];
    tgo_philox4x32_10(ctr, gk, r);
    return r[0];
}

static uint32_t gossip_neighbour(const oracle* o, uint32_t peer, uint32_t k) {
    uint32_t N = o->o.n_peers;
    uint32_t d = gossip_hash(o, peer, k, 0x474F5350u) % (N - 1);
    return d >= peer ? d + 1 : d;
}

int tgo_gossip_init(void* p, const tgsim_gossip* g) {
    oracle* o = (oracle*)p;
    if (!o || !g || g->n_floods == 0 || g->n_floods > 64 || g->degree == 0 || g->degree > 64 ||
        g->msg_len == 0 || g->msg_len > 65535 || o->o.n_peers < 2)
        return -EINVAL;
    if (g->start_tick < o->now_tick) return fail(o, -EINVAL, "gossip: start tick in the past");
    o->g = *g;
    free(o->g_first);
    free(o->g_fwd);
    o->g_first = (uint32_t*)malloc(sizeof(uint32_t) * 64 * o->nsrc);
    o->g_fwd = (uint64_t*)calloc(o->nsrc, sizeof(uint64_t));
    for (size_t i = 0; i < 64ull * o->nsrc; ++i) o->g_first[i] = 0xFFFFFFFFu;
    for (uint32_t f = 0; f < g->n_floods; ++f) {
        uint32_t origin = gossip_hash(o, f, 0, 0x4F524947u) % o->o.n_peers;
        if (origin < o->o.shard_begin || origin >= o->o.shard_end) continue;
        o->g_first[64ull * (origin - o->o.shard_begin) + f] = (uint32_t)(g->start_tick + (uint64_t)f * g->start_gap_ticks);
    }
    o->gossip_on = 1;
    o->gossip_late = 0;
    return 0;
}

static void gossip_receive(oracle* o, const tgsim_delivery* recs, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        const tgsim_delivery* r = &recs[i];
        uint32_t f = r->seq / o->g.degree;
        if (f >= o->g.n_floods || (r->flags & TGSIM_FLAG_CORRUPT)) continue;
        uint32_t s = r->dst - o->o.shard_begin;
        if (o->g_fwd[s] >> f & 1) continue;
        uint64_t t = r->t_ns / o->o.tick_ns + 1;
        if (t > 0xFFFFFFFEull) t = 0xFFFFFFFEull;
        if (t < o->g_first[64ull * s + f]) o->g_first[64ull * s + f] = (uint32_t)t;
    }
}

int tgo_gen_gossip(void* p, uint32_t n_ticks) {
    oracle* o = (oracle*)p;
    if (!o || !o->gossip_on || n_ticks == 0 || n_ticks > 65536) return -EINVAL;
    if (o->n_off) return fail(o, -EBUSY, "host packets already pending for the next step");
    if (o->gossip_late)
        return fail(o, -EINVAL, "gossip: a receipt preceded an earlier window (tgsim_gossip_init starts a new flood)");
    for (size_t i = 0; i < o->gq_n; ++i) /* a queued late window is reported first */
        if (o->gq[i].late) return gen_report_late(o, i);
    uint64_t A = o->now_tick + o->gq_ticks, B = A + n_ticks;
    /* A receipt before the window (lookahead shorter than the window) fails the flood before any
     * peer's forwarded set changes: the window is queued empty and marked late, and the call that
     * resolves it reports it (gen_report_late), as the HIP engine does (its generation runs ahead
     * of the host, so it learns of the late receipt only when it resolves the window's size). */
    for (uint32_t s = 0; s < o->nsrc; ++s)
        for (uint32_t f = 0; f < o->g.n_floods; ++f) {
            uint32_t t = o->g_first[64ull * s + f];
            if (!(o->g_fwd[s] >> f & 1) && t < A) {
                struct genwin* lw = gen_window(o, n_ticks);
                lw->late = 1;
                lw->late_tick = t;
                lw->win0 = A;
                o->gq_ticks += n_ticks;
                return 0;
            }
        }
    struct genwin* w = gen_window(o, n_ticks);
    for (uint32_t s = 0; s < o->nsrc; ++s) {
        uint32_t src = o->o.shard_begin + s;
        for (;;) { /* floods due in the window, earliest receipt first, then by flood id */
            int best = -1;
            for (uint32_t f = 0; f < o->g.n_floods; ++f) {
                if (o->g_fwd[s] >> f & 1) continue;
                uint32_t t = o->g_first[64ull * s + f];
                if (t >= B) continue;
                if (best < 0 || t < o->g_first[64ull * s + (uint32_t)best]) best = (int)f;
            }
            if (best < 0) break;
            o->g_fwd[s] |= 1ull << best;
            uint32_t t = o->g_first[64ull * s + (uint32_t)best];
            for (uint32_t k = 0; k < o->g.degree; ++k) {
                tgsim_pkt pk;
                pk.src = src;
                pk.dst = gossip_neighbour(o, src, k);
                pk.seq = (uint32_t)best * o->g.degree + k;
                pk.len = (uint16_t)o->g.msg_len;
                pk.tick = (uint16_t)(t - A);
                gen_push(w, &pk);
            }
        }
    }
    o->gq_ticks += n_ticks;
    return 0;
}

int64_t tgo_gossip_reached(void* p, uint64_t* out, size_t cap) {
    oracle* o = (oracle*)p;
    if (!o || !o->gossip_on) return -EINVAL;
    for (uint32_t f = 0; f < o->g.n_floods && f < cap; ++f) {
        uint64_t c = 0;
        for (uint32_t s = 0; s < o->nsrc; ++s) c += o->g_fwd[s] >> f & 1;
        out[f] = c;
    }
    return o->g.n_floods;
}

/* Diagnostics (test infrastructure only): source s's departure ring (oldest first) and queued
 * items' eligibility times (heap order).  Returns ring_n << 32 | heap_n. */
int64_t tgo_debug_queue(void* p, uint32_t s, uint64_t* ring_d, uint64_t* item_e) {
    oracle* o = (oracle*)p;
    if (!o || s >= o->nsrc) return -EINVAL;
    const source* S = &o->src[s];
    for (uint32_t k = 0; k < S->ring_n; ++k) ring_d[k] = S->ring[(S->ring_head + k) % HCAP];
    for (uint32_t k = 0; k < S->heap_n; ++k) item_e[k] = S->heap[k].e;
    return ((int64_t)S->ring_n << 32) | S->heap_n;
}
