"""ctypes mirror of include/tgsim.h (plain C structs; no torch types cross the boundary)."""
from __future__ import annotations

import ctypes as C

import numpy as np

ABI_VERSION = 2
EXTERNAL = 0xFFFFFFFF

# enum tgsim_verdict
V_SCHEDULED, V_DISCONNECTED, V_NO_ROUTE, V_BLACKHOLE, V_PROHIBIT, V_LOSS, V_QUEUE_FULL, V_EXTERNAL = range(8)
V_NONE = 15
VERDICT_NAMES = ["scheduled", "disconnected", "no_route", "blackhole", "prohibit", "loss",
                 "queue_full", "external"]

FLAG_DUP = 0x1
FLAG_CORRUPT = 0x2

OPT_DISCARD_DELIVERIES = 0x2
OPT_METRICS = 0x4
OPT_K8S = 0x8           # K8sNetwork.ConfigureNetwork semantics (k8s_network.go:114-256)
SYNC_STATES = 65536     # K7 device sync counters
METRICS_SRC, METRICS_DST, METRICS_HIST = 0, 1, 2
METRICS_SRC_WORDS, METRICS_DST_WORDS, METRICS_BINS = 12, 2, 64
# columns of the per-instance source table (include/tgsim.h TGSIM_METRICS_SRC)
METRICS_SRC_COLUMNS = ["offered", "offered_bytes"] + [f"verdict_{i}" for i in range(8)] + ["served", "served_bytes"]


class Opts(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32),
        ("n_peers", C.c_uint32),
        ("shard_begin", C.c_uint32),
        ("shard_end", C.c_uint32),
        ("seed", C.c_uint64),
        ("tick_ns", C.c_uint64),
        ("queue_limit", C.c_uint32),
        ("flags", C.c_uint32),
        ("lookahead_ns", C.c_uint64),
        ("subnet_base", C.c_uint32),
        ("device", C.c_int32),
    ]


class Rule(C.Structure):
    _fields_ = [("prefix", C.c_uint32), ("len", C.c_uint8), ("action", C.c_uint8), ("_pad", C.c_uint16)]


class Shape(C.Structure):
    _fields_ = [
        ("latency_ns", C.c_int64),
        ("jitter_ns", C.c_int64),
        ("bandwidth_bps", C.c_uint64),
        ("loss", C.c_float),
        ("corrupt", C.c_float),
        ("corrupt_corr", C.c_float),
        ("reorder", C.c_float),
        ("reorder_corr", C.c_float),
        ("duplicate", C.c_float),
        ("duplicate_corr", C.c_float),
        ("_pad", C.c_uint32),
    ]


class Config(C.Structure):
    _fields_ = [
        ("network", C.c_char_p),
        ("enable", C.c_uint8),
        ("routing_policy", C.c_uint8),
        ("has_ipv4", C.c_uint8),
        ("has_ipv6", C.c_uint8),
        ("ipv4", C.c_uint32),
        ("shape", Shape),
        ("rules", C.POINTER(Rule)),
        ("n_rules", C.c_uint32),
        ("_pad2", C.c_uint32),
        ("ipv6", C.c_uint8 * 16),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("offered", C.c_uint64),
        ("scheduled", C.c_uint64),
        ("cloned", C.c_uint64),
        ("corrupted", C.c_uint64),
        ("by_verdict", C.c_uint64 * 8),
        ("bytes_scheduled", C.c_uint64),
        ("now_tick", C.c_uint64),
        ("queue_state_bytes", C.c_uint64),
        ("flushed", C.c_uint64),
        ("lost_in_flight", C.c_uint64),
    ]


class Gossip(C.Structure):
    _fields_ = [
        ("n_floods", C.c_uint32),
        ("degree", C.c_uint32),
        ("msg_len", C.c_uint32),
        ("start_gap_ticks", C.c_uint32),
        ("start_tick", C.c_uint64),
    ]


class CommInfo(C.Structure):
    _fields_ = [("rank", C.c_int32), ("nranks", C.c_int32), ("exchanged_records", C.c_uint64),
                ("max_rank_count", C.c_uint64), ("slot_cap", C.c_uint64), ("bounds", C.c_uint32 * 9),
                ("_pad", C.c_uint32)]


COMM_ID_BYTES = 128

PKT_DTYPE = np.dtype([("src", "<u4"), ("dst", "<u4"), ("seq", "<u4"), ("len", "<u2"), ("tick", "<u2")])
DELIVERY_DTYPE = np.dtype([("t_ns", "<u8"), ("src", "<u4"), ("dst", "<u4"), ("seq", "<u4"),
                           ("len", "<u2"), ("flags", "<u2")])
# tgsim_config as a numpy record (batch configuration without per-peer ctypes objects).
SHAPE_DTYPE = np.dtype([("latency_ns", "<i8"), ("jitter_ns", "<i8"), ("bandwidth_bps", "<u8"), ("loss", "<f4"),
                        ("corrupt", "<f4"), ("corrupt_corr", "<f4"), ("reorder", "<f4"), ("reorder_corr", "<f4"),
                        ("duplicate", "<f4"), ("duplicate_corr", "<f4"), ("_pad", "<u4")])
CONFIG_DTYPE = np.dtype([("network", "<u8"), ("enable", "u1"), ("routing_policy", "u1"), ("has_ipv4", "u1"),
                         ("has_ipv6", "u1"), ("ipv4", "<u4"), ("shape", SHAPE_DTYPE), ("rules", "<u8"),
                         ("n_rules", "<u4"), ("_pad2", "<u4"), ("ipv6", "u1", (16,))])
assert SHAPE_DTYPE.itemsize == 56 and CONFIG_DTYPE.itemsize == 104
assert PKT_DTYPE.itemsize == 16 and DELIVERY_DTYPE.itemsize == 24
assert C.sizeof(CommInfo) == 72 and C.sizeof(Gossip) == 24 and C.sizeof(Opts) == 56 and C.sizeof(Shape) == 56 and C.sizeof(Config) == 104

# Every symbol include/tgsim.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "tgsim_create", "tgsim_destroy", "tgsim_last_error", "tgsim_abi_version", "tgsim_configure",
    "tgsim_configure_batch", "tgsim_link_generation",
    "tgsim_submit", "tgsim_gen_storm", "tgsim_step", "tgsim_step_sim", "tgsim_deliver",
    "tgsim_deliver_async", "tgsim_wait_event", "tgsim_sync", "tgsim_step_sim_launch", "tgsim_step_sim_finish",
    "tgsim_step_sim_counts", "tgsim_delivery_event", "tgsim_step_sim_launch_slotted", "tgsim_step_sim_release",
    "tgsim_deliver_slotted_async", "tgsim_step_sim_launch_slotted_n", "tgsim_deliver_slotted_n_async",
    "tgsim_sim_capacity", "tgsim_drain", "tgsim_pending_deliveries", "tgsim_verdicts", "tgsim_stats",
    "tgsim_signal", "tgsim_signal_async", "tgsim_barrier_poll", "tgsim_sync_counters", "tgsim_sim_kernel_ms", "tgsim_delivery_kernel_ms", "tgsim_stream", "tgsim_debug_stamps",
    "tgsim_debug_fused_windows", "tgsim_debug_sparse_windows", "tgsim_debug_carry_bytes", "tgsim_debug_bucket_records", "tgsim_debug_exec_faults", "tgsim_step_n",
    "tgsim_gossip_init", "tgsim_gen_gossip", "tgsim_gossip_reached", "tgsim_metrics",
    "tgsim_comm_id", "tgsim_comm_init", "tgsim_comm_step", "tgsim_comm_launch", "tgsim_comm_finish", "tgsim_comm_run", "tgsim_comm_barrier", "tgsim_comm_info",
    "tgsim_bridge_create", "tgsim_bridge_destroy", "tgsim_bridge_send", "tgsim_bridge_step",
    "tgsim_bridge_recv", "tgsim_bridge_pending", "tgsim_bridge_in_flight", "tgsim_bridge_now_tick",
    "tgsim_bridge_link_removed",
    "tgsim_udp_front_create", "tgsim_udp_front_port", "tgsim_udp_front_register", "tgsim_udp_front_bind_peer",
    "tgsim_udp_front_pump", "tgsim_udp_front_destroy",
]


def declare(lib: C.CDLL, prefix: str) -> None:
    """Sets argtypes/restype for the engine-shaped API under `prefix` (tgsim_ or tgo_)."""
    vp = C.c_void_p

    def f(name, res, *args):
        fn = getattr(lib, prefix + name, None)
        if fn is None:
            return
        fn.restype = res
        fn.argtypes = list(args)

    f("create", C.c_int, C.POINTER(Opts), C.POINTER(vp))
    f("destroy", None, vp)
    f("last_error", C.c_char_p, vp)
    f("configure", C.c_int, vp, C.c_uint32, C.POINTER(Config))
    f("configure_batch", C.c_int64, vp, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)
    f("link_generation", C.c_int64, vp, C.c_uint32)
    f("submit", C.c_int, vp, C.c_void_p, C.c_size_t)
    f("gen_storm", C.c_int, vp, C.c_double, C.c_uint32)
    f("step", C.c_int, vp, C.c_uint32)
    f("step_n", C.c_int, vp, C.c_uint32, C.c_uint32)
    f("step_sim", C.c_int, vp, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), vp, C.c_size_t,
      C.POINTER(C.c_uint64))
    f("step_sim_launch", C.c_int, vp, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), vp, C.c_size_t)
    f("step_sim_finish", C.c_int, vp, C.POINTER(C.c_uint64))
    f("step_sim_counts", C.c_int, vp, C.POINTER(C.c_uint64))
    f("delivery_event", C.c_int, vp, vp)
    f("step_sim_launch_slotted", C.c_int, vp, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), vp, C.c_uint64, vp)
    f("step_sim_release", C.c_int, vp)
    f("step_sim_launch_slotted_n", C.c_int, vp, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), vp,
      C.c_uint64, vp)
    f("deliver_slotted_n_async", C.c_int, vp, vp, C.c_uint32, C.c_uint32, C.c_uint64, vp)
    f("deliver_slotted_async", C.c_int, vp, vp, C.c_uint32, C.c_uint64, vp)
    f("deliver", C.c_int, vp, vp, C.c_size_t)
    f("deliver_async", C.c_int, vp, vp, C.c_size_t, vp)
    f("wait_event", C.c_int, vp, vp)
    f("sync", C.c_int, vp)
    f("sim_capacity", C.c_int64, vp)
    f("drain", C.c_int64, vp, C.c_void_p, C.c_size_t)
    f("pending_deliveries", C.c_int64, vp)
    f("verdicts", C.c_int64, vp, C.c_void_p, C.c_size_t)
    f("stats", C.c_int, vp, C.POINTER(Stats))
    f("signal", C.c_int64, vp, C.c_uint32, C.c_uint32)
    f("barrier_poll", C.c_int, vp, C.c_uint32, C.c_uint64)
    f("signal_async", C.c_int, vp, C.c_uint32, C.c_uint32)
    f("sync_counters", C.c_int, vp, C.POINTER(vp), C.POINTER(C.c_uint32), vp)
    f("sim_kernel_ms", C.c_double, vp, C.POINTER(C.c_uint64), C.c_int)
    f("delivery_kernel_ms", C.c_double, vp, C.POINTER(C.c_uint64), C.c_int)
    f("stream", vp, vp)
    f("debug_stamps", C.c_int64, vp, C.c_void_p, C.c_size_t)
    f("debug_fused_windows", C.c_int64, vp)
    f("debug_sparse_windows", C.c_int64, vp)
    f("debug_exec_faults", C.c_int64)
    f("debug_carry_bytes", C.c_int64, vp)
    f("debug_bucket_records", C.c_int64, vp)
    f("abi_version", C.c_uint32)
    f("gossip_init", C.c_int, vp, C.POINTER(Gossip))
    f("gen_gossip", C.c_int, vp, C.c_uint32)
    f("gossip_reached", C.c_int64, vp, C.c_void_p, C.c_size_t)
    f("offered", C.c_int64, vp, C.c_void_p, C.c_size_t)
    f("metrics", C.c_int64, vp, C.c_uint32, C.c_void_p, C.c_size_t)
    f("comm_id", C.c_int, vp)
    f("comm_init", C.c_int, vp, vp, C.c_int, C.c_int)
    f("comm_step", C.c_int, vp, C.c_uint32)
    f("comm_launch", C.c_int, vp, C.c_uint32)
    f("comm_finish", C.c_int, vp)
    f("comm_run", C.c_int, vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64)
    f("comm_barrier", C.c_int, vp, C.c_uint32, C.c_uint64)
    f("comm_info", C.c_int, vp, C.POINTER(CommInfo))
