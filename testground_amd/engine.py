"""Python handle over the engine's C ABI (include/tgsim.h).

``Engine`` always drives the HIP library ``libtgsim.so``; it raises ``EngineUnavailable`` when the
library or a GPU is missing — there is no CPU fallback in the product path.  ``CABIEngine`` is the
generic wrapper over any library exporting the same function set under a prefix (the tests use it
to drive the CPU oracle with identical inputs).
"""
from __future__ import annotations

import ctypes as C
import errno
import os
from pathlib import Path
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .network import Config, to_c

PKG = Path(__file__).resolve().parent
LIB_PATH = PKG / "libtgsim.so"


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{msg} (errno {-code}: {errno.errorcode.get(-code, '?')})")
        self.code = code
        self.msg = msg


class EngineUnavailable(EngineError):
    pass


_LIB: Optional[C.CDLL] = None


def load_library(path: Optional[Path] = None) -> C.CDLL:
    """Loads libtgsim.so (in-tree).  Fails loudly if it has not been built."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = Path(path or os.environ.get("TGSIM_LIB", LIB_PATH))
    if not p.exists():
        raise EngineUnavailable(-errno.ENOENT, f"HIP engine library not built: {p} (run __graft_entry__.build())")
    lib = C.CDLL(str(p))
    abi.declare(lib, "tgsim_")
    if lib.tgsim_abi_version() != abi.ABI_VERSION:
        raise EngineUnavailable(-errno.EPROTO, "libtgsim ABI version mismatch")
    if path is None:
        _LIB = lib
    return lib


class CABIEngine:
    """Engine-shaped C ABI wrapper (prefix 'tgsim_' for the product, 'tgo_' for the oracle)."""

    def __init__(self, lib: C.CDLL, prefix: str, n_peers: int, seed: int = 0x7E576A0D00000001,
                 tick_ns: int = 1000, queue_limit: int = 0, shard: Tuple[int, int] = (0, 0),
                 lookahead_ns: int = 0, flags: int = 0, subnet_base: int = 0, device: int = -1):
        self._lib = lib
        self._p = prefix
        o = abi.Opts()
        o.abi_version = abi.ABI_VERSION
        o.n_peers = n_peers
        o.shard_begin, o.shard_end = shard
        o.seed = seed & 0xFFFFFFFFFFFFFFFF
        o.tick_ns = tick_ns
        o.queue_limit = queue_limit
        o.flags = flags
        o.lookahead_ns = lookahead_ns
        o.subnet_base = subnet_base
        o.device = device
        self.n_peers = n_peers
        self.subnet_base = subnet_base or (16 << 24)  # the engine's default data network, 16.0.0.0
        self.shard = (shard[0], shard[1] if shard[1] else n_peers) if shard != (0, 0) else (0, n_peers)
        self.tick_ns = tick_ns
        h = C.c_void_p()
        rc = self._fn("create")(C.byref(o), C.byref(h))
        if rc != 0:
            exc = EngineUnavailable if rc in (-errno.ENODEV, -errno.EPROTO) else EngineError
            raise exc(rc, f"{prefix}create failed")
        self._h = h
        self._launched: list = []  # rank counts of launched, unfinished steps (step_sim_launch)

    def _fn(self, name):
        return getattr(self._lib, self._p + name)

    def _check(self, rc: int, what: str) -> int:
        if rc < 0:
            msg = self._fn("last_error")(self._h)
            raise EngineError(rc, f"{what}: {msg.decode() if msg else ''}")
        return rc

    # -- lifecycle -----------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._fn("destroy")(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- configuration -------------------------------------------------------------------------
    def configure(self, peer: int, cfg: Config) -> None:
        c, keep = to_c(cfg)
        self._check(self._fn("configure")(self._h, peer, C.byref(c)), f"configure peer {peer}")
        del keep

    def configure_batch(self, peers: np.ndarray, cfgs: np.ndarray) -> None:
        """Batch of ConfigureNetwork calls; cfgs is an abi.CONFIG_DTYPE array whose `network`
        pointers reference live buffers (see network.configs_array)."""
        peers = np.ascontiguousarray(peers, dtype=np.uint32)
        cfgs = np.ascontiguousarray(cfgs, dtype=abi.CONFIG_DTYPE)
        if len(peers) != len(cfgs):
            raise ValueError("peers and cfgs differ in length")
        rcs = np.zeros(len(peers), dtype=np.int32)
        failed = self._fn("configure_batch")(self._h, peers.ctypes.data, cfgs.ctypes.data, len(peers),
                                             rcs.ctypes.data)
        if failed:
            i = int(np.nonzero(rcs)[0][0])
            self._check(int(rcs[i]), f"configure_batch: peer {int(peers[i])} (and {failed - 1} more)")

    def link_generation(self, peer: int) -> int:
        """How many times peer's data link has been removed (disconnect or re-addressing)."""
        return self._check(self._fn("link_generation")(self._h, peer), "link_generation")

    # -- data path -----------------------------------------------------------------------------
    def submit(self, pkts: np.ndarray) -> None:
        pkts = np.ascontiguousarray(pkts, dtype=abi.PKT_DTYPE)
        self._check(self._fn("submit")(self._h, pkts.ctypes.data, len(pkts)), "submit")

    def gen_storm(self, lam: float, n_ticks: int) -> None:
        self._check(self._fn("gen_storm")(self._h, float(lam), n_ticks), "gen_storm")

    def gossip_init(self, n_floods: int = 64, degree: int = 8, msg_len: int = 1024, start_gap_ticks: int = 0,
                    start_tick: Optional[int] = None) -> None:
        g = abi.Gossip(n_floods, degree, msg_len, start_gap_ticks, self.stats()["now_tick"] if start_tick is None
                       else start_tick)
        self._check(self._fn("gossip_init")(self._h, C.byref(g)), "gossip_init")
        self.n_floods = n_floods

    def gen_gossip(self, n_ticks: int) -> None:
        self._check(self._fn("gen_gossip")(self._h, n_ticks), "gen_gossip")

    def gossip_reached(self) -> np.ndarray:
        out = np.zeros(64, dtype=np.uint64)
        n = self._check(self._fn("gossip_reached")(self._h, out.ctypes.data, 64), "gossip_reached")
        return out[:n]

    def step(self, n_ticks: int) -> None:
        self._check(self._fn("step")(self._h, n_ticks), "step")

    def step_n(self, n_ticks: int, n_steps: int) -> None:
        """n_steps windows of n_ticks (tgsim_step_n: generated windows run fused, up to eight per launch)."""
        self._check(self._fn("step_n")(self._h, n_ticks, n_steps), "step_n")

    def step_sim(self, n_ticks: int, bounds: Sequence[int], d_out: int, out_cap: int) -> np.ndarray:
        nr = len(bounds) - 1
        b = (C.c_uint32 * len(bounds))(*bounds)
        counts = (C.c_uint64 * nr)()
        self._check(self._fn("step_sim")(self._h, n_ticks, nr, b, C.c_void_p(d_out), out_cap, counts), "step_sim")
        return np.array(list(counts), dtype=np.uint64)

    def step_sim_launch(self, n_ticks: int, bounds: Sequence[int], d_out: int, out_cap: int) -> None:
        """First half of step_sim: the step runs on the engine stream; step_sim_finish waits for
        it and returns the per-rank counts. The host may enqueue other work (and one more launched
        step) in between."""
        nr = len(bounds) - 1
        b = (C.c_uint32 * len(bounds))(*bounds)
        self._check(self._fn("step_sim_launch")(self._h, n_ticks, nr, b, C.c_void_p(d_out), out_cap),
                    "step_sim_launch")
        self._launched.append(nr)

    def step_sim_finish(self) -> np.ndarray:
        """Counts of the oldest launched step (up to two may be pending)."""
        counts = (C.c_uint64 * self._launched.pop(0))()
        self._check(self._fn("step_sim_finish")(self._h, counts), "step_sim_finish")
        return np.array(list(counts), dtype=np.uint64)

    def step_sim_counts(self) -> np.ndarray:
        """step_sim_finish without waiting for earlier asynchronous deliveries (the caller orders
        the reuse of their input buffers with delivery_event)."""
        counts = (C.c_uint64 * self._launched.pop(0))()
        self._check(self._fn("step_sim_counts")(self._h, counts), "step_sim_counts")
        return np.array(list(counts), dtype=np.uint64)

    def step_sim_launch_slotted(self, n_ticks: int, bounds: Sequence[int], d_out: int, slot_cap: int,
                                routed_event: int = 0) -> None:
        """Slotted pipelined step: records for rank r go to chunk r of (slot_cap + 1) records in
        d_out, after a count header; routed_event is recorded when d_out is complete."""
        b = (C.c_uint32 * len(bounds))(*bounds)
        self._check(self._fn("step_sim_launch_slotted")(self._h, n_ticks, len(bounds) - 1, b, C.c_void_p(d_out),
                                                         slot_cap, C.c_void_p(routed_event or None)),
                    "step_sim_launch_slotted")

    def step_sim_release(self) -> None:
        """Retires the oldest launched slotted step without waiting for it."""
        self._check(self._fn("step_sim_release")(self._h), "step_sim_release")

    def step_sim_launch_slotted_n(self, n_ticks: int, n_win: int, bounds: Sequence[int], d_out: int, slot_cap: int,
                                  routed_event: int = 0) -> None:
        """Fused slotted group: n_win generated windows in one launch; d_out holds n_ranks x n_win
        chunks of (slot_cap + 1) records (rank-major), one launched step for step_sim_release."""
        b = (C.c_uint32 * len(bounds))(*bounds)
        self._check(self._fn("step_sim_launch_slotted_n")(self._h, n_ticks, n_win, len(bounds) - 1, b,
                                                           C.c_void_p(d_out), slot_cap,
                                                           C.c_void_p(routed_event or None)),
                    "step_sim_launch_slotted_n")

    def deliver_slotted_n_async(self, d_in: int, n_ranks: int, n_win: int, slot_cap: int, wait_event: int = 0) -> None:
        self._check(self._fn("deliver_slotted_n_async")(self._h, C.c_void_p(d_in), n_ranks, n_win, slot_cap,
                                                         C.c_void_p(wait_event or None)), "deliver_slotted_n_async")

    def deliver_slotted_async(self, d_in: int, n_ranks: int, slot_cap: int, wait_event: int = 0) -> None:
        self._check(self._fn("deliver_slotted_async")(self._h, C.c_void_p(d_in), n_ranks, slot_cap,
                                                       C.c_void_p(wait_event or None)), "deliver_slotted_async")

    def delivery_event(self, event: int) -> None:
        """Records a raw hipEvent_t on the delivery stream after the deliveries enqueued so far."""
        self._check(self._fn("delivery_event")(self._h, C.c_void_p(event)), "delivery_event")

    def deliver(self, d_in: int, n: int) -> None:
        self._check(self._fn("deliver")(self._h, C.c_void_p(d_in), n), "deliver")

    def deliver_async(self, d_in: int, n: int, wait_event: int = 0) -> None:
        """Delivery enqueued on the engine's delivery stream after `wait_event` (a raw
        hipEvent_t, e.g. torch.cuda.Event().cuda_event); overlaps the next step_sim."""
        self._check(self._fn("deliver_async")(self._h, C.c_void_p(d_in), n, C.c_void_p(wait_event or None)),
                    "deliver_async")

    def wait_event(self, event: int) -> None:
        self._check(self._fn("wait_event")(self._h, C.c_void_p(event)), "wait_event")

    def sync(self) -> None:
        self._check(self._fn("sync")(self._h), "sync")

    def sim_capacity(self) -> int:
        return self._check(self._fn("sim_capacity")(self._h), "sim_capacity")

    def pending(self) -> int:
        return self._check(self._fn("pending_deliveries")(self._h), "pending")

    def drain(self) -> np.ndarray:
        n = self.pending() if hasattr(self._lib, self._p + "pending_deliveries") else None
        if n is None:  # oracle: ask with a large buffer
            out = np.empty(1 << 22, dtype=abi.DELIVERY_DTYPE)
            k = self._check(self._fn("drain")(self._h, out.ctypes.data, len(out)), "drain")
            return out[:k].copy()
        out = np.empty(n, dtype=abi.DELIVERY_DTYPE)
        k = self._check(self._fn("drain")(self._h, out.ctypes.data, n), "drain")
        return out[:k]

    def verdicts(self) -> np.ndarray:
        n = self._check(self._fn("verdicts")(self._h, None, 0), "verdicts")
        out = np.empty(n, dtype=np.uint8)
        if n:
            self._check(self._fn("verdicts")(self._h, out.ctypes.data, n), "verdicts")
        return out

    def metrics(self) -> dict:
        """K8 metrics tables accumulated since create (engine flag abi.OPT_METRICS): `src`
        [instances of this shard, 12] (columns abi.METRICS_SRC_COLUMNS), `dst` [instances, 2]
        (records, bytes delivered), `hist` [2, 64] (log2 bins of the per-step netem backlog and of
        the per-step records delivered, per instance)."""
        out = {}
        for kind, key, shape in ((abi.METRICS_SRC, "src", (-1, abi.METRICS_SRC_WORDS)),
                                 (abi.METRICS_DST, "dst", (-1, abi.METRICS_DST_WORDS)),
                                 (abi.METRICS_HIST, "hist", (2, abi.METRICS_BINS))):
            n = self._check(self._fn("metrics")(self._h, kind, None, 0), "metrics")
            a = np.zeros(n, dtype=np.uint64)
            self._check(self._fn("metrics")(self._h, kind, a.ctypes.data, n), "metrics")
            out[key] = a.reshape(shape)
        return out

    def stats(self) -> dict:
        s = abi.Stats()
        self._check(self._fn("stats")(self._h, C.byref(s)), "stats")
        d = {k: getattr(s, k) for k in ("offered", "scheduled", "cloned", "corrupted", "bytes_scheduled", "now_tick",
                                   "queue_state_bytes", "flushed", "lost_in_flight")}
        d["by_verdict"] = {abi.VERDICT_NAMES[i]: s.by_verdict[i] for i in range(8)}
        return d

    # -- sync counters -------------------------------------------------------------------------
    def signal(self, state: int, n: int = 1) -> int:
        return self._check(self._fn("signal")(self._h, state, n), "signal")

    def signal_async(self, state: int, n: int = 1) -> None:
        """signal() without waiting for the new value (K7 counters stay on the device)."""
        self._check(self._fn("signal_async")(self._h, state, n), "signal_async")

    def barrier_poll(self, state: int, target: int) -> bool:
        return bool(self._check(self._fn("barrier_poll")(self._h, state, target), "barrier_poll"))

    def sync_counters(self, event: int = 0) -> Tuple[int, int]:
        """(address, states) of the sync counter table (device memory on the HIP engine, host
        memory on the oracle); `event` (a raw hipEvent_t) is recorded after every issued signal."""
        ptr, n = C.c_void_p(), C.c_uint32()
        self._check(self._fn("sync_counters")(self._h, C.byref(ptr), C.byref(n), C.c_void_p(event or None)),
                    "sync_counters")
        return int(ptr.value or 0), int(n.value)

    # -- RCCL exchange owned by the engine (tgsim_comm_*) --------------------------------------------
    def comm_init(self, comm_id: bytes, rank: int, nranks: int) -> None:
        """Joins this engine to the run's exchange (collective; comm_id from comm_id() on one rank)."""
        buf = C.create_string_buffer(bytes(comm_id), abi.COMM_ID_BYTES)
        self._check(self._fn("comm_init")(self._h, buf, rank, nranks), "comm_init")

    def comm_step(self, n_ticks: int) -> None:
        self._check(self._fn("comm_step")(self._h, n_ticks), "comm_step")

    def comm_launch(self, n_ticks: int) -> None:
        self._check(self._fn("comm_launch")(self._h, n_ticks), "comm_launch")

    def comm_finish(self) -> None:
        self._check(self._fn("comm_finish")(self._h), "comm_finish")

    def comm_run(self, n_ticks: int, n_steps: int, fuse: int = 1, slot_cap: int = 0) -> None:
        self._check(self._fn("comm_run")(self._h, n_ticks, n_steps, fuse, slot_cap), "comm_run")

    def comm_barrier(self, state: int, target: int) -> bool:
        return bool(self._check(self._fn("comm_barrier")(self._h, state, target), "comm_barrier"))

    def comm_info(self) -> dict:
        i = abi.CommInfo()
        self._check(self._fn("comm_info")(self._h, C.byref(i)), "comm_info")
        return {"rank": i.rank, "nranks": i.nranks, "exchanged_records": i.exchanged_records,
                "max_rank_count": i.max_rank_count, "slot_cap": i.slot_cap, "bounds": list(i.bounds[:i.nranks + 1])}

    # -- instrumentation -----------------------------------------------------------------------
    def carry_bytes(self) -> int:
        """HBM bytes the simulate kernels moved carrying queues between windows (tgsim_debug_carry_bytes)."""
        if not hasattr(self._lib, self._p + "debug_carry_bytes"):  # an older library (A/B runs)
            return 0
        return self._check(self._fn("debug_carry_bytes")(self._h), "debug_carry_bytes")

    def bucket_records(self) -> int:
        """Records written straight into destination buckets (tgsim_debug_bucket_records)."""
        if not hasattr(self._lib, self._p + "debug_bucket_records"):  # an older library (A/B runs)
            return 0
        return self._check(self._fn("debug_bucket_records")(self._h), "debug_bucket_records")

    def sim_kernel_ms(self, reset: bool = False) -> Tuple[float, int]:
        n = C.c_uint64()
        ms = self._fn("sim_kernel_ms")(self._h, C.byref(n), 1 if reset else 0)
        return ms, n.value

    def delivery_kernel_ms(self, reset: bool = False) -> Tuple[float, int]:
        """Average delivery span (ms) per delivered window on the delivery stream (HIP events)."""
        n = C.c_uint64()
        ms = self._fn("delivery_kernel_ms")(self._h, C.byref(n), 1 if reset else 0)
        return ms, n.value


class Engine(CABIEngine):
    """The MI355X engine (libtgsim.so)."""

    def __init__(self, n_peers: int, **kw):
        super().__init__(load_library(), "tgsim_", n_peers, **kw)


def comm_id() -> bytes:
    """A fresh RCCL communicator id (tgsim_comm_id) for tgsim_comm_init; made on one rank and handed
    to the others by the host."""
    lib = load_library()
    buf = C.create_string_buffer(abi.COMM_ID_BYTES)
    rc = lib.tgsim_comm_id(buf)
    if rc:
        raise EngineError(rc, "tgsim_comm_id")
    return buf.raw


def packets(rows: Iterable[tuple]) -> np.ndarray:
    """Builds a packet array from (src, dst, seq, len, tick) tuples."""
    return np.array(list(rows), dtype=abi.PKT_DTYPE)
