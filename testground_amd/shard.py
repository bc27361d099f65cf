"""Peer-sharded stepping across ranks.

Shaping is egress-only and per source (pkg/sidecar/link.go:22-40), so every rank owns a
contiguous range of sources and computes their verdicts and delivery times locally.  The only
exchange is the hand-off of scheduled 24-B records to the destination's rank:

    simulate -> records grouped by destination shard
    exchange -> per-rank record counts, then the records (RCCL over xGMI on GPUs)
    deliver  -> per-destination delivery order on the receiving rank

On GPUs the engine does all of it itself (`CommStepper` over tgsim_comm_*: its own RCCL
communicator, exchange stream and buffers), so the Go host of INTEGRATION.md and this module make
the same calls.  `ShardedStepper` is the same exchange written with torch.distributed over the
engine's split-phase calls (tgsim_step_sim_launch / _deliver_async): the tests run it with CPU
oracle shards over `gloo`, as the restatement the engine's own exchange is checked against.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

REC = 24  # sizeof(tgsim_delivery)


def init_rccl(device: torch.device, **kw) -> None:
    """RCCL process group whose collectives run on a high-priority stream.  HIP maps streams onto a
    few hardware queues; the engine's simulate stream keeps the next steps' k_sim queued, so an
    exchange placed on the same queue would wait behind them.  High-priority streams (the
    exchange's, RCCL's and the engine's delivery stream) take a queue of their own."""
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    dist.init_process_group("nccl", pg_options=opts, device_id=device, **kw)


class _DevArray:
    """__cuda_array_interface__ view of engine-owned device memory (zero copy)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i8", "data": (ptr, False), "version": 2}


def device_table(ptr: int, n: int, device: torch.device) -> torch.Tensor:
    """The engine's K7 counter table (n u64 in device memory) as an int64 tensor, without a copy."""
    with torch.cuda.device(device):
        return torch.as_tensor(_DevArray(ptr, n), device=device)


def shard_bounds(n_peers: int, world: int) -> List[int]:
    """Contiguous source ranges, as even as possible: rank r owns [b[r], b[r+1])."""
    return [(n_peers * r) // world for r in range(world)] + [n_peers]


class CommStepper:
    """The engine's own exchange (tgsim_comm_*), with ShardedStepper's interface: step() is one
    closed-loop window (tgsim_comm_step), run() the pipelined slotted run (tgsim_comm_run),
    barrier() the device all-reduce of a sync counter (tgsim_comm_barrier).  The RCCL id is made
    on rank 0 and broadcast over the host's process group."""

    def __init__(self, engine, bounds: Sequence[int], device: str = "cuda", group=None,
                 slot_cap: Optional[int] = None):
        from .engine import comm_id
        self.engine = engine
        self.bounds = list(bounds)
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        ids = [comm_id() if rank == 0 else None]
        dist.broadcast_object_list(ids, src=0, group=group, device=torch.device(device))
        engine.comm_init(ids[0], rank, world)
        got = engine.comm_info()["bounds"]
        if got != self.bounds:
            raise ValueError(f"engine shards {got} differ from the stepper's bounds {self.bounds}")
        self.slot_cap = slot_cap
        self.world = world

    @property
    def max_count(self) -> int:
        return self.engine.comm_info()["max_rank_count"]

    @property
    def exchanged_records(self) -> int:
        return self.engine.comm_info()["exchanged_records"]

    def step(self, n_ticks: int, between: Optional[Callable[[], object]] = None) -> int:
        """One window on every rank (collective).  `between` runs on the host while the window
        simulates (its ConfigureNetwork calls take effect at the next launch): at N > 1 before
        comm_finish, which waits for the exchanged counts; at one rank comm_finish waits for nothing,
        so it goes first and the delivery is queued behind the simulation at once (run before it,
        the host work held the delivery back by ~0.35 ms per C5 epoch)."""
        self.engine.comm_launch(n_ticks)
        if between is not None and self.world > 1:
            between()
        self.engine.comm_finish()
        if between is not None and self.world == 1:
            between()
        return -1

    def run(self, n_steps: int, n_ticks: int, fuse: int = 1) -> int:
        self.engine.comm_run(n_ticks, n_steps, fuse, self.slot_cap or 0)
        self.slot_cap = self.engine.comm_info()["slot_cap"]
        return -1

    def barrier(self, state: int, target: int) -> bool:
        return self.engine.comm_barrier(state, target)


class ShardedStepper:
    """One step = step_sim -> exchange -> deliver on every rank; run() pipelines many.  On GPUs the
    delivery of step k runs on the engine's delivery stream beside the k_sim of the next step
    (tgsim_deliver_async).  The engine's simulate stream waits for the collective that still reads
    the output buffer it is about to overwrite, and the exchange stream waits for the delivery that
    still reads the input buffer it is about to overwrite (events, not host synchronization).

    Exact mode (step(), and run() without slot_cap): the per-rank record counts are exchanged
    first (an all-to-all of the count vector), so the host waits for each step's routing and for
    that collective.  Slotted mode (run() with slot_cap, on GPUs): every rank sends every rank a
    fixed chunk of slot_cap records behind a count header, so nothing the host needs comes from the
    device and the host only enqueues; a chunk that would overflow fails the run with -ENOSPC.
    max_count (the largest per-rank count an exact step saw) sizes slot_cap."""

    def __init__(self, engine, bounds: Sequence[int], device: str = "cuda", group=None,
                 slot_cap: Optional[int] = None):
        self.engine = engine
        self.bounds = list(bounds)
        self.device = torch.device(device)
        self.group = group
        # records out of step k in _out[k % 3] (two launched steps + the one being exchanged), into
        # this rank in _in[k % 2]; _ev[j]: the exchange that last read _out[j]
        self._out: List[Optional[torch.Tensor]] = [None] * 3
        self._in: List[Optional[torch.Tensor]] = [None] * 2
        self._ev: List[Optional[torch.cuda.Event]] = [None] * 3
        self._dev: List[Optional[torch.cuda.Event]] = [None] * 2  # _dev[i]: the delivery that last read _in[i]
        self._k = 0
        # the exchange's stream: high priority, off the simulate stream's hardware queue (init_rccl)
        self._xs = torch.cuda.Stream(self.device, priority=-1) if self.device.type == "cuda" else None
        self.slot_cap = slot_cap
        self.max_count = 0
        self.exchanged_records = 0  # records (slotted: record slots) this rank has sent, all steps
        self._routed: List[Optional[torch.cuda.Event]] = [None] * 3  # slotted: out[j] complete
        self._sig_ev: Optional[torch.cuda.Event] = None  # after the engine's issued signals

    def _buf(self, bufs: list, i: int, n_bytes: int) -> torch.Tensor:
        b = bufs[i]
        if b is None or b.numel() < n_bytes:
            b = torch.empty(max(REC, int(n_bytes * 1.25)), dtype=torch.uint8, device=self.device)
            bufs[i] = b
        return b

    def _launch(self, n_ticks: int):
        k = self._k
        self._k += 1
        j = k % 3
        out = self._buf(self._out, j, self.engine.sim_capacity() * REC)
        if self.device.type == "cuda" and self._ev[j] is not None:  # an earlier exchange still reads out[j]
            self.engine.wait_event(self._ev[j].cuda_event)
        self.engine.step_sim_launch(n_ticks, self.bounds, out.data_ptr(), out.numel() // REC)
        return k, out

    def _exchange(self, k: int, out: torch.Tensor, cnt: np.ndarray) -> int:
        if self._xs is None:
            return self._exchange_on(k, out, cnt)
        with torch.cuda.stream(self._xs):
            return self._exchange_on(k, out, cnt)

    def _exchange_on(self, k: int, out: torch.Tensor, cnt: np.ndarray) -> int:
        cuda = self.device.type == "cuda"
        self.max_count = max(self.max_count, int(cnt.max()) if len(cnt) else 0)
        self.exchanged_records += int(cnt.sum())
        send = torch.as_tensor(cnt.astype(np.int64), device=self.device)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        rcnt = recv.cpu().numpy()
        n_in = int(rcnt.sum())
        i = k % 2
        if cuda:
            if self._dev[i] is not None:  # the delivery of step k - 2 still reads _in[i]
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(self._dev[i])
                if self._in[i] is not None and self._in[i].numel() < n_in * REC:
                    self._dev[i].synchronize()  # growing: the old block returns to the allocator
        inb = self._buf(self._in, i, n_in * REC)
        dist.all_to_all_single(inb[: n_in * REC], out[: int(cnt.sum()) * REC],
                               [int(x) * REC for x in rcnt], [int(x) * REC for x in cnt], group=self.group)
        if cuda:  # the collective runs on torch's stream: the delivery stream waits for it
            self.engine.deliver_async(inb.data_ptr(), n_in, self._exchanged(k))
            self._mark_delivery(i)
        else:
            self.engine.deliver(inb.data_ptr(), n_in)
        return n_in

    def _exchanged(self, k: int) -> int:
        """Event after the exchange of step k on the current (exchange) stream."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._ev[k % 3] = ev
        return ev.cuda_event

    def _mark_delivery(self, i: int) -> None:
        """_dev[i]: recorded on the delivery stream after the delivery just enqueued (from _in[i])."""
        dv = self._dev[i] or torch.cuda.Event()
        if self._dev[i] is None:
            dv.record(torch.cuda.current_stream(self.device))  # creates the event
        self.engine.delivery_event(dv.cuda_event)
        self._dev[i] = dv

    def _event(self, evs: list, j: int) -> torch.cuda.Event:
        ev = evs[j]
        if ev is None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))  # creates the event
            evs[j] = ev
        return ev

    def _launch_slotted(self, n_ticks: int, n_win: int = 1):
        """One launched step: a window, or a fused group of n_win windows (tgsim_step_sim_launch_slotted_n:
        rank-major chunks, window-minor, all moved by one all-to-all)."""
        k = self._k
        self._k += 1
        j = k % 3
        n_r = len(self.bounds) - 1
        out = self._buf(self._out, j, n_r * n_win * (self.slot_cap + 1) * REC)
        if self._ev[j] is not None:  # an earlier exchange still reads out[j]
            self.engine.wait_event(self._ev[j].cuda_event)
        routed = self._event(self._routed, j)
        if n_win > 1:
            self.engine.step_sim_launch_slotted_n(n_ticks, n_win, self.bounds, out.data_ptr(), self.slot_cap,
                                                  routed.cuda_event)
        else:
            self.engine.step_sim_launch_slotted(n_ticks, self.bounds, out.data_ptr(), self.slot_cap, routed.cuda_event)
        return k, out, n_win

    def _exchange_slotted(self, k: int, out: torch.Tensor, n_win: int = 1) -> None:
        n_r = len(self.bounds) - 1
        size = n_r * n_win * (self.slot_cap + 1) * REC
        i = k % 2
        with torch.cuda.stream(self._xs):
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(self._routed[k % 3])  # the routing of step k filled out
            if self._dev[i] is not None:  # the delivery of step k - 2 still reads _in[i]
                cur.wait_event(self._dev[i])
            if self._in[i] is not None and self._in[i].numel() < size and self._dev[i] is not None:
                self._dev[i].synchronize()  # growing: the old block returns to the allocator
            inb = self._buf(self._in, i, size)
            self.exchanged_records += n_r * n_win * (self.slot_cap + 1)
            dist.all_to_all_single(inb[:size], out[:size], group=self.group)
            if n_win > 1:
                self.engine.deliver_slotted_n_async(inb.data_ptr(), n_r, n_win, self.slot_cap, self._exchanged(k))
            else:
                self.engine.deliver_slotted_async(inb.data_ptr(), n_r, self.slot_cap, self._exchanged(k))
            self._mark_delivery(i)

    def step(self, n_ticks: int, between: Optional[Callable[[], object]] = None) -> int:
        """One window on every rank (collective).  Returns the records delivered to this rank.
        `between` runs on the host while the window simulates (e.g. staging the next epoch's
        ConfigureNetwork calls, which take effect at the next launch)."""
        k, out = self._launch(n_ticks)
        if between is not None:
            between()
        return self._exchange(k, out, self._finish())

    def _finish(self) -> np.ndarray:
        if self.device.type == "cuda":
            return self.engine.step_sim_counts()
        return self.engine.step_sim_finish()

    def run(self, n_steps: int, n_ticks: int, fuse: int = 1) -> int:
        """n_steps windows with the simulation two steps ahead of the exchange: while the host
        exchanges step k, the engine's simulate stream already holds steps k+1 and k+2, so it never
        idles on the host.  Only for steps with no host-side change between them (pre-generated
        traffic, no reshaping, no receipts feeding generation); the results are identical to
        n_steps calls of step().  Returns the records delivered to this rank, or -1 in slotted
        mode (the host never reads a count there).  fuse > 1 (slotted mode): groups of up to `fuse`
        generated windows per launch and per all-to-all."""
        if self.slot_cap and self.device.type == "cuda":
            groups = [fuse] * (n_steps // fuse) + ([n_steps % fuse] if n_steps % fuse else []) if fuse > 1 \
                else [1] * n_steps
            pend = [self._launch_slotted(n_ticks, w) for w in groups[:2]]
            for s in range(len(groups)):
                k, out, w = pend.pop(0)
                self.engine.step_sim_release()
                if s + 2 < len(groups):
                    pend.append(self._launch_slotted(n_ticks, groups[s + 2]))
                self._exchange_slotted(k, out, w)
            return -1  # the host never read a count
        total = 0
        pend = [self._launch(n_ticks) for _ in range(min(2, n_steps))]
        for s in range(n_steps):
            k, out = pend.pop(0)
            cnt = self._finish()
            if s + 2 < n_steps:
                pend.append(self._launch(n_ticks))
            total += self._exchange(k, out, cnt)
        return total

    def barrier(self, state: int, target: int) -> bool:
        """Global barrier over the shards' sync counters (K7): the per-rank counts of `state` are
        summed with an all-reduce and compared with target (SignalAndWait semantics).  On GPUs the
        counter is read straight from the engine's device table on the exchange stream, behind an
        event recorded after every signal the engine issued (no host copy before the collective;
        the comparison itself is the barrier's one host read).  On CPU (oracle shards, gloo) the
        table is host memory."""
        if self.device.type != "cuda":
            t = torch.tensor([self.engine.signal(state, 0)], dtype=torch.int64)
            dist.all_reduce(t, group=self.group)
            return int(t.item()) >= target
        ev = self._sig_ev or torch.cuda.Event()
        if self._sig_ev is None:
            ev.record(torch.cuda.current_stream(self.device))  # creates the event
            self._sig_ev = ev
        ptr, n = self.engine.sync_counters(ev.cuda_event)
        table = device_table(ptr, n, self.device)
        with torch.cuda.stream(self._xs):
            torch.cuda.current_stream(self.device).wait_event(ev)
            t = table[state:state + 1].clone()
            dist.all_reduce(t, group=self.group)
            return int(t.item()) >= target
