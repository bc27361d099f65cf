"""Peer-sharded stepping across ranks.

Shaping is egress-only and per source (pkg/sidecar/link.go:22-40), so every rank owns a
contiguous range of sources and computes their verdicts and delivery times locally.  The only
exchange is the hand-off of scheduled 24-B records to the destination's rank:

    engine.step_sim  -> records grouped by destination shard (caller-owned buffer)
    all_to_all       -> per-rank record counts, then the records (RCCL over xGMI on GPUs)
    engine.deliver   -> per-destination delivery order on the receiving rank

The same code drives the HIP engine with CUDA buffers (bench.py, backend "nccl" = RCCL) and, in
tests, CPU-oracle shards with CPU buffers over `gloo`.
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


def shard_bounds(n_peers: int, world: int) -> List[int]:
    """Contiguous source ranges, as even as possible: rank r owns [b[r], b[r+1])."""
    return [(n_peers * r) // world for r in range(world)] + [n_peers]


class ShardedStepper:
    """One step = step_sim -> exchange -> deliver on every rank; run() pipelines many.  On GPUs the
    delivery of step k runs on the engine's delivery stream beside the k_sim of the next step
    (tgsim_deliver_async).  The host never blocks on device work except for the step's per-rank
    record counts: the engine's simulate stream waits for the collective that still reads the
    output buffer it is about to overwrite, and the exchange stream waits for the delivery that
    still reads the input buffer it is about to overwrite (events, not host synchronization).  The
    counts themselves are host values (pinned edges), so they are exchanged over a CPU (gloo)
    group: a device collective would queue behind the running k_sim for a CU."""

    def __init__(self, engine, bounds: Sequence[int], device: str = "cuda", group=None):
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
        # host-side count exchange (collective: every rank constructs its stepper)
        ranks = dist.get_process_group_ranks(group) if group is not None else None
        self._cpu_group = dist.new_group(ranks=ranks, backend="gloo") if self.device.type == "cuda" else group

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
        send = torch.as_tensor(cnt.astype(np.int64))
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self._cpu_group)
        rcnt = recv.numpy()
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
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._ev[k % 3] = ev
            self.engine.deliver_async(inb.data_ptr(), n_in, ev.cuda_event)
            dv = self._dev[i] or torch.cuda.Event()
            if self._dev[i] is None:
                dv.record(torch.cuda.current_stream(self.device))  # creates the event
            self.engine.delivery_event(dv.cuda_event)
            self._dev[i] = dv
        else:
            self.engine.deliver(inb.data_ptr(), n_in)
        return n_in

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

    def run(self, n_steps: int, n_ticks: int) -> int:
        """n_steps windows with the simulation two steps ahead of the exchange: while the host
        exchanges step k, the engine's simulate stream already holds steps k+1 and k+2, so it never
        idles on the host.  Only for steps with no host-side change between them (pre-generated
        traffic, no reshaping, no receipts feeding generation); the results are identical to
        n_steps calls of step()."""
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
        """Global barrier over the shards' sync counters: the per-rank counts of `state` are summed
        with an all-reduce and compared with target (SignalAndWait semantics).  The counters are
        host values (tgsim_signal), so the sum runs on the host group: a device all-reduce would
        wait for a CU behind the running k_sim only to be copied back."""
        local = self.engine.signal(state, 0)
        t = torch.tensor([local], dtype=torch.int64)
        dist.all_reduce(t, group=self._cpu_group)
        return int(t.item()) >= target
