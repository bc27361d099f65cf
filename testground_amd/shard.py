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

from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

REC = 24  # sizeof(tgsim_delivery)


def shard_bounds(n_peers: int, world: int) -> List[int]:
    """Contiguous source ranges, as even as possible: rank r owns [b[r], b[r+1])."""
    return [(n_peers * r) // world for r in range(world)] + [n_peers]


class ShardedStepper:
    """One step = step_sim -> exchange -> deliver on every rank.  On GPUs the delivery of step k
    runs on the engine's delivery stream beside the k_sim of step k+1 (tgsim_deliver_async): the
    exchange buffers are double-buffered, the engine's simulate stream waits for the collective that
    still reads the output buffer it is about to overwrite, and step_sim returns only after the
    previous delivery has released its input buffer."""

    def __init__(self, engine, bounds: Sequence[int], device: str = "cuda", group=None):
        self.engine = engine
        self.bounds = list(bounds)
        self.device = torch.device(device)
        self.group = group
        self._out: List[Optional[torch.Tensor]] = [None, None]
        self._in: List[Optional[torch.Tensor]] = [None, None]
        self._ev: List[Optional[torch.cuda.Event]] = [None, None]
        self._k = 0

    def _buf(self, bufs: list, i: int, n_bytes: int) -> torch.Tensor:
        b = bufs[i]
        if b is None or b.numel() < n_bytes:
            b = torch.empty(max(REC, int(n_bytes * 1.25)), dtype=torch.uint8, device=self.device)
            bufs[i] = b
        return b

    def step(self, n_ticks: int) -> int:
        """One window on every rank (collective).  Returns the records delivered to this rank."""
        cuda = self.device.type == "cuda"
        i = self._k & 1
        self._k += 1
        cap = self.engine.sim_capacity()
        out = self._buf(self._out, i, cap * REC)
        if cuda and self._ev[i] is not None:  # the exchange of two steps ago still reads out[i]
            self.engine.wait_event(self._ev[i].cuda_event)
        cnt = self.engine.step_sim(n_ticks, self.bounds, out.data_ptr(), out.numel() // REC)
        send = torch.as_tensor(cnt.astype(np.int64), device=self.device)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        rcnt = recv.cpu().numpy()
        n_in = int(rcnt.sum())
        inb = self._buf(self._in, i, n_in * REC)
        dist.all_to_all_single(inb[: n_in * REC], out[: int(cnt.sum()) * REC],
                               [int(x) * REC for x in rcnt], [int(x) * REC for x in cnt], group=self.group)
        if cuda:  # the collective runs on torch's stream: the engine's delivery stream waits for it
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._ev[i] = ev
            self.engine.deliver_async(inb.data_ptr(), n_in, ev.cuda_event)
        else:
            self.engine.deliver(inb.data_ptr(), n_in)
        return n_in

    def barrier(self, state: int, target: int) -> bool:
        """Global barrier over the shards' sync counters: the per-rank counts of `state` are summed
        with an all-reduce (RCCL on GPUs) and compared with target (SignalAndWait semantics)."""
        local = self.engine.signal(state, 0)
        t = torch.tensor([local], dtype=torch.int64, device=self.device)
        dist.all_reduce(t, group=self.group)
        return int(t.item()) >= target
