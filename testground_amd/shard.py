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
    def __init__(self, engine, bounds: Sequence[int], device: str = "cuda", group=None):
        self.engine = engine
        self.bounds = list(bounds)
        self.device = torch.device(device)
        self.group = group
        self._out: Optional[torch.Tensor] = None
        self._in: Optional[torch.Tensor] = None

    def _buf(self, attr: str, n_bytes: int) -> torch.Tensor:
        b = getattr(self, attr)
        if b is None or b.numel() < n_bytes:
            b = torch.empty(max(REC, int(n_bytes * 1.25)), dtype=torch.uint8, device=self.device)
            setattr(self, attr, b)
        return b

    def step(self, n_ticks: int) -> int:
        """One window on every rank (collective).  Returns the records delivered to this rank."""
        cuda = self.device.type == "cuda"
        if cuda:  # the engine writes `out` on its own stream: torch's last use of it must be done
            torch.cuda.current_stream(self.device).synchronize()
        cap = self.engine.sim_capacity()
        out = self._buf("_out", cap * REC)
        cnt = self.engine.step_sim(n_ticks, self.bounds, out.data_ptr(), out.numel() // REC)
        send = torch.as_tensor(cnt.astype(np.int64), device=self.device)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        rcnt = recv.cpu().numpy()
        n_in = int(rcnt.sum())
        inb = self._buf("_in", n_in * REC)
        dist.all_to_all_single(inb[: n_in * REC], out[: int(cnt.sum()) * REC],
                               [int(x) * REC for x in rcnt], [int(x) * REC for x in cnt], group=self.group)
        if cuda:  # the collective ran on torch's stream; the engine reads `inb` on its own
            torch.cuda.current_stream(self.device).synchronize()
        self.engine.deliver(inb.data_ptr(), n_in)
        return n_in

    def barrier(self, state: int, target: int) -> bool:
        """Global barrier over the shards' sync counters: the per-rank counts of `state` are summed
        with an all-reduce (RCCL on GPUs) and compared with target (SignalAndWait semantics)."""
        local = self.engine.signal(state, 0)
        t = torch.tensor([local], dtype=torch.int64, device=self.device)
        dist.all_reduce(t, group=self.group)
        return int(t.item()) >= target
