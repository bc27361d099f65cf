"""World-size-2 `gloo` run of the sharded step (testground_amd/shard.py) on CPU: each rank owns half
of the sources (an oracle shard), records are exchanged with all_to_all, and the result must equal
a single engine over all sources, step by step: verdicts per shard and deliveries per destination."""
import ctypes
import os
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from testground_amd import abi, workloads
from testground_amd.build import build_oracle
from testground_amd.engine import CABIEngine

N, STEPS, WINDOW, LAM = 200, 3, 1500, 0.5


def _oracle(n, **kw):
    lib = ctypes.CDLL(str(build_oracle()))
    abi.declare(lib, "tgo_")
    return CABIEngine(lib, "tgo_", n, **kw)


def _rank(rank, world, port, outdir):
    import torch.distributed as dist

    from testground_amd.shard import ShardedStepper, shard_bounds

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = shard_bounds(N, world)
    eng = _oracle(N, shard=(b[rank], b[rank + 1]))
    workloads.configure_storm(eng, N)
    st = ShardedStepper(eng, b, device="cpu")
    for k in range(STEPS):
        eng.gen_storm(LAM, WINDOW)
        st.step(WINDOW)
        np.save(os.path.join(outdir, f"v{rank}_{k}.npy"), eng.verdicts())
        np.save(os.path.join(outdir, f"d{rank}_{k}.npy"), eng.drain())
    dist.destroy_process_group()


def test_two_rank_gloo_equals_single_engine():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rank, args=(world, 29600 + os.getpid() % 300, d), nprocs=world,
                           start_method="spawn", join=True)
        ref = _oracle(N)
        workloads.configure_storm(ref, N)
        for k in range(STEPS):
            ref.gen_storm(LAM, WINDOW)
            ref.step(WINDOW)
            v = np.concatenate([np.load(os.path.join(d, f"v{r}_{k}.npy")) for r in range(world)])
            dl = np.concatenate([np.load(os.path.join(d, f"d{r}_{k}.npy")) for r in range(world)])
            vr, dr = ref.verdicts(), ref.drain()
            assert len(v) == len(vr) > 10_000 and (v == vr).all(), f"step {k}: verdicts"
            assert len(dl) == len(dr) and (dl == dr).all(), f"step {k}: deliveries"
