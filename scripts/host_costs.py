"""Host cost of the C5 epoch loop's calls: configure_batch of one epoch's reshape
(10 % of 100,000 peers) timed as the C call alone and through the Python wrapper, the asynchronous
step, signal_async and barrier_poll; medians over repeated epochs on a settled engine."""
import ctypes as C
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

torch.cuda.init()
from testground_amd import abi, workloads  # noqa: E402
from testground_amd.engine import Engine  # noqa: E402

n, window, lam = 100_000, 1000, 0.2
e = Engine(n, flags=abi.OPT_DISCARD_DELIVERIES)
workloads.configure_storm(e, n)
for _ in range(20):
    e.gen_storm(lam, window)
    e.step(window)
plans = [workloads.epoch_plan(n, k) for k in range(1, 41)]
t_c, t_py, t_step, t_sig, t_bar = [], [], [], [], []
fn = e._fn("configure_batch")
for k in range(40):
    e.gen_storm(lam, window)
torch.cuda.synchronize()
for k in range(40):
    sel, cfg = plans[k]
    peers = np.ascontiguousarray(sel, dtype=np.uint32)
    rcs = np.zeros(len(peers), dtype=np.int32)
    t0 = time.perf_counter()
    if k % 2:
        fn(e._h, peers.ctypes.data, cfg.ctypes.data, len(peers), rcs.ctypes.data)
        t_c.append(time.perf_counter() - t0)
    else:
        e.configure_batch(sel, cfg)
        t_py.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    e.step(window)
    t_step.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    e.signal_async(k % 1024, n)
    t_sig.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    e.barrier_poll(k % 1024, (k // 1024 + 1) * n)
    t_bar.append(time.perf_counter() - t0)
med = lambda v: float(np.median(v)) * 1e6  # noqa: E731
print(f"configure_batch of {len(plans[0][0])} peers: C call {med(t_c):.0f} us, through Engine {med(t_py):.0f} us; "
      f"step {med(t_step):.0f} us; signal_async {med(t_sig):.0f} us; barrier_poll {med(t_bar):.0f} us (medians)")
