"""Host time per call of the single-engine 1M-peer gossip loop (gen_gossip, step), three floods in one
process: where a window's time goes when the closed loop runs slow."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
from testground_amd import abi, workloads  # noqa: E402
from testground_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
for run in range(3):
    e = Engine(n, flags=abi.OPT_DISCARD_DELIVERIES, lookahead_ns=workloads.GOSSIP_MIN_LAT)
    workloads.configure_gossip(e, n)
    window = workloads.gossip_window_ticks(e)
    for _ in range(2):
        e.step(window)
    e.gossip_init(n_floods=64, degree=8, msg_len=1024, start_gap_ticks=1000)
    e.sync()
    tg, ts = [], []
    t0 = time.perf_counter()
    for _ in range(70):
        a = time.perf_counter()
        e.gen_gossip(window)
        b = time.perf_counter()
        e.step(window)
        c = time.perf_counter()
        tg.append(b - a)
        ts.append(c - b)
    e.sync()
    wall = (time.perf_counter() - t0) / 70
    tg, ts = np.array(tg) * 1e6, np.array(ts) * 1e6
    print(f"run {run}: {wall * 1e3:.3f} ms/window; gen mean {tg.mean():.0f} p50 {np.median(tg):.0f} max {tg.max():.0f} us; "
          f"step mean {ts.mean():.0f} p50 {np.median(ts):.0f} max {ts.max():.0f} us", flush=True)
    e.close()
