"""Timeline of one fused launch (tgsim_step_n) from the in-kernel stamps: per window the span, the
mean source duration and the time tickets spent waiting for their source's previous window, plus
the resident-ticket count over the launch (TGSIM_STAMPS; libtgsim.so or TGSIM_LIB)."""
import argparse
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ["TGSIM_STAMPS"] = "1"
import torch  # noqa: E402

torch.cuda.init()
from testground_amd import abi, workloads  # noqa: E402
from testground_amd.engine import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--peers", type=int, default=10000)
ap.add_argument("--window", type=int, default=2000)
ap.add_argument("--settle", type=int, default=60)
ap.add_argument("--groups", type=int, default=3, help="fused launches of --fuse windows (the last is reported)")
ap.add_argument("--fuse", type=int, default=4)
a = ap.parse_args()
e = Engine(a.peers, flags=abi.OPT_DISCARD_DELIVERIES)
workloads.configure_storm(e, a.peers)
for _ in range(a.settle):
    e.gen_storm(0.5, a.window)
    e.step(a.window)
for _ in range(a.groups):
    for _ in range(a.fuse):
        e.gen_storm(0.5, a.window)
    e.step_n(a.window, a.fuse)
n = e._lib.tgsim_debug_stamps(e._h, None, 0)
st = np.zeros(n, dtype=np.uint64)
e._lib.tgsim_debug_stamps(e._h, st.ctypes.data, n)
st = st.reshape(-1, 32).astype(np.int64)
g = len(st) // a.peers
t0 = st[:, 0].min()
start, end = (st[:, 0] - t0) / 100, (st[:, 4] - t0) / 100  # us
wait = st[:, 31] / 100
print(f"fused launch of {g} windows, {len(st)} tickets, span {end.max():.1f} us ({end.max() / g:.1f} per window)")
for w in range(g):
    sl = slice(w * a.peers, (w + 1) * a.peers)
    dur = end[sl] - start[sl]
    print(f"  window {w}: start {start[sl].min():7.1f} .. {start[sl].max():7.1f}, end max {end[sl].max():7.1f} us, "
          f"source mean {dur.mean():6.1f} us (load {np.mean(st[sl, 1] - st[sl, 0]) / 100:5.2f}, "
          f"writeback {np.mean(st[sl, 4] - st[sl, 3]) / 100:5.2f}), waited: {np.count_nonzero(wait[sl] > 1)} tickets, "
          f"{wait[sl].sum():.0f} us in total, max {wait[sl].max():.1f}")
ts = np.linspace(0, end.max(), 24)
print("  resident tickets over time:", [int(((start <= t) & (end > t)).sum()) for t in ts])
print(f"  work / (2304 slots): {(end - start).sum() / 2304:.1f} us")
