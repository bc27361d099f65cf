"""Source-major fused launch (k_sim_fused, tgsim_step_n) from the in-kernel stamps: each source's
chain of windows (start of its first window to the end of its last), the longest chains, the
per-window durations of the heaviest sources, the tail (when the last chains start and end) and the
resident sources over the launch.  TGSIM_STAMPS; libtgsim.so or TGSIM_LIB."""
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
ap.add_argument("--fuse", type=int, default=8)
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
S = a.peers
t0 = st[:, 0].min()
start = ((st[:, 0] - t0) / 100).reshape(g, S)  # us, [window, dispatch position]
end = ((st[:, 4] - t0) / 100).reshape(g, S)
dur = end - start
span = end.max()
cs, ce = start[0], end[g - 1]
chain = ce - cs
print(f"fused launch of {g} windows x {S} sources: span {span:.1f} us ({span / g:.1f} per window); "
      f"window duration mean {dur.mean():.1f} us (load {np.mean(st[:, 1] - st[:, 0]) / 100:.2f}, "
      f"write-back {np.mean(st[:, 4] - st[:, 3]) / 100:.2f}); sum of work / 2304 slots {dur.sum() / 2304:.1f} us")
top = np.argsort(-chain)[:8]
print("longest chains (dispatch position: start, end, chain us, per-window us):")
for p in top:
    print(f"  {p:5d}: {cs[p]:7.1f} {ce[p]:7.1f} {chain[p]:7.1f}  " + " ".join(f"{x:5.0f}" for x in dur[:, p]))
inner = (start[1:] - end[:-1])  # gap between consecutive windows of a source (re-split, bookkeeping)
print(f"gap between a source's windows: mean {inner.mean():.2f} us, max {inner.max():.2f}")
last_start = np.sort(cs)[-50:]
print(f"last 50 chain starts {last_start[0]:.1f} .. {last_start[-1]:.1f} us; chains ending after {0.9 * span:.0f} us: "
      f"{int((ce > 0.9 * span).sum())}")
ts = np.linspace(0, span, 24)
print("resident sources over time:", [int(((cs <= t) & (ce > t)).sum()) for t in ts])
print("chain length deciles (us):", [round(float(x), 1) for x in np.percentile(chain, np.arange(0, 101, 10))])
