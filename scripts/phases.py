"""Per-source phase breakdown of the simulate kernel from its in-kernel stamps (TGSIM_STAMPS=1), for the
bench's dense workloads: storm (C3), open (the sub-capacity variant), epochs (C5).  Phases: heap and
ring load, timing-wheel load, batches, end-of-window HTB, park + write-back; plus the wheel's counts
(items loaded from due buckets, parked after the load, far items at the end and those left in the heap
array).  usage: phases.py --workload open [--fused]"""
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
ap.add_argument("--workload", default="storm", choices=["storm", "open", "epochs"])
ap.add_argument("--peers", type=int, default=0)
ap.add_argument("--settle-ms", type=float, default=120.0)
ap.add_argument("--fused", action="store_true", help="time one fused group of 8 windows (tgsim_step_n)")
a = ap.parse_args()
peers = a.peers or (100_000 if a.workload == "epochs" else 10_000)
lam = {"storm": 0.5, "open": workloads.STORM_OPEN_LAMBDA, "epochs": 0.2}[a.workload]
window = 1000 if a.workload == "epochs" else 2000
e = Engine(peers, flags=abi.OPT_DISCARD_DELIVERIES)
workloads.configure_storm(e, peers, open_links=a.workload == "open")
n_settle = int(a.settle_ms * 1000 / window + 0.999)
for k in range(n_settle + 4):
    if a.workload == "epochs" and k:
        workloads.epoch_reshape(e, peers, k)
    e.gen_storm(lam, window)
    e.step(window)
if a.fused:
    for _ in range(8):
        e.gen_storm(lam, window)
    e.step_n(window, 8)
n = e._lib.tgsim_debug_stamps(e._h, None, 0)
st = np.zeros(n, dtype=np.uint64)
e._lib.tgsim_debug_stamps(e._h, st.ctypes.data, n)
st = st.reshape(-1, 32).astype(np.int64)
live = st[:, 4] > 0
st = st[live]
us = lambda x: x * 10 / 1000  # noqa: E731  (s_memrealtime: 100 MHz)
ph = {"loads": us(st[:, 10] - st[:, 0]), "set-up": us(st[:, 1] - st[:, 10]),
      "batches": us(st[:, 2] - st[:, 1]), "end htb": us(st[:, 3] - st[:, 2]), "park+store": us(st[:, 4] - st[:, 3]),
      "total": us(st[:, 4] - st[:, 0])}
span = us(st[:, 4].max() - st[:, 0].min())
print(f"{a.workload} peers={peers} window={window} rows={len(st)} span {span:.1f} us"
      + (f" ({span / 8:.1f} us per window, 8 fused)" if a.fused else "") + f" lib={os.environ.get('TGSIM_LIB', 'libtgsim.so')}")
for k, v in ph.items():
    print(f"  {k:15s} mean {v.mean():8.2f} us  p50 {np.median(v):8.2f}  p90 {np.percentile(v, 90):8.2f}  max {v.max():8.2f}")
w8, w9 = st[:, 8].astype(np.uint64), st[:, 9].astype(np.uint64)
f = lambda x, sh, m: ((x >> np.uint64(sh)) & np.uint64(m)).astype(np.int64)  # noqa: E731
nd, pk, fn0, kept = f(w8, 0, 0xFFFF), f(w8, 16, 0xFFFF), f(w8, 32, 0xFFFF), f(w8, 48, 0xFFFF)
g, rb = f(w9, 32, 0xFF), f(w9, 40, 1)
w11 = st[:, 11].astype(np.uint64)
rl, rn0 = f(w11, 0, 0xFFFF), f(w11, 16, 0xFFFF)
q, rn = f(st[:, 7].astype(np.uint64), 32, 0xFFFFFFFF), f(st[:, 7].astype(np.uint64), 0, 0xFFFFFFFF)
for name, v in [("wheel items loaded", nd), ("parked after load", pk), ("far at end", fn0), ("far kept in heap", kept),
                ("ring loaded", rl), ("ring at start", rn0), ("heap items at end", q), ("wheel g", g), ("rebuild", rb)]:
    print(f"  {name:20s} mean {v.mean():8.2f}  p50 {np.median(v):8.1f}  p90 {np.percentile(v, 90):8.1f}  max {v.max():6d}")
