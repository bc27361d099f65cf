"""k_sim phase breakdown from in-kernel s_memrealtime stamps (diagnostic build path)."""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

os.environ["TGSIM_STAMPS"] = "1"
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

torch.cuda.init()
from testground_amd import abi, workloads  # noqa: E402
from testground_amd.engine import Engine  # noqa: E402

peers = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
lam = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
ql = int(sys.argv[3]) if len(sys.argv) > 3 else 0
nsteps = int(sys.argv[4]) if len(sys.argv) > 4 else 4
e = Engine(peers, flags=abi.OPT_DISCARD_DELIVERIES, queue_limit=ql)
workloads.configure_storm(e, peers)
for _ in range(nsteps):
    e.gen_storm(lam, 2000)
    e.step(2000)
n = e._lib.tgsim_debug_stamps(e._h, None, 0)
st = np.zeros(n, dtype=np.uint64)
e._lib.tgsim_debug_stamps(e._h, st.ctypes.data, n)
st = st.reshape(-1, 8).astype(np.int64)
t0 = st[:, 0].min()
ph = np.diff(st[:, :5], axis=1) * 10 / 1000  # us (100 MHz)
tot = (st[:, 4] - st[:, 0]) * 10 / 1000
print(f"steps={nsteps} peers={peers} lam={lam} ql={ql} wgs={len(st)} kernel span {(st[:, 4].max() - t0) * 10 / 1e6:.3f} ms")
for name, col in zip(["load", "batches", "end_htb", "writeback"], ph.T):
    print(f"  {name:10s} mean {col.mean():8.2f} us  p50 {np.median(col):8.2f}  max {col.max():8.2f}")
print(f"  total      mean {tot.mean():8.2f} us  p50 {np.median(tot):8.2f}  max {tot.max():8.2f}")
src_of = st[:, 5] >> 32
nbat = st[:, 5] & 0xFFFFFFFF
print(f"  batches/wg mean {nbat.mean():.1f}; queue (heap, ring) mean {np.mean(st[:, 7] >> 32):.0f}, {np.mean(st[:, 7] & 0xffffffff):.0f}")
start = (st[:, 0] - t0) * 10 / 1000
end = (st[:, 4] - t0) * 10 / 1000
ts = np.linspace(0, end.max(), 20)
conc = [int(((start <= t) & (end > t)).sum()) for t in ts]
print("  concurrency over time:", conc)
shapes = workloads.storm_shapes(peers)
order = np.argsort(-tot)[:12]
print("  slowest workgroups (= sources):")
for i in order:
    s = shapes[src_of[i]]
    print(f"    wg {i:5d} src {src_of[i]:5d} start {start[i]:7.1f} us {tot[i]:8.1f} us  batches {nbat[i]}  heap {st[i,7]>>32} ring {st[i,7]&0xffffffff}  "
          f"L {s.Latency/1e6:6.2f} ms J {s.Jitter/1e6:5.2f} ms bw {s.Bandwidth/1e6:5.0f} Mb loss {s.Loss:.2f} reo {s.Reorder:.2f} dup {s.Duplicate:.2f}")
