"""Working-set census of the C3 storm on the CPU oracle (diagnostic): per source and window start,
how much of its netem queue a window can touch.  ring prefix k = entries before the first with
d >= H (H = window end + lookahead), g = ring entries behind it, f = queued items with e >= H;
bound = limit - g - f is what a window could ever hold in LDS if g and f stay in HBM."""
import ctypes, sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from testground_amd import abi, workloads
from testground_amd.build import build_oracle
from testground_amd.engine import CABIEngine

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
W, LA, LIM = 2000, 2000 * 1000, 1000
lib = ctypes.CDLL(str(build_oracle()))
abi.declare(lib, "tgo_")
lib.tgo_debug_queue.restype = ctypes.c_int64
lib.tgo_debug_queue.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
e = CABIEngine(lib, "tgo_", n, lookahead_ns=LA)
workloads.configure_storm(e, n)
shapes = workloads.storm_shape_arrays(n, workloads.SEED)
ring = np.zeros(1024, np.uint64); item = np.zeros(1024, np.uint64)
rows = []
for w in range(68):
    if w >= 60:
        H = (w * W + W) * 1000 + LA
        for s in range(n):
            v = lib.tgo_debug_queue(e._h, s, ring.ctypes.data, item.ctypes.data)
            rn, hn = v >> 32, v & 0xFFFFFFFF
            d = ring[:rn]; big = np.nonzero(d >= H)[0]
            k = int(big[0]) if len(big) else rn
            f = int((item[:hn] >= H).sum())
            rows.append((w, s, rn, hn, k, rn - k, f, LIM - (rn - k) - f, rn + hn - (rn - k) - f))
    e.gen_storm(0.5, W)
    e.step(W)
a = np.array(rows)
bw = np.asarray(shapes["bandwidth_bps"])
print("windows 60-67, sources", n)
for name, col in (("total", None), ("ws_now", 8), ("bound", 7)):
    x = a[:, 2] + a[:, 3] if col is None else a[:, col]
    print(f"{name:7s} p50 {np.percentile(x,50):.0f} p90 {np.percentile(x,90):.0f} p99 {np.percentile(x,99):.0f} max {x.max()}")
for c in (512, 640, 768):
    print(f"bound > {c}: {(a[:,7] > c).mean()*100:.2f} % of source-windows, ws_now > {c}: {(a[:,8] > c).mean()*100:.2f} %")
for b in sorted(set(bw)):
    m = bw[a[:, 1]] == b
    print(f"bw {b/1e6:6.0f} Mbit: total p50 {np.median(a[m,2]+a[m,3]):.0f} ring {np.median(a[m,2]):.0f} k {np.median(a[m,4]):.0f} g {np.median(a[m,5]):.0f} f {np.median(a[m,6]):.0f} bound p50 {np.median(a[m,7]):.0f} p99 {np.percentile(a[m,7],99):.0f} max {a[m,7].max()}")
