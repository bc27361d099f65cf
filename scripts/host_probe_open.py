"""Host vs device time of the sub-capacity storm's step_n (bench --shapes open): the host call's own
duration against the synchronized wall time, per window."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

torch.cuda.init()
from testground_amd import abi, workloads  # noqa: E402
from testground_amd.engine import Engine  # noqa: E402

n, window, lam = 10_000, 2000, workloads.STORM_OPEN_LAMBDA
e = Engine(n, flags=abi.OPT_DISCARD_DELIVERIES)
workloads.configure_storm(e, n, open_links=True)
for _ in range(60):
    e.gen_storm(lam, window)
    e.step(window)
for rep in range(3):
    for _ in range(30):
        e.gen_storm(lam, window)
    e.sync()
    t0 = time.perf_counter()
    e.step_n(window, 30)
    t1 = time.perf_counter()
    e.sync()
    t2 = time.perf_counter()
    print(f"rep {rep}: host call {1e6 * (t1 - t0) / 30:.1f} us/window, wall {1e6 * (t2 - t0) / 30:.1f} us/window")
