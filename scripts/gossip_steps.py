"""Per-window wall times of the C4 gossip loop (bench.py --workload gossip), to find stalls."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from testground_amd import abi, workloads  # noqa: E402
from testground_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
torch.cuda.set_device(0)
eng = Engine(n, device=0, flags=abi.OPT_DISCARD_DELIVERIES, lookahead_ns=workloads.GOSSIP_MIN_LAT)
workloads.configure_gossip(eng, n)
eng.gossip_init(n_floods=64, degree=8, msg_len=1024, start_gap_ticks=1000, start_tick=0)
ts = []
for k in range(steps):
    t = time.perf_counter()
    t1 = time.perf_counter()
    eng.gen_gossip(5000)
    t2 = time.perf_counter()
    eng.step(5000)
    t3 = time.perf_counter()
    ts.append((k, (t2 - t1) * 1e3, (t3 - t2) * 1e3))
eng.sync()
for k, g, s in ts:
    print(f"window {k:3d}  gen {g:8.2f} ms  step {s:8.2f} ms")
