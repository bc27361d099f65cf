"""Host time of the routed closed loop at one rank (TGSIM_COMM_ROUTE1=1, the engine's exchange as a
Go host drives it): per window, the host's time in gen_gossip, comm_launch and comm_finish against
the window's wall time.  usage: host_probe_routed.py [peers]"""
import os
import sys
import time
from pathlib import Path

os.environ.setdefault("TGSIM_COMM_ROUTE1", "1")
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

torch.cuda.init()
from testground_amd import abi, workloads  # noqa: E402
from testground_amd.engine import Engine  # noqa: E402
from testground_amd.shard import CommStepper  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
dist.init_process_group("gloo", rank=0, world_size=1)
e = Engine(n, shard=(0, n), flags=abi.OPT_DISCARD_DELIVERIES, lookahead_ns=workloads.GOSSIP_MIN_LAT)
workloads.configure_gossip(e, n)
st = CommStepper(e, [0, n], device="cpu")
window = workloads.gossip_window_ticks(e)
for _ in range(2):
    e.step(window) if False else st.step(window)
e.gossip_init(n_floods=64, degree=8, msg_len=1024, start_gap_ticks=1000)
t = {"gen": [], "launch": [], "finish": [], "wall": []}
for k in range(70):
    t0 = time.perf_counter()
    e.gen_gossip(window)
    t1 = time.perf_counter()
    e.comm_launch(window)
    t2 = time.perf_counter()
    e.comm_finish()
    t3 = time.perf_counter()
    t["gen"].append(t1 - t0)
    t["launch"].append(t2 - t1)
    t["finish"].append(t3 - t2)
    t["wall"].append(t3 - t0)
e.sync()
for k, v in t.items():
    v = np.array(v) * 1e6
    print(f"{k:7s} mean {v.mean():8.1f} us  p50 {np.median(v):8.1f}  max {v.max():8.1f}")
dist.destroy_process_group()
