"""Per-step cost of the sharded stepping path (step_sim -> all_to_all -> deliver) against the
single-shard asynchronous step, on one GPU (world size 1, RCCL)."""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from testground_amd import abi, workloads  # noqa: E402
from testground_amd.engine import Engine  # noqa: E402
from testground_amd.shard import ShardedStepper, init_rccl  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29531")
torch.cuda.set_device(0)
init_rccl(torch.device("cuda", 0), rank=0, world_size=1)
n, win, steps = 10_000, 2000, 10
for mode in os.environ.get("MODES", "local,sharded,pipelined").split(","):
    e = Engine(n, flags=abi.OPT_DISCARD_DELIVERIES)
    workloads.configure_storm(e, n)
    st = ShardedStepper(e, [0, n], device="cuda:0") if mode != "local" else None
    step = e.step if st is None else st.step
    for _ in range(60 + steps):
        e.gen_storm(0.5, win)
    for _ in range(60):
        step(win)
    torch.cuda.synchronize()
    e.sim_kernel_ms(reset=True)
    t0 = time.perf_counter()
    if mode == "pipelined":
        st.run(steps, win)
    else:
        for _ in range(steps):
            step(win)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    k, _ = e.sim_kernel_ms()
    print(f"{mode}: {el * 1e3:.3f} ms/step, k_sim {k:.3f} ms, other {el * 1e3 - k:.3f} ms", flush=True)
    e.close()
dist.destroy_process_group()
