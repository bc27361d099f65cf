"""k_sim phase breakdown from in-kernel stamps (diagnostic library libtgsim_prof.so).

Phase stamps (s_memrealtime, 100 MHz) per workgroup plus, in the profile build, s_memtime cycle
counters of the sequential recurrence: admit / heap_pop / heap_push (cycles and counts), the
parallel phase, the replay loop and the number of queue-full runs resolved by ballot.
"""
import argparse
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ["TGSIM_STAMPS"] = "1"
os.environ.setdefault("TGSIM_LIB", str(ROOT / "testground_amd" / "libtgsim_prof.so"))
import torch  # noqa: E402

torch.cuda.init()
from testground_amd import abi, workloads  # noqa: E402
from testground_amd.engine import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--peers", type=int, default=10000)
ap.add_argument("--lam", type=float, default=0.5)
ap.add_argument("--ql", type=int, default=0)
ap.add_argument("--steps", type=int, default=65, help="steps of --window ticks (the last one is reported)")
ap.add_argument("--window", type=int, default=2000)
ap.add_argument("--workload", default="storm", choices=["storm", "gossip"])
ap.add_argument("--top", type=int, default=12)
a = ap.parse_args()

kw = dict(lookahead_ns=workloads.GOSSIP_MIN_LAT) if a.workload == "gossip" else {}
e = Engine(a.peers, flags=abi.OPT_DISCARD_DELIVERIES, queue_limit=a.ql, **kw)
if a.workload == "gossip":
    workloads.configure_gossip(e, a.peers)
    e.gossip_init(n_floods=64, degree=8, msg_len=1024, start_gap_ticks=1000, start_tick=0)
    a.window = workloads.gossip_window_ticks(e)
else:
    workloads.configure_storm(e, a.peers)
for _ in range(a.steps):
    if a.workload == "gossip":
        e.gen_gossip(a.window)
    else:
        e.gen_storm(a.lam, a.window)
    e.step(a.window)
n = e._lib.tgsim_debug_stamps(e._h, None, 0)
st = np.zeros(n, dtype=np.uint64)
e._lib.tgsim_debug_stamps(e._h, st.ctypes.data, n)
st = st.reshape(-1, 32).astype(np.int64)
t0 = st[:, 0].min()
ph = np.diff(st[:, :5], axis=1) * 10 / 1000  # us (100 MHz)
tot = (st[:, 4] - st[:, 0]) * 10 / 1000
print(f"{a.workload} steps={a.steps} peers={a.peers} lam={a.lam} ql={a.ql} wgs={len(st)} "
      f"kernel span {(st[:, 4].max() - t0) * 10 / 1e6:.3f} ms")
for name, col in zip(["load", "batches", "end_htb", "writeback"] if a.workload == "storm" else ["lvl1", "lvl2+draws", "gather+htb", "writes"], ph.T):
    print(f"  {name:10s} mean {col.mean():8.2f} us  p50 {np.median(col):8.2f}  max {col.max():8.2f}")
print(f"  total      mean {tot.mean():8.2f} us  p50 {np.median(tot):8.2f}  max {tot.max():8.2f}")
src_of = st[:, 5] >> 32
nbat = st[:, 5] & 0xFFFFFFFF
print(f"  batches/wg mean {nbat.mean():.1f}; queue (heap, ring) mean {np.mean(st[:, 7] >> 32):.0f}, "
      f"{np.mean(st[:, 7] & 0xffffffff):.0f}")
start = (st[:, 0] - t0) * 10 / 1000
end = (st[:, 4] - t0) * 10 / 1000
ts = np.linspace(0, end.max(), 20)
print("  concurrency over time:", [int(((start <= t) & (end > t)).sum()) for t in ts])
pf = st[:, 8:32]  # profile build counters (see k_sim PROF_* slots)
nb = np.maximum(nbat, 1)
names = {0: "parallel", 1: "windows", 7: "S+htb", 8: "departures", 9: "decide", 10: "window-end",
         11: "commit", 4: "insert", 14: "ins-search", 15: "ins-shift", 12: "serve-mid", 13: "serve-end",
         16: "refill", 20: "rf-count", 21: "rf-take", 22: "rf-insert"}
print("  cycles per batch (mean over wgs): " + ", ".join(f"{v} {np.mean(pf[:, k] / nb):.0f}" for k, v in names.items()))
print(f"  per batch: {np.mean(pf[:, 3] / nb):.2f} windows, {np.mean(pf[:, 2] / nb):.2f} full-queue runs, "
      f"{np.mean(pf[:, 5] / nb):.2f} inserted items, {np.mean(pf[:, 6] / nb):.2f} shift chunks, "
      f"{np.mean(pf[:, 17] / nb):.2f} refill rounds, {np.mean(pf[:, 18] / nb):.2f} refilled items, "
      f"{np.mean(pf[:, 19] / nb):.2f} pool appends, {np.mean(pf[:, 23] / nb):.2f} windows ended by an admission")
# the heavy-source chain's limit.  A sub-window ends early when an item admitted in
# it becomes eligible before a later packet of it (reorder, or a delay <= 0 with J > L); absorbing
# those into the sub-window's departure scan would leave windows - admission-ended sub-windows.
top = np.argsort(-tot)[:512]
w_top, a_top = pf[top, 3].sum(), pf[top, 23].sum()
print(f"  512 slowest sources: {np.mean(pf[top, 3] / nb[top]):.2f} sub-windows per batch, "
      f"{np.mean(tot[top] / np.maximum(pf[top, 3], 1)):.2f} us per sub-window, {a_top / max(w_top, 1) * 100:.1f} % of "
      f"their sub-windows ended by an admission; the slowest source {tot[top[0]]:.1f} us with {pf[top[0], 3]} "
      f"sub-windows, {pf[top[0], 23]} of them admission-ended (absorbing them: >= "
      f"{tot[top[0]] * (1 - pf[top[0], 23] / max(pf[top[0], 3], 1)):.1f} us if time scales with sub-windows)")
shapes = workloads.storm_shapes(a.peers) if a.workload == "storm" else None
print("  slowest workgroups (= sources):")
for i in np.argsort(-tot)[:a.top]:
    line = (f"    src {src_of[i]:7d} start {start[i]:7.1f} us {tot[i]:8.1f} us  batches {nbat[i]:3d}  "
            f"q {st[i, 7] >> 32}/{st[i, 7] & 0xffffffff}  win x{pf[i, 3]} items {pf[i, 5]} chunks {pf[i, 6]} "
            f"refills {pf[i, 17]}/{pf[i, 18]} pool+ {pf[i, 19]}  "
            + " ".join(f"{v} {pf[i, k] // nb[i]}" for k, v in names.items()))
    if shapes:
        s = shapes[src_of[i]]
        line += (f"  L {s.Latency / 1e6:6.2f} J {s.Jitter / 1e6:5.2f} bw {s.Bandwidth / 1e6:5.0f} "
                 f"reo {s.Reorder:.2f}")
    print(line)
# Launch tail: which workgroups finish last, when they started, and how duration depends on the
# dispatch position (workgroup id = dispatch order).
span = end.max()
tail = end > 0.85 * span
print(f"  tail (end > 85 % of span): {tail.sum()} wgs, start mean {start[tail].mean():.1f} us, "
      f"duration mean {tot[tail].mean():.1f} us, max {tot[tail].max():.1f}")
dec = np.array_split(np.arange(len(st)), 10)
print("  duration by dispatch decile (mean us):", [round(float(tot[d].mean()), 1) for d in dec])
print("  start by dispatch decile (mean us):   ", [round(float(start[d].mean()), 1) for d in dec])
print("  end by dispatch decile (max us):      ", [round(float(end[d].max()), 1) for d in dec])
if shapes:  # per bandwidth class: phase times and profile cycles per batch
    bwc = np.array([shapes[i].Bandwidth for i in src_of]) / 1e6
    for c in np.unique(bwc):
        m = bwc == c
        line = (f"  bw {c:6.0f} Mbit/s: {m.sum():5d} srcs, total {tot[m].mean():6.1f} us (load {ph[m, 0].mean():5.2f}, "
                f"batches {ph[m, 1].mean():6.2f}, end {ph[m, 2].mean():5.2f}, wb {ph[m, 3].mean():5.2f}); per batch: "
                + ", ".join(f"{v} {np.mean(pf[m, k] / nb[m]):.0f}" for k, v in names.items()) +
                f"; windows {np.mean(pf[m, 3] / nb[m]):.2f}, fullq {np.mean(pf[m, 2] / nb[m]):.2f}")
        print(line)
if shapes:
    lat = np.array([shapes[i].Latency for i in src_of]) / 1e6
    jit = np.array([shapes[i].Jitter for i in src_of]) / 1e6
    bw = np.array([shapes[i].Bandwidth for i in src_of]) / 1e6
    print(f"  tail sources: L {lat[tail].mean():.1f} ms, J {jit[tail].mean():.1f} ms, "
          f"bw mix {dict(zip(*np.unique(bw[tail], return_counts=True)))}")
