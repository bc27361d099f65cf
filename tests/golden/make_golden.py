"""Generates the golden fixtures of tests/golden/ with the CPU oracle (oracle/tgoracle.c).

The reference path (Go sidecar + Linux netem/HTB) cannot run in this image, so the
fixtures are the oracle's own outputs on small, fully specified inputs: per-peer shapes, the offered
packets of each step, and the expected verdict bytes, delivery records (drain order) and statistics.
They pin the oracle against regressions (tests/test_golden.py, CPU) and are the inputs/outputs the
HIP engine must reproduce bit for bit (same test, -m gpu).

    python tests/golden/make_golden.py      # rewrites tests/golden/*.npz
"""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from testground_amd import abi, workloads  # noqa: E402
from testground_amd.build import build_oracle  # noqa: E402
from testground_amd.engine import CABIEngine  # noqa: E402
from testground_amd.network import configs_array  # noqa: E402

HERE = Path(__file__).resolve().parent
SHAPE_KEYS = ("latency_ns", "jitter_ns", "bandwidth_bps", "loss", "duplicate", "corrupt", "reorder")


def case_storm():
    """C3 in miniature: 24 storm-shaped sources, random all-to-all host packets, 3 steps."""
    n, ticks, steps = 24, 3000, 3
    shapes = workloads.storm_shape_arrays(n, seed=1234)
    rng = np.random.default_rng(99)
    pkts = []
    seq = np.zeros(n, dtype=np.uint32)
    for _ in range(steps):
        m = 20_000
        src = rng.integers(0, n, m)
        p = np.zeros(m, dtype=abi.PKT_DTYPE)
        p["src"] = src
        p["dst"] = (src + 1 + rng.integers(0, n - 1, m)) % n
        p["len"] = rng.integers(64, 1501, m)
        p["tick"] = rng.integers(0, ticks, m)
        order = np.lexsort((p["tick"], src))
        counts = np.bincount(src, minlength=n)
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
        s = np.empty(m, dtype=np.uint32)
        s[order] = np.arange(m) - starts[src[order]] + seq[src[order]]
        seq += counts.astype(np.uint32)
        p["seq"] = s
        pkts.append(p)
    return dict(n=n, ticks=ticks, queue_limit=0, lookahead_ns=0, shapes=shapes, pkts=pkts)


def case_edge():
    """Zero latency, jitter > latency, 50 % reorder, 20 % duplicates, a 16-packet netem limit."""
    n, ticks = 8, 1000
    ms = 1_000_000
    shapes = dict(latency_ns=np.array([0, 50_000, 1 * ms, 2 * ms, 0, 5 * ms, 1 * ms, 20 * ms], dtype=np.int64),
                  jitter_ns=np.array([0, 100_000, 3 * ms, 0, 1 * ms, 5 * ms, 0, 2 * ms], dtype=np.int64),
                  bandwidth_bps=np.array([0, 10**6, 10**7, 10**8, 10**9, 0, 10**7, 10**6], dtype=np.int64),
                  loss=np.array([0, 5, 0, 1, 0, 10, 0, 0], dtype=np.float32),
                  duplicate=np.array([20, 0, 20, 0, 5, 0, 20, 0], dtype=np.float32),
                  corrupt=np.array([0, 10, 0, 0, 50, 0, 0, 1], dtype=np.float32),
                  reorder=np.array([50, 0, 5, 0, 0, 50, 0, 0], dtype=np.float32))
    rng = np.random.default_rng(7)
    pkts = []
    for step in range(2):
        m = 6000
        src = rng.integers(0, n, m)
        p = np.zeros(m, dtype=abi.PKT_DTYPE)
        p["src"] = src
        p["dst"] = (src + 1 + rng.integers(0, n - 1, m)) % n
        p["len"] = rng.integers(40, 1500, m)
        p["tick"] = rng.integers(0, ticks, m)
        p["seq"] = rng.permutation(m).astype(np.uint32) + np.uint32(step * m)
        pkts.append(p)
    return dict(n=n, ticks=ticks, queue_limit=16, lookahead_ns=0, shapes=shapes, pkts=pkts)


CASES = {"storm24": case_storm, "edge8": case_edge}


def run(engine, case):
    engine.configure_batch(np.arange(case["n"]), configs_array(**{k: case["shapes"][k] for k in SHAPE_KEYS},
                                                               routing_policy=2))
    out = []
    for p in case["pkts"]:
        engine.submit(p)
        engine.step(case["ticks"])
        st = engine.stats()
        out.append(dict(verdicts=engine.verdicts(), deliveries=engine.drain(),
                        stats=np.array([st["offered"], st["scheduled"], st["cloned"], st["corrupted"],
                                        st["bytes_scheduled"], st["queue_state_bytes"]]
                                       + [st["by_verdict"][k] for k in sorted(st["by_verdict"])], dtype=np.uint64)))
    return out


def load(name):
    z = np.load(HERE / f"{name}.npz")  # allow_pickle=False (default): data only
    k = int(z["steps"])
    case = dict(n=int(z["n"]), ticks=int(z["ticks"]), queue_limit=int(z["queue_limit"]),
                lookahead_ns=int(z["lookahead_ns"]), shapes={key: z[key] for key in SHAPE_KEYS},
                pkts=[z[f"pkts{i}"] for i in range(k)])
    expect = [dict(verdicts=z[f"verdicts{i}"], deliveries=z[f"deliveries{i}"], stats=z[f"stats{i}"])
              for i in range(k)]
    return case, expect


def main():
    lib = ctypes.CDLL(str(build_oracle()))
    abi.declare(lib, "tgo_")
    for name, make in CASES.items():
        case = make()
        e = CABIEngine(lib, "tgo_", case["n"], queue_limit=case["queue_limit"], lookahead_ns=case["lookahead_ns"])
        res = run(e, case)
        arrays = dict(n=case["n"], ticks=case["ticks"], queue_limit=case["queue_limit"],
                      lookahead_ns=case["lookahead_ns"], steps=len(case["pkts"]),
                      **{k: case["shapes"][k] for k in SHAPE_KEYS})
        for i, (p, r) in enumerate(zip(case["pkts"], res)):
            arrays[f"pkts{i}"] = p
            arrays[f"verdicts{i}"] = r["verdicts"]
            arrays[f"deliveries{i}"] = r["deliveries"]
            arrays[f"stats{i}"] = r["stats"]
        np.savez_compressed(HERE / f"{name}.npz", **arrays)
        print(name, [len(r["deliveries"]) for r in res])


if __name__ == "__main__":
    main()
