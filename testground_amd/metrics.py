"""K8 metrics export: the engine's device-side counters and histograms as InfluxDB line protocol.

The reference's plans record metrics through sdk-go `runenv.D()` / `runenv.R()` (counters and
histograms, e.g. plans/benchmarks/storm.go:72-208), which land in InfluxDB and are read back by
pkg/metrics: `SHOW MEASUREMENTS ... =~ /results.<name>.*/` and `SELECT last("value"), "run" ...
GROUP BY "run"` (pkg/metrics/viewer.go:46, :149).  `lines()` emits series in that shape: measurement
`results.<plan>.<metric>`, tag `run`, per-instance tag `instance` (or `bin` for histograms), field
`value`, timestamp in ns.
"""
from __future__ import annotations

from typing import Dict, Iterable, List

import numpy as np

from . import abi

SRC_METRICS = ["netem.offered", "netem.offered_bytes"] + [
    f"verdict.{abi.VERDICT_NAMES[i]}" for i in range(8)] + ["htb.served", "htb.served_bytes"]
DST_METRICS = ["delivery.records", "delivery.bytes"]
HIST_METRICS = ["hist.backlog", "hist.delivered"]


def _escape(v: str) -> str:
    return v.replace(" ", r"\ ").replace(",", r"\,").replace("=", r"\=")


def lines(m: Dict[str, np.ndarray], plan: str, run: str, ts_ns: int, shard_begin: int = 0,
          instances: Iterable[int] | None = None) -> List[str]:
    """One line per (metric, instance) of `m` (Engine.metrics()), plus one per histogram bin."""
    tags = f"run={_escape(run)}"
    out: List[str] = []
    src, dst = m["src"], m["dst"]
    sel = range(src.shape[0]) if instances is None else [i - shard_begin for i in instances]
    for col, name in enumerate(SRC_METRICS):
        meas = _escape(f"results.{plan}.{name}")
        out += [f"{meas},{tags},instance={shard_begin + i} value={int(src[i, col])}i {ts_ns}" for i in sel]
    for col, name in enumerate(DST_METRICS):
        meas = _escape(f"results.{plan}.{name}")
        out += [f"{meas},{tags},instance={shard_begin + i} value={int(dst[i, col])}i {ts_ns}" for i in sel]
    for h, name in enumerate(HIST_METRICS):
        meas = _escape(f"results.{plan}.{name}")
        out += [f"{meas},{tags},bin={b} value={int(c)}i {ts_ns}" for b, c in enumerate(m["hist"][h]) if c]
    return out
