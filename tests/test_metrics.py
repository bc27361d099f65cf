"""K8 metrics (include/tgsim.h TGSIM_METRICS_*): per-instance counters and log2 histograms.

CPU: the oracle's tables are consistent with its own statistics, drain and queue state, and the
line-protocol export has the shape pkg/metrics/viewer.go queries (`results.<name>.*`, tag `run`,
field `value`).  GPU: the engine's device-side tables equal the oracle's, bit for bit."""
import numpy as np
import pytest

from testground_amd import abi
from testground_amd import metrics as mx
from testground_amd import workloads as wl
from testground_amd.engine import EngineError


def _run(e, n, steps=3, ticks=1500):
    wl.configure_storm(e, n)
    drained = []
    for _ in range(steps):
        e.gen_storm(0.5, ticks)
        e.step(ticks)
        drained.append(e.drain())
    return np.concatenate(drained)


def test_oracle_metrics_consistent(make_oracle):
    n, steps = 200, 3
    e = make_oracle(n, flags=abi.OPT_METRICS)
    d = _run(e, n, steps)
    m, s = e.metrics(), e.stats()
    src, dst, hist = m["src"], m["dst"], m["hist"]
    assert src.shape == (n, 12) and dst.shape == (n, 2) and hist.shape == (2, 64)
    assert int(src[:, 0].sum()) == s["offered"]
    for k, name in enumerate(abi.VERDICT_NAMES[:8]):
        assert int(src[:, 2 + k].sum()) == s["by_verdict"][name], name
    assert int(src[:, 10].sum()) == s["scheduled"] == len(d)
    assert int(src[:, 11].sum()) == s["bytes_scheduled"] == int(d["len"].sum())
    assert (dst[:, 0] == np.bincount(d["dst"], minlength=n)).all()
    assert (dst[:, 1] == np.bincount(d["dst"], weights=d["len"], minlength=n).astype(np.uint64)).all()
    assert (src[:, 10] == np.bincount(d["src"], minlength=n)).all()
    assert int(hist[0].sum()) == int(hist[1].sum()) == n * steps  # one entry per instance and step


def test_metrics_need_the_flag(make_oracle):
    e = make_oracle(4)
    with pytest.raises(EngineError, match="TGSIM_OPT_METRICS"):
        e.metrics()


def test_line_protocol_shape(make_oracle):
    n = 20
    e = make_oracle(n, flags=abi.OPT_METRICS)
    _run(e, n, 1, 500)
    out = mx.lines(e.metrics(), "storm", "run 1", 1_700_000_000_000_000_000)
    assert len(out) >= (len(mx.SRC_METRICS) + len(mx.DST_METRICS)) * n
    meas, rest = out[0].split(",", 1)
    assert meas == "results.storm.netem.offered" and rest.startswith(r"run=run\ 1,instance=0 value=")
    assert all(line.split(" ")[-1] == "1700000000000000000" for line in out)
    assert any(line.startswith("results.storm.hist.backlog,run=run\\ 1,bin=") for line in out)


@pytest.mark.gpu
def test_gpu_metrics_equal_oracle(make_oracle):
    import torch

    torch.cuda.init()
    from testground_amd.engine import Engine

    n = 300
    g, c = Engine(n, flags=abi.OPT_METRICS), make_oracle(n, flags=abi.OPT_METRICS)
    _run(g, n)
    _run(c, n)
    mg, mc = g.metrics(), c.metrics()
    for k in ("src", "dst", "hist"):
        assert (mg[k] == mc[k]).all(), k


@pytest.mark.gpu
def test_gpu_metrics_sharded_equal_oracle(make_oracle):
    """Two shards (step_sim -> exchange -> deliver): per-shard tables equal the oracle shards'."""
    import torch

    torch.cuda.init()
    from testground_amd.engine import Engine

    n, half = 240, 120
    gs = [Engine(n, shard=(0, half), flags=abi.OPT_METRICS), Engine(n, shard=(half, n), flags=abi.OPT_METRICS)]
    cs = [make_oracle(n, shard=(0, half), flags=abi.OPT_METRICS), make_oracle(n, shard=(half, n), flags=abi.OPT_METRICS)]
    for e in gs + cs:
        wl.configure_storm(e, n)
    for _ in range(2):
        for group, on_gpu in ((gs, True), (cs, False)):
            for e in group:
                e.gen_storm(0.5, 1000)
            outs = []
            for e in group:
                cap = max(1, e.sim_capacity())
                if on_gpu:
                    buf = torch.empty(cap * 24, dtype=torch.uint8, device="cuda")
                    cnt = e.step_sim(1000, [0, half, n], buf.data_ptr(), cap)
                else:
                    buf = np.zeros(cap, dtype=abi.DELIVERY_DTYPE)
                    cnt = e.step_sim(1000, [0, half, n], buf.ctypes.data, cap)
                outs.append((buf, cnt))
            for k, e in enumerate(group):
                if on_gpu:
                    parts = [b[int(cn[:k].sum()) * 24: int(cn[:k + 1].sum()) * 24] for b, cn in outs]
                    inbound = torch.cat(parts)
                    torch.cuda.current_stream().synchronize()
                    e.deliver(inbound.data_ptr(), inbound.numel() // 24)
                else:
                    inbound = np.concatenate([b[int(cn[:k].sum()): int(cn[:k + 1].sum())] for b, cn in outs])
                    e.deliver(inbound.ctypes.data, len(inbound))
    for g, c in zip(gs, cs):
        mg, mc = g.metrics(), c.metrics()
        for k in ("src", "dst", "hist"):
            assert (mg[k] == mc[k]).all(), k
