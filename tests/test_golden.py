"""Golden fixtures (tests/golden/*.npz, written by tests/golden/make_golden.py from the CPU oracle):
the oracle must keep reproducing them (CPU), and the HIP engine must reproduce them bit for bit
through its C ABI (-m gpu)."""
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
import make_golden  # noqa: E402

CASES = sorted(make_golden.CASES)


def _check(engine, name):
    case, expect = make_golden.load(name)
    got = make_golden.run(engine, case)
    for i, (g, x) in enumerate(zip(got, expect)):
        assert np.array_equal(g["verdicts"], x["verdicts"]), f"{name} step {i}: verdicts"
        assert len(g["deliveries"]) == len(x["deliveries"]), f"{name} step {i}: delivery count"
        assert (g["deliveries"] == x["deliveries"]).all(), f"{name} step {i}: deliveries"
        assert np.array_equal(g["stats"], x["stats"]), f"{name} step {i}: statistics"


@pytest.mark.parametrize("name", CASES)
def test_oracle_reproduces_golden(make_oracle, name):
    case, _ = make_golden.load(name)
    _check(make_oracle(case["n"], queue_limit=case["queue_limit"], lookahead_ns=case["lookahead_ns"]), name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_engine_reproduces_golden(name):
    try:
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:  # pragma: no cover
        pass
    from testground_amd.engine import Engine

    case, _ = make_golden.load(name)
    _check(Engine(case["n"], queue_limit=case["queue_limit"], lookahead_ns=case["lookahead_ns"]), name)


def test_oracle_reproduces_fullsize_c5_prefix(make_oracle):
    """The committed full-size digests (tests/golden/fullsize_*.json, checked against the HIP engine
    by tests/test_gpu_fullsize_digests.py) still describe the current oracle: its first two C5
    epochs at 100,000 instances (about 40 M packets) reproduce their digests."""
    import make_fullsize as mf

    fx = mf.load("c5")
    entries = iter(fx["entries"][:2])

    class Stop(Exception):
        pass

    def sink(label, got):
        want = next(entries, None)
        if want is None:
            raise Stop
        assert want["label"] == label
        for key in ("n_verdicts", "verdicts", "n_deliveries", "deliveries", "stats"):
            assert got[key] == want[key], f"c5 {label}: {key}"

    with pytest.raises(Stop):
        mf.run_c5(make_oracle(mf.C5["peers"]), sink)
