"""BASELINE.json configs[2..4] at full size, HIP engine against the CPU oracle, window by window.

tests/golden/fullsize_{c3,c4,c5}.json hold the oracle's per-window digests (SHA-256 of the verdict
bytes and of the drain-ordered delivery records, their counts, every statistic), written by
tests/golden/make_fullsize.py in the build container.  Here the HIP engine runs the same drivers
through the paths the bench times:

  c3  10,000-instance storm: 60 single windows (k_sim), then two groups of eight windows in one
      tgsim_step_n call each (k_sim_fused);
  c4  1,000,000-peer gossip flood, 70 windows (k_sim_sparse + k_sim_list, device-side receipts and
      forward generation);
  c5  100,000-instance epochs with 10 % reshaped per epoch and a device barrier (k_sim, batched
      ConfigureNetwork).

A bug shared by two engine paths (fused and unfused, sparse and dense) cannot pass these: the
checker is the oracle, not the engine itself."""
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
import make_fullsize as mf  # noqa: E402

pytestmark = pytest.mark.gpu

try:  # torch ships its own HIP runtime: let it initialise first when both share a process
    import torch

    if torch.cuda.is_available():
        torch.cuda.init()
except ImportError:  # pragma: no cover
    torch = None


def _compare(name):
    from testground_amd.engine import Engine

    fx = mf.load(name)
    fn, cfg, kw = mf.RUNS[name]
    assert fx["config"] == cfg, f"{name}: fixture was generated for another configuration"
    expect = iter(fx["entries"])
    seen = [0]

    def sink(label, got):
        want = next(expect)
        assert want["label"] == label
        for key in ("n_verdicts", "n_deliveries", "stats", "reached"):
            assert got.get(key) == want.get(key), f"{name} {label}: {key} {got.get(key)} != oracle {want.get(key)}"
        for key in ("verdicts", "deliveries"):
            assert got.get(key) == want.get(key), f"{name} {label}: {key} digest differs from the oracle's"
        seen[0] += 1

    eng = Engine(cfg["peers"], **kw)
    fn(eng, sink)
    if name == "c3":  # the groups ran as the bench runs them: k_sim_fused, eight windows per launch
        assert int(eng._fn("debug_fused_windows")(eng._h)) == cfg["groups"] * cfg["group"]
    eng.close()
    assert seen[0] == len(fx["entries"])
    print(f"{name}: {seen[0]} digests equal to the oracle's", flush=True)


@pytest.mark.timeout(600)
def test_c3_storm_10k_equals_oracle():
    _compare("c3")


@pytest.mark.timeout(900)
def test_c4_gossip_1m_equals_oracle():
    _compare("c4")


@pytest.mark.timeout(600)
def test_c5_epochs_100k_equals_oracle():
    _compare("c5")
