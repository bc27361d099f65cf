"""The bounded local delivery of TGSIM_OPT_DISCARD_DELIVERIES: without a host round
trip the single-window delivery sizes its buffers from what the window's sources can emit.  Up to
2 GiB of buffers that bound is the worst case (2 per offered packet + the netem limit per source),
so no valid window can exceed it; beyond that (1M-peer shards) it allows TGSIM_DELIVER_SLACK queued
items per source and k_deliver_guard fails a window beyond it with -ENOSPC instead of writing past
the buffers.  The workload that used to trip the guard with valid traffic: a burst fills every netem
queue of a 1 Gbit/s, 50 ms link, then silence; 50 ms later each source releases ~330 queued items per
2 ms window while offering nothing."""
import numpy as np
import pytest

from testground_amd import abi
from testground_amd.engine import EngineError
from testground_amd.network import configs_array

pytestmark = pytest.mark.gpu

N, W = 64, 2000


def _burst_then_silence(e, windows=40):
    e.configure_batch(np.arange(N), configs_array(np.full(N, 50_000_000), bandwidth_bps=np.full(N, 1_000_000_000)))
    e.gen_storm(2.0, W)  # ~4,000 packets per source in 2 ms: every queue at the limit of 1,000
    e.step(W)
    for _ in range(windows):
        e.step(W)  # nothing offered: the queued items become eligible at 50 ms and drain at 1 Gbit/s
    e.sync()
    return e.stats()


def test_discard_delivery_releases_deep_queues_exactly(make_oracle):
    from testground_amd.engine import Engine

    gpu = Engine(N, flags=abi.OPT_DISCARD_DELIVERIES)
    got = _burst_then_silence(gpu)
    gpu.close()
    want = _burst_then_silence(make_oracle(N))
    assert got == want
    assert want["scheduled"] > 40 * N  # the release windows really emitted deep queues


def test_forced_slack_guard_reports_enospc(monkeypatch):
    from testground_amd.engine import Engine

    monkeypatch.setenv("TGSIM_DELIVER_SLACK", "1")
    gpu = Engine(N, flags=abi.OPT_DISCARD_DELIVERIES)
    with pytest.raises(EngineError) as ei:
        _burst_then_silence(gpu)
    assert ei.value.code == -28  # -ENOSPC, never a silent loss
    gpu.close()
