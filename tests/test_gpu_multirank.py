"""The engine's own exchange (tgsim_comm_*) with 2 and 3 ranks on one GPU, against one engine over
all peers: the routing, the count all-to-all, the grouped send/recv of the records, the slotted
chunks of the pipelined run and the barrier all-reduce, with more than one rank — the N > 1 path
that bench.py --gpus N and a Go host drive.  RCCL refuses two ranks on one device and the pool's
boxes have one GPU, so the ranks are threads of this process and the transport is the test double
tests/mockrccl/mock_rccl.cpp, linked into a test build of the engine (libtgsim_mockcomm.so:
the product's kernel and engine objects, tgsim_comm.cpp compiled with -DTGSIM_COMM_TEST_TRANSPORT).
Everything but the transport is the product code: the same routing kernels, exchange stream,
buffers, events and delivery.  Each rank's verdicts are its sources' and its drain its
destinations', so concatenated in rank order they equal the single engine's, window by window."""
import ctypes
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from testground_amd import abi
from testground_amd import workloads as wl
from testground_amd.build import MOCK_COMM_LIB
from testground_amd.engine import CABIEngine, Engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    if not MOCK_COMM_LIB.exists():
        pytest.fail(f"{MOCK_COMM_LIB} not built (__graft_entry__.build())")
    lib = ctypes.CDLL(str(MOCK_COMM_LIB))
    abi.declare(lib, "tgsim_")
    return lib


def _comm_id(lib) -> bytes:
    buf = ctypes.create_string_buffer(abi.COMM_ID_BYTES)
    assert lib.tgsim_comm_id(buf) == 0
    return buf.raw


def _ranks(lib, n, bounds, fn, **kw):
    """Runs fn(rank, engine) on one thread per rank (every collective call is made by all ranks at
    once, as processes would); returns the per-rank results in rank order."""
    world = len(bounds) - 1
    engs = [CABIEngine(lib, "tgsim_", n, shard=(bounds[r], bounds[r + 1]), device=0, **kw) for r in range(world)]
    cid = _comm_id(lib)

    def one(r):
        engs[r].comm_init(cid, r, world)
        return fn(r, engs[r])

    with ThreadPoolExecutor(world) as ex:
        futs = [ex.submit(one, r) for r in range(world)]
        out = [f.result(timeout=300) for f in futs]
    info = [e.comm_info() for e in engs]
    for e in engs:
        e.close()
    return out, info


@pytest.mark.parametrize("bounds", [[0, 130, 300], [0, 90, 200, 300]])
def test_ranks_storm_step_equals_single(lib, bounds):
    """Closed-window steps (tgsim_comm_step: exact counts, then the records) of the storm."""
    n, ticks, windows = 300, 1500, 6

    def rank(r, e):
        wl.configure_storm(e, n)
        got = []
        for _ in range(windows):
            e.gen_storm(0.5, ticks)
            e.comm_step(ticks)
            got.append((e.verdicts(), e.drain()))
        return got

    per_rank, info = _ranks(lib, n, bounds, rank)
    ref = Engine(n)
    wl.configure_storm(ref, n)
    for k in range(windows):
        ref.gen_storm(0.5, ticks)
        ref.step(ticks)
        v = np.concatenate([per_rank[r][k][0] for r in range(len(per_rank))])
        d = np.concatenate([per_rank[r][k][1] for r in range(len(per_rank))])
        vr, dr = ref.verdicts(), ref.drain()
        assert len(v) == len(vr) and (v == vr).all(), f"window {k}: verdicts"
        assert len(d) == len(dr) > 100 and (d == dr).all(), f"window {k}: deliveries"
    assert all(i["nranks"] == len(bounds) - 1 and i["bounds"] == bounds for i in info)
    assert sum(i["exchanged_records"] for i in info) > 1000


@pytest.mark.parametrize("fuse", [1, 4])
def test_ranks_slotted_run_equals_single(lib, fuse):
    """tgsim_comm_run: fixed-size chunks sized from the exact windows before it (max over the ranks
    through the all-reduce), two launches ahead of the exchange; fuse=4: fused groups (one launch
    and one all-to-all per four windows, rank-major chunks, window-minor)."""
    n, ticks, exact, steps = 2000, 1000, 2, 9
    bounds = [0, 600, 1300, 2000]

    def rank(r, e):
        wl.configure_storm(e, n)
        for _ in range(exact + steps):
            e.gen_storm(0.5, ticks)
        for _ in range(exact):
            e.comm_step(ticks)
        e.comm_run(ticks, steps, fuse, 0)
        e.sync()
        return e.drain(), e.stats()

    per_rank, info = _ranks(lib, n, bounds, rank)
    ref = Engine(n)
    wl.configure_storm(ref, n)
    want = []
    for _ in range(exact + steps):
        ref.gen_storm(0.5, ticks)
        ref.step(ticks)
        want.append(ref.drain())
    for r in range(3):
        lo, hi = bounds[r], bounds[r + 1]
        mine = np.concatenate([w[(w["dst"] >= lo) & (w["dst"] < hi)] for w in want])
        got = per_rank[r][0]
        assert len(got) == len(mine) > 10_000 and (got == mine).all(), f"rank {r}"
    st = ref.stats()
    assert sum(p[1]["offered"] for p in per_rank) == st["offered"]
    assert sum(p[1]["scheduled"] for p in per_rank) == st["scheduled"]
    caps = {i["slot_cap"] for i in info}
    assert len(caps) == 1 and caps.pop() > 0, "one slot capacity, agreed over the ranks"


def test_ranks_gossip_closed_loop_equals_single(lib):
    """C4's loop at two ranks: forwards generated from the records each rank received, receipts
    feeding the next window."""
    n, windows = 1500, 25
    kw = dict(lookahead_ns=wl.GOSSIP_MIN_LAT)

    def rank(r, e):
        wl.configure_gossip(e, n)
        e.gossip_init(n_floods=8, degree=8, msg_len=1024, start_gap_ticks=300, start_tick=0)
        w = wl.gossip_window_ticks(e)
        got = []
        for _ in range(windows):
            e.gen_gossip(w)
            e.comm_step(w)
            got.append(e.drain())
        return got, e.gossip_reached()

    per_rank, _ = _ranks(lib, n, [0, 700, 1500], rank, **kw)
    ref = Engine(n, **kw)
    wl.configure_gossip(ref, n)
    ref.gossip_init(n_floods=8, degree=8, msg_len=1024, start_gap_ticks=300, start_tick=0)
    w = wl.gossip_window_ticks(ref)
    total = 0
    for k in range(windows):
        ref.gen_gossip(w)
        ref.step(w)
        d = np.concatenate([per_rank[r][0][k] for r in range(2)])
        dr = ref.drain()
        assert len(d) == len(dr) and (d == dr).all(), f"window {k}"
        total += len(dr)
    assert total > 10_000
    assert (per_rank[0][1] + per_rank[1][1] == ref.gossip_reached()).all()


def test_ranks_epochs_barrier(lib):
    """C5 at two ranks: reshaping staged while the window simulates, the sync counters summed over
    the ranks on the device (tgsim_comm_barrier), the same deliveries as one engine."""
    n, ticks, epochs = 3000, 800, 4
    bounds = [0, 1400, 3000]

    def rank(r, e):
        wl.configure_storm(e, n)
        mine = bounds[r + 1] - bounds[r]
        got = []
        for k in range(epochs):
            e.gen_storm(0.2, ticks)
            e.comm_launch(ticks)
            wl.epoch_reshape(e, n, k + 1)  # staged: applies from the next launch
            e.comm_finish()
            state, rnd = wl.epoch_state(k)
            e.signal_async(state, mine)
            got.append((e.drain(), e.comm_barrier(state, rnd * n), e.comm_barrier(state, rnd * n + 1)))
        return got

    per_rank, _ = _ranks(lib, n, bounds, rank)
    ref = Engine(n)
    wl.configure_storm(ref, n)
    for k in range(epochs):
        if k:
            wl.epoch_reshape(ref, n, k)
        ref.gen_storm(0.2, ticks)
        ref.step(ticks)
        d = np.concatenate([per_rank[r][k][0] for r in range(2)])
        dr = ref.drain()
        assert len(d) == len(dr) > 0 and (d == dr).all(), f"epoch {k}"
        assert all(per_rank[r][k][1] for r in range(2)), f"epoch {k}: the barrier released"
        assert not any(per_rank[r][k][2] for r in range(2)), f"epoch {k}: one more than signalled"


@pytest.mark.parametrize("where", ["count all-to-all", "all-reduce"])
def test_rank_that_stops_times_out_peers(lib, monkeypatch, where):
    """a rank that stops before a collective (here: returns before its count
    all-to-all, or before the barrier's all-reduce) must not hang the others.  RCCL's collectives
    are asynchronous, so the others' exchange streams stop where RCCL's kernel would wait; the test
    transport does the same for a partner that never posts (MOCKRCCL_ABANDON_MS: the call returns and
    a gate kernel holds the stream), and the engine's bounded host wait (TGSIM_COMM_TIMEOUT_MS) fails
    the rank with -ETIMEDOUT naming the rank and the window; every later call fails fast, and
    destroying the engine aborts the communicator (which opens the gate) instead of draining it.
    The stopped rank finishes its own device work first: a spinning gate holds up any stream that
    shares its hardware queue."""
    import errno
    import threading
    import time

    from testground_amd.engine import EngineError

    monkeypatch.setenv("TGSIM_COMM_TIMEOUT_MS", "1500")
    monkeypatch.setenv("MOCKRCCL_ABANDON_MS", "300")
    n, ticks = 300, 1000
    bounds = [0, 150, 300]
    idle = threading.Event()

    def rank(r, e):
        wl.configure_storm(e, n)
        e.gen_storm(0.5, ticks)
        if where == "all-reduce":  # one good window first, then the barrier the other rank skips
            e.comm_step(ticks)
            e.signal_async(1, bounds[r + 1] - bounds[r])
        if r == 1:
            e.sync()  # stops here, its device work done: never posts the collective
            idle.set()
            return None
        assert idle.wait(60)
        t0 = time.monotonic()
        try:
            if where == "count all-to-all":
                e.comm_step(ticks)
            else:
                e.comm_barrier(1, n)
        except EngineError as ex:
            waited = time.monotonic() - t0
            try:  # the communicator is unusable from now on
                e.comm_step(ticks)
                again = 0
            except EngineError as ex2:
                again = ex2.code
            return ex.code, ex.msg, waited, again
        return "no error", "", time.monotonic() - t0, 0

    t0 = time.monotonic()
    per_rank, _ = _ranks(lib, n, bounds, rank)
    assert time.monotonic() - t0 < 60, "a rank hung instead of timing out"
    code, msg, waited, again = per_rank[0]
    assert code == -errno.ETIMEDOUT, (code, msg)
    assert 1.4 <= waited < 30, waited
    assert "rank 0 of 2 waited" in msg and where in msg and "window" in msg, msg
    assert again == -errno.ETIMEDOUT
