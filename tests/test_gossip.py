"""C4 gossip flood workload on the CPU oracle: the driver's semantics checked
against an independent restatement.

* Reachability: a peer has flood f iff a path of non-lost edges leads to it from f's origin.
  Loss is keyed by (seed, src, dst, seq) only, so the reached set is a pure graph property,
  recomputed here by BFS from the Philox draws.
* Forward-on-first-receipt: every forward of (peer, flood) is offered at floor(d/tick) + 1 of the
  peer's earliest receipt of that flood, exactly once, to the `degree` hashed neighbours.
"""
import numpy as np
import pytest

from testground_amd import abi
from testground_amd import workloads as wl
from testground_amd.engine import EngineError

N, FLOODS, DEG = 600, 6, 8


def _philox(oracle_lib, ctr, key):
    import ctypes as C
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    oracle_lib.tgo_philox4x32_10(c, k, o)
    return list(o)


def _run(make_oracle, n=N, floods=FLOODS, windows=40):
    e = make_oracle(n, lookahead_ns=wl.GOSSIP_MIN_LAT)
    wl.configure_gossip(e, n)
    e.gossip_init(n_floods=floods, degree=DEG, msg_len=1024, start_gap_ticks=700, start_tick=0)
    W = wl.gossip_window_ticks(e)
    offered = []
    delivered = []
    import ctypes as C
    for k in range(windows):
        e.gen_gossip(W)
        pk = np.zeros(1 << 20, dtype=abi.PKT_DTYPE)
        m = e._lib.tgo_offered(e._h, pk.ctypes.data, len(pk))
        pk = pk[:m].copy()
        pk_abs = pk["tick"].astype(np.int64) + k * W
        offered.append((pk, pk_abs))
        e.step(W)
        delivered.append(e.drain())
    return e, W, offered, delivered


def test_gossip_reachability_and_first_receipt(oracle_lib, make_oracle):
    e, W, offered, delivered = _run(make_oracle)
    key = [wl.SEED & 0xFFFFFFFF, wl.SEED >> 32]
    gk = [key[0] ^ 0x3C6EF372, key[1] ^ 0xA54FF53A]
    thr = oracle_lib.tgo_percentage2u32(1.0)

    def nbr(p, k):
        d = _philox(oracle_lib, [p, k, 0x474F5350, 0], gk)[0] % (N - 1)
        return d + (d >= p)

    nb = [[nbr(p, k) for k in range(DEG)] for p in range(N)]
    reached = e.gossip_reached()
    for f in range(FLOODS):
        origin = _philox(oracle_lib, [f, 0, 0x4F524947, 0], gk)[0] % N
        seen = {origin}
        stack = [origin]
        while stack:
            p = stack.pop()
            for k, q in enumerate(nb[p]):
                lost = thr >= _philox(oracle_lib, [p, q, f * DEG + k, 0], key)[1]
                if not lost and q not in seen:
                    seen.add(q)
                    stack.append(q)
        assert reached[f] == len(seen), f"flood {f}: {reached[f]} reached vs BFS {len(seen)}"
        assert len(seen) > 0.99 * N

    allp = np.concatenate([p for p, _ in offered])
    ticks = np.concatenate([t for _, t in offered])
    alld = np.concatenate(delivered)
    assert len(alld) > 0
    # every (src, flood) forwards exactly once, to its hashed neighbours
    flood = allp["seq"] // DEG
    k = allp["seq"] % DEG
    pairs = allp["src"].astype(np.int64) * 64 + flood
    u, cnt = np.unique(pairs, return_counts=True)
    assert (cnt == DEG).all()
    assert sum(reached) == len(u)
    nb_arr = np.array(nb)
    assert (allp["dst"] == nb_arr[allp["src"], k]).all()
    # forward tick = tick after the earliest receipt (origins: their start tick)
    first = {}
    rf = alld["seq"] // DEG
    rt = alld["t_ns"] // 1000 + 1
    for dst, f, t in zip(alld["dst"], rf, rt):
        key_ = int(dst) * 64 + int(f)
        if key_ not in first or t < first[key_]:
            first[key_] = int(t)
    for s, f, t in zip(allp["src"], flood, ticks):
        key_ = int(s) * 64 + int(f)
        if key_ in first:
            assert t == first[key_] or t == 700 * int(f), (s, f, t, first[key_])
        else:
            assert t == 700 * int(f)  # the origin


def test_gossip_window_longer_than_lookahead_is_rejected(make_oracle):
    e = make_oracle(200, lookahead_ns=wl.GOSSIP_MIN_LAT)
    wl.configure_gossip(e, 200)
    e.gossip_init(n_floods=2, degree=4, msg_len=512, start_tick=0)
    W = 2 * wl.gossip_window_ticks(e)  # receipts land inside windows already simulated
    with pytest.raises(EngineError, match="precedes the window"):
        for _ in range(20):
            e.gen_gossip(W)
            e.step(W)


def _late_run(e):
    """Windows twice the lookahead: a receipt lands before a later window.  Returns the index of the
    window whose gen or step failed, the flood state then, and whether the error stayed."""
    wl.configure_gossip(e, 200)
    e.gossip_init(n_floods=2, degree=4, msg_len=512, start_tick=0)
    W = 2 * wl.gossip_window_ticks(e)
    for k in range(20):
        try:
            e.gen_gossip(W)  # the oracle fails here; the HIP engine, generating ahead, at the step
            e.step(W)
        except EngineError as err:
            assert "precedes the window" in str(err)
            break
    else:
        raise AssertionError("no late receipt in 20 windows")
    reached = e.gossip_reached()
    with pytest.raises(EngineError, match="preceded an earlier window"):
        e.gen_gossip(W)  # sticky until gossip_init
    assert (e.gossip_reached() == reached).all()
    e.gossip_init(n_floods=2, degree=4, msg_len=512, start_tick=e.stats()["now_tick"] + 1)
    e.gen_gossip(wl.gossip_window_ticks(e))  # a new flood runs again
    e.step(wl.gossip_window_ticks(e))
    return k, reached


@pytest.mark.gpu
def test_gossip_late_receipt_gpu_equals_oracle(make_oracle):
    """the late window changes no peer's forwarded floods on either engine (the HIP
    engine's write kernels see the flag its count kernel set), the error is sticky until
    tgsim_gossip_init, and both engines fail at the same window with the same flood state."""
    from testground_amd.engine import Engine

    k_cpu, r_cpu = _late_run(make_oracle(200, lookahead_ns=wl.GOSSIP_MIN_LAT))
    gpu = Engine(200, lookahead_ns=wl.GOSSIP_MIN_LAT)
    k_gpu, r_gpu = _late_run(gpu)
    gpu.close()
    assert k_gpu == k_cpu
    assert (r_gpu == r_cpu).all()


def test_gossip_late_receipt_is_sticky_on_oracle(make_oracle):
    _late_run(make_oracle(200, lookahead_ns=wl.GOSSIP_MIN_LAT))


def _late_run_ahead(e, depth):
    """windows generated `depth` ahead of the steps (the bench's rotation), twice the
    lookahead long, so a receipt precedes a generated window.  The late window is reported by the
    call that resolves it (its step, or the next gen_gossip); it and anything queued after it are
    dropped, the valid windows before it stay queued and step normally.  Returns every call's
    outcome, with each step's deliveries."""
    import hashlib

    wl.configure_gossip(e, 200)
    e.gossip_init(n_floods=2, degree=4, msg_len=512, start_tick=0)
    W = 2 * wl.gossip_window_ticks(e)
    ev, failed_at = [], None

    def call(kind, fn):
        try:
            fn()
        except EngineError as err:
            msg = str(err)
            ev.append((kind, "late" if "precedes the window" in msg else "sticky" if "preceded an earlier" in msg else msg))
            return False
        if kind == "step":
            d = e.drain()
            ev.append((kind, len(d), hashlib.sha256(d.tobytes()).hexdigest()[:16], e.stats()["now_tick"]))
        else:
            ev.append((kind, "ok"))
        return True

    for _ in range(depth):
        call("gen", lambda: e.gen_gossip(W))
    for k in range(30):
        ok = call("step", lambda: e.step(W))
        ok = call("gen", lambda: e.gen_gossip(W)) and ok
        if not ok and failed_at is None:
            failed_at = k
        if failed_at is not None and k >= failed_at + depth + 1:
            break
    assert failed_at is not None, "no late receipt in 30 windows"
    return ev


@pytest.mark.parametrize("depth", [2, 3])
def test_gossip_late_receipt_ahead_on_oracle(make_oracle, depth):
    ev = _late_run_ahead(make_oracle(200, lookahead_ns=wl.GOSSIP_MIN_LAT), depth)
    first = next(i for i, x in enumerate(ev) if x[1] == "late")
    # every window generated before the late one was stepped, with deliveries, before the report or after it
    steps_ok = [x for x in ev if x[0] == "step" and x[1] not in ("late", "sticky")]
    assert len(steps_ok) >= depth and all(isinstance(x[1], int) for x in steps_ok)
    assert ev.count(("gen", "late")) + ev.count(("step", "late")) == 1, ev  # reported once
    assert all(x[1] == "sticky" for x in ev[first + 1:] if x[0] == "gen"), ev  # then sticky


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [2, 3])
def test_gossip_late_receipt_ahead_gpu_equals_oracle(make_oracle, depth):
    """The same calls on the HIP engine and the oracle: the same outcome at every call (which call
    reports the late window, which windows still step) and the same deliveries at every step."""
    from testground_amd.engine import Engine

    cpu = _late_run_ahead(make_oracle(200, lookahead_ns=wl.GOSSIP_MIN_LAT), depth)
    gpu_e = Engine(200, lookahead_ns=wl.GOSSIP_MIN_LAT)
    gpu = _late_run_ahead(gpu_e, depth)
    gpu_e.close()
    assert gpu == cpu


def test_gossip_init_contract(make_oracle):
    e = make_oracle(10)
    for bad in (dict(n_floods=0), dict(n_floods=65), dict(degree=0), dict(degree=65), dict(msg_len=0)):
        kw = dict(n_floods=1, degree=1, msg_len=100, start_tick=0)
        kw.update(bad)
        with pytest.raises(EngineError):
            e.gossip_init(**kw)
