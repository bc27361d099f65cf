"""The local sync endpoint (testground_amd/sync_service.py): plan instances in
processes of their own meet at barriers and exchange topic entries through it, with the signal and
barrier counters in the engine (sidecar.EngineSyncClient: tgsim_signal / tgsim_barrier_poll), while
their datagrams cross the simulated network through the native UDP front end.  The wire format is
this engine's own (parity-unpinned: the sdk-go protocol is not in the reference); what is pinned is
the sync semantics the reference's plans rely on -- 1-based SignalEntry sequence numbers, a barrier
that releases when its state's count reaches the target, pub/sub with the topic's history
(sidecar_handler.go:40-44, :75-80; plans/network/pingpong.go:64-67)."""
import json
import subprocess
import sys
import threading
import time
from pathlib import Path

import pytest

from testground_amd import network as nw
from testground_amd.sidecar import Context, EngineSyncClient, SyncClient
from testground_amd.sync_service import SyncService, SyncServiceClient

WINDOW = 1000  # ticks of 1 us


def test_sync_service_semantics():
    """Signal sequence numbers, barrier release, SignalAndWait, pub/sub history, errors: one service
    over the in-memory client, two client connections (two plan instances)."""
    svc = SyncService(SyncClient())
    a, b = SyncServiceClient(svc.address, timeout_s=5), SyncServiceClient(svc.address, timeout_s=5)
    try:
        assert a.SignalEntry("s") == 1 and b.SignalEntry("s") == 2
        a.Barrier("s", 2)  # reached
        assert a.Publish("t", {"k": 1}) == 1
        sub = b.Subscribe("t")
        assert sub.get(timeout=5) == {"k": 1}  # the history first
        assert b.Publish("t", [2, 3]) == 2
        assert sub.get(timeout=5) == [2, 3]
        done = {}
        th = threading.Thread(target=lambda: done.setdefault("seq", a.SignalAndWait("both", 2)))
        th.start()
        time.sleep(0.1)
        assert "seq" not in done  # waits for the second instance
        assert b.SignalAndWait("both", 2) in (1, 2)
        th.join(timeout=5)
        assert done["seq"] in (1, 2)
        short = SyncServiceClient(svc.address, timeout_s=0.2)
        with pytest.raises(RuntimeError, match="barrier"):
            short.Barrier("never", 1)
        short.Close()
    finally:
        a.Close()
        b.Close()
        svc.close()


def _run_two_plans(engine, n_msgs=12, lat_ms=3):
    """Two plan processes (tests/sync_plan.py) over the engine: they publish their data ports, the
    harness (the runner's role) registers them with the front end and signals `network-initialized`
    once per instance, they exchange datagrams through the simulated link and meet at `done`."""
    from testground_amd.bridge import NativeBridge, NativeUdpFront

    n = 2
    for i in range(n):
        engine.configure(i, nw.Config(Network="default", Enable=True, Default=nw.LinkShape(Latency=lat_ms * nw.Millisecond)))
    bridge = NativeBridge(engine, n, WINDOW)
    front = NativeUdpFront(bridge)
    lock = threading.Lock()  # the engine is driven by the pump below and by the service's threads
    sync = EngineSyncClient(engine, lock=lock)
    svc = SyncService(sync)
    vaddr = [front.bind_peer(i) for i in range(n)]
    procs = [subprocess.Popen([sys.executable, str(Path(__file__).with_name("sync_plan.py")), svc.address[0],
                               str(svc.address[1]), str(i), str(n), vaddr[1 - i][0], str(vaddr[1 - i][1]),
                               str(n_msgs)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for i in range(n)]
    ctx = Context()
    ports = sync.Subscribe(ctx, "ports")
    registered = 0
    try:
        deadline = time.time() + 90
        while any(p.poll() is None for p in procs) and time.time() < deadline:
            with lock:
                front.pump()
            while not ports.empty():
                p = ports.get_nowait()
                front.register(int(p["instance"]), ("127.0.0.1", int(p["port"])))
                registered += 1
                if registered == n:  # every instance's network is up: the sidecar's signal
                    for _ in range(n):
                        sync.SignalEntry(ctx, "network-initialized")
            time.sleep(0.002)
        outs = [p.communicate(timeout=10) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        svc.close()
        front.close()
    assert [p.returncode for p in procs] == [0, 0], [o[1][-2000:] for o in outs]
    res = [json.loads(o[0].strip().splitlines()[-1]) for o in outs]
    for r in res:
        me = r["instance"]
        assert sorted(d for d, _ in r["got"]) == sorted("from-%d-msg-%03d" % (1 - me, k) for k in range(n_msgs))
        assert all(tuple(a) == tuple(vaddr[1 - me]) for _, a in r["got"])  # from the peer's data address
    assert sorted(r["done_seq"] for r in res) == [1, 2]
    # the counters are the engine's: both states reached their targets on the device table
    with lock:
        assert engine.barrier_poll(sync.state_id("network-initialized"), n)
        assert engine.barrier_poll(sync.state_id("done"), n)


def test_two_plan_processes_through_sync_service(make_oracle):
    _run_two_plans(make_oracle(2, lookahead_ns=WINDOW * 1000))


@pytest.mark.gpu
def test_two_plan_processes_through_sync_service_gpu():
    """The same over the HIP engine: the barriers are the device counters (K7)."""
    import torch

    from testground_amd.engine import Engine

    if torch.cuda.is_available():
        torch.cuda.init()
    _run_two_plans(Engine(2, lookahead_ns=WINDOW * 1000))
