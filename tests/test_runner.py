"""`local:mi355x-sim` runner (testground_amd/runner.py): plans run as simulated instances of one
engine.  CPU tests drive the runner over the CPU oracle (the checker) through the runner's
engine_factory; the GPU test runs the same plan on the HIP engine and compares the results."""
import io
import ipaddress
import tarfile

import pytest

from testground_amd import network as nw
from testground_amd import runner as rn
from testground_amd import workloads as wl
from testground_amd.sidecar import Context


def pingpong_plan(env: rn.PlanEnv) -> None:
    """plans/network/pingpong.go:23-187 on the simulated data plane: configure 100 ms latency and
    1 Mibit/s (callback "network-configured"), re-address to subnet.a.b.((seq>>8)+1).seq/12
    (callback "ip-changed", :54-81; the sidecar reconnects the instance) and exchange the new
    addresses over the "peers" topic (:204-244), ping-pong with RTT in [200, 215] ms
    (pingpong.go:185), reconfigure to 10 ms (callback "latency-reduced", :191-194), RTT in
    [20, 35] ms (:195).  Round-trip times go to rtt.txt in the instance's outputs dir."""
    env.net.WaitNetworkInitialized(env.ctx)
    peer = 1 - env.seq
    rtts = []

    def ping_pong(lo_ms, hi_ms):
        env.sync.SignalAndWait(env.ctx, f"ready-{lo_ms}", env.runenv.TestInstanceCount)
        t0 = env.data.now_ns()
        env.data.send(peer, bytes([env.seq]))
        got_own = got_other = False
        while not (got_own and got_other):
            for t_ns, src, data, _f in env.data.recv(timeout_ns=10 * 10**9):
                if data[0] == env.seq:
                    rtt = t_ns - t0
                    rtts.append(rtt)
                    if not lo_ms * nw.Millisecond <= rtt <= hi_ms * nw.Millisecond:
                        raise AssertionError(f"expected an RTT between {lo_ms} and {hi_ms} ms, got {rtt} ns")
                    got_own = True
                else:
                    env.data.send(src, data, at_ns=t_ns)  # echo at the arrival time
                    got_other = True
        env.sync.SignalAndWait(env.ctx, f"done-{lo_ms}", env.runenv.TestInstanceCount)

    cfg = wl.pingpong_config(100 * nw.Millisecond)
    env.net.ConfigureNetwork(env.ctx, cfg)
    n = env.runenv.TestInstanceCount
    seq = env.sync.SignalAndWait(env.ctx, "ip-allocation", n)
    net = ipaddress.IPv4Network(env.runenv.TestSubnet, strict=False).network_address.packed
    ip = ipaddress.IPv4Address(bytes([net[0], net[1], (seq >> 8) + 1, seq & 0xFF]))
    cfg.IPv4 = (str(ip), 12)
    cfg.CallbackState = "ip-changed"
    env.net.ConfigureNetwork(env.ctx, cfg)
    own = env.net.GetDataNetworkIP()
    assert own == str(ip), (own, ip)
    env.sync.SignalAndWait(env.ctx, "listening", n)
    q = env.sync.PublishSubscribe(env.ctx, "peers", own)
    addrs = [q.get() for _ in range(n)]
    assert len(set(addrs)) == n and own in addrs
    env.sync.SignalAndWait(env.ctx, "got-other-addrs", n)
    ping_pong(200, 215)
    cfg.Default.Latency = 10 * nw.Millisecond
    cfg.CallbackState = "latency-reduced"
    env.net.ConfigureNetwork(env.ctx, cfg)
    ping_pong(20, 35)
    with open(f"{env.runenv.TestOutputsPath}/rtt.txt", "w") as f:
        f.write(" ".join(map(str, rtts)))


def failing_plan(env: rn.PlanEnv) -> None:
    if env.group_seq == 1:
        raise RuntimeError("boom")


def sleeper_plan(env: rn.PlanEnv) -> None:
    env.data.sleep(int(env.runenv.TestInstanceParams["sleep_ms"]) * nw.Millisecond)


def _job(run_id, groups, cfg):
    return rn.RunInput(RunID=run_id, TestPlan="network", TestCase="ping-pong",
                       TotalInstances=sum(g.Instances for g in groups), Groups=groups, RunnerConfig=cfg)


def _cfg(tmp_path, factory, **kw):
    return rn.LocalSimRunnerCfg(outputs_dir=str(tmp_path), engine_factory=factory, run_timeout_s=60, **kw)


def _rtts(tmp_path, run_id):
    return [open(tmp_path / "network" / run_id / "single" / str(i) / "rtt.txt").read() for i in (0, 1)]


def test_runner_surface():
    r = rn.LocalSimRunner()
    assert r.ID() == "local:mi355x-sim"
    assert r.ConfigType() is rn.LocalSimRunnerCfg
    assert r.CompatibleBuilders() == ["exec:py"]
    res = rn.Result(Outcome=rn.OUTCOME_SUCCESS, Outcomes={"a": rn.GroupOutcome(2, 3)})
    assert str(res) == "outcome = success (a:2/3)"


def test_runner_rejects_bad_input(tmp_path, make_oracle):
    r = rn.LocalSimRunner()
    g = [rn.RunGroup("single", 2, pingpong_plan)]
    job = _job("bad", g, _cfg(tmp_path, make_oracle))
    job.TotalInstances = 3
    with pytest.raises(ValueError, match="TotalInstances"):
        r.Run(Context(), job)
    with pytest.raises(ValueError, match="artifact"):
        r.Run(Context(), _job("bad2", [rn.RunGroup("single", 2, "not a plan")], _cfg(tmp_path, make_oracle)))


def test_runner_pingpong_over_oracle(tmp_path, make_oracle):
    """The reference's ping-pong test case as a plan: two instances, sidecar-applied shapes,
    both RTT windows met; the run is reproducible and its outputs can be collected."""
    r = rn.LocalSimRunner()
    outs = []
    for run_id in ("r1", "r2"):
        out = r.Run(Context(), _job(run_id, [rn.RunGroup("single", 2, pingpong_plan)], _cfg(tmp_path, make_oracle)))
        assert out.Result.Outcome == rn.OUTCOME_SUCCESS, out.Result.Errors
        assert str(out.Result.Outcomes["single"]) == "2/2"
        outs.append(_rtts(tmp_path, run_id))
    assert outs[0] == outs[1]  # conservative clock: same simulated times every run
    buf = io.BytesIO()
    r.CollectOutputs(Context(), rn.CollectionInput("r1", "network"), buf, _cfg(tmp_path, make_oracle))
    names = tarfile.open(fileobj=io.BytesIO(buf.getvalue()), mode="r:gz").getnames()
    assert "r1/single/0/rtt.txt" in names and "r1/run.json" in names


def test_runner_outcomes_per_group(tmp_path, make_oracle):
    """cluster_k8s.go:1235-1245: the run fails unless every group has ok == total."""
    r = rn.LocalSimRunner()
    g = [rn.RunGroup("good", 2, sleeper_plan, {"sleep_ms": "5"}), rn.RunGroup("bad", 2, failing_plan)]
    out = r.Run(Context(), _job("mixed", g, _cfg(tmp_path, make_oracle)))
    assert out.Result.Outcome == rn.OUTCOME_FAILURE
    assert str(out.Result.Outcomes["good"]) == "2/2" and str(out.Result.Outcomes["bad"]) == "1/2"
    assert "boom" in out.Result.Errors["bad[001]"]
    assert out.Result.SimulatedNs >= 5 * nw.Millisecond


def test_runner_sim_time_cap(tmp_path, make_oracle):
    r = rn.LocalSimRunner()
    cfg = _cfg(tmp_path, make_oracle, max_sim_ns=20 * nw.Millisecond)
    out = r.Run(Context(), _job("cap", [rn.RunGroup("g", 1, sleeper_plan, {"sleep_ms": "100"})], cfg))
    assert out.Result.Outcome != rn.OUTCOME_SUCCESS
    assert "simulation stopped" in out.Result.Errors["g[000]"]


@pytest.mark.gpu
def test_runner_pingpong_gpu_equals_oracle(tmp_path, make_oracle):
    """The ping-pong plan on the HIP engine (the runner's default engine): success, and the same
    round-trip times as over the oracle."""
    import torch
    assert torch.cuda.is_available()
    r = rn.LocalSimRunner()
    gpu = r.Run(Context(), _job("gpu", [rn.RunGroup("single", 2, pingpong_plan)], _cfg(tmp_path, None)))
    assert gpu.Result.Outcome == rn.OUTCOME_SUCCESS, gpu.Result.Errors
    cpu = r.Run(Context(), _job("cpu", [rn.RunGroup("single", 2, pingpong_plan)], _cfg(tmp_path, make_oracle)))
    assert cpu.Result.Outcome == rn.OUTCOME_SUCCESS, cpu.Result.Errors
    assert _rtts(tmp_path, "gpu") == _rtts(tmp_path, "cpu")


def splitbrain_plan(case: str, ok: dict):
    """plans/splitbrain/main.go:61-180 as a plan: sequence numbers from SignalEntry give the
    region (seq % 3, :84-87); region-A instances install one /32 rule per region-B instance with
    the case's action through ConfigureNetwork (callback "reconfigured<seq>", target 1,
    :101-140); then every instance contacts every other one and answers every request it gets.
    ok[(i, j)] = instance i got j's answer; the expectation is expectErrors (:50-58)."""
    def plan(env: rn.PlanEnv) -> None:
        n = env.runenv.TestInstanceCount
        env.net.WaitNetworkInitialized(env.ctx)
        seq = env.sync.SignalEntry(env.ctx, "ip-allocation")
        env.sync.Publish(env.ctx, "nodes", (env.seq, seq % 3))
        env.sync.SignalAndWait(env.ctx, "published", n)
        q = env.sync.Subscribe(env.ctx, "nodes")
        region = dict(q.get_nowait() for _ in range(n))
        if region[env.seq] == wl.REGION_A:
            action = {"drop": nw.FilterAction.Drop, "reject": nw.FilterAction.Reject,
                      "accept": nw.FilterAction.Accept}[case]
            rules = [nw.LinkRule(Subnet=(str(ipaddress.IPv4Address(wl.peer_ip(p))), 32),
                                 LinkShape=nw.LinkShape(Filter=action))
                     for p, r in sorted(region.items()) if r == wl.REGION_B]
            env.net.ConfigureNetwork(env.ctx, nw.Config(
                Network="default", Enable=True, Default=nw.LinkShape(Latency=nw.Millisecond),
                Rules=rules, CallbackState=f"reconfigured{seq}", CallbackTarget=1))
        env.sync.SignalAndWait(env.ctx, "configured", n)
        for p in range(n):
            if p != env.seq:
                env.data.send(p, b"Q")
        deadline = env.data.now_ns() + 50 * nw.Millisecond
        while env.data.now_ns() < deadline:
            for t_ns, src, data, _f in env.data.recv(timeout_ns=deadline - env.data.now_ns()):
                if data == b"Q":
                    env.data.send(src, b"A", at_ns=t_ns)
                else:
                    ok[(env.seq, src)] = region
    return plan


@pytest.mark.parametrize("case", ["accept", "reject", "drop"])
def test_runner_splitbrain_over_oracle(tmp_path, make_oracle, case):
    n = 9
    ok = {}
    r = rn.LocalSimRunner()
    out = r.Run(Context(), _job(f"sb-{case}", [rn.RunGroup("all", n, splitbrain_plan(case, ok))],
                                _cfg(tmp_path, make_oracle)))
    assert out.Result.Outcome == rn.OUTCOME_SUCCESS, out.Result.Errors
    region = next(iter(ok.values()))
    for i in range(n):
        for j in range(n):
            if i != j:
                reachable = not wl.expect_errors(case, region[i], region[j])
                assert ((i, j) in ok) == reachable, (case, i, j, region[i], region[j])


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["reject", "drop"])
def test_runner_splitbrain_gpu(tmp_path, case):
    """The splitbrain plan on the HIP engine: rules applied by the sidecar handler on the device
    filter exactly the region A <-> B pairs."""
    import torch
    assert torch.cuda.is_available()
    n = 9
    ok = {}
    out = rn.LocalSimRunner().Run(Context(), _job(f"sbg-{case}", [rn.RunGroup("all", n, splitbrain_plan(case, ok))],
                                                  _cfg(tmp_path, None)))
    assert out.Result.Outcome == rn.OUTCOME_SUCCESS, out.Result.Errors
    region = next(iter(ok.values()))
    for i in range(n):
        for j in range(n):
            if i != j:
                assert ((i, j) in ok) == (not wl.expect_errors(case, region[i], region[j])), (i, j)


def test_runner_healthcheck(tmp_path, make_oracle):
    """healthcheck.go:13-56: the outputs dir check is fixed by creating it; checks that pass
    report their fix as unnecessary; the engine checks pass with a working engine."""
    r = rn.LocalSimRunner()
    cfg = rn.LocalSimRunnerCfg(outputs_dir=str(tmp_path / "out"), engine_factory=make_oracle)
    rep = r.Healthcheck(Context(), fix=False, cfg=cfg)
    st = {c.Name: c.Status for c in rep.Checks}
    # the run would not load libtgsim.so with an engine_factory: that check is omitted
    assert st == {"outputs-dir": rn.HEALTH_FAILED, "engine-library": rn.HEALTH_OMITTED,
                  "engine-device": rn.HEALTH_OK}
    assert not rep.ChecksSucceeded() and rep.Fixes == []
    rep = r.Healthcheck(Context(), fix=True, cfg=cfg)
    assert [f.Status for f in rep.Fixes] == [rn.HEALTH_OK, rn.HEALTH_UNNECESSARY, rn.HEALTH_UNNECESSARY]
    assert r.Healthcheck(Context(), cfg=cfg).ChecksSucceeded()


def subscriber_plan(env: rn.PlanEnv) -> None:
    """One instance publishes after sleeping in simulated time; the other blocks in a topic get(),
    which waits through the clock (so the publisher's sleep can advance time)."""
    if env.seq == 0:
        env.data.sleep(3 * nw.Millisecond)
        env.sync.Publish(env.ctx, "t", {"at": env.data.now_ns()})
    else:
        got = env.sync.Subscribe(env.ctx, "t").get()
        assert got["at"] >= 3 * nw.Millisecond


def test_runner_clocked_subscription(tmp_path, make_oracle):
    r = rn.LocalSimRunner()
    out = r.Run(Context(), _job("sub", [rn.RunGroup("g", 2, subscriber_plan)], _cfg(tmp_path, make_oracle)))
    assert out.Result.Outcome == rn.OUTCOME_SUCCESS, out.Result.Errors


def test_runner_clock_readiness_error_fails_fast(tmp_path, make_oracle):
    """A readiness check that raises (here: a barrier poll on a broken engine) stops the run with
    the cause instead of leaving every instance waiting for run_timeout."""
    import time

    def broken(n, **kw):
        e = make_oracle(n, **kw)

        def boom(*a, **k):
            raise RuntimeError("barrier poll exploded")
        e.barrier_poll = boom
        return e

    def plan(env):
        env.sync.Barrier(env.ctx, "never", 5)

    cfg = _cfg(tmp_path, broken)
    cfg.run_timeout_s = 30
    t0 = time.monotonic()
    out = rn.LocalSimRunner().Run(Context(), _job("boom", [rn.RunGroup("g", 2, plan)], cfg))
    assert out.Result.Outcome != rn.OUTCOME_SUCCESS
    assert time.monotonic() - t0 < 20
    assert any("exploded" in e for e in out.Result.Errors.values()), out.Result.Errors


def endpoint_plan(env: rn.PlanEnv) -> None:
    """Plan code that reaches the run's sync counters through the run's sync endpoint (as code in
    another process would, sync_service.SyncServiceClient over RunParams.SyncServiceHost/Port) and
    meets the other instance there; the in-process view of the same state agrees."""
    from testground_amd.sync_service import SyncServiceClient

    rp = env.runenv
    assert rp.SyncServiceHost and rp.SyncServicePort
    c = SyncServiceClient((rp.SyncServiceHost, rp.SyncServicePort), timeout_s=20)
    try:
        seq = c.SignalEntry("via-endpoint")
        assert 1 <= seq <= rp.TestInstanceCount
        c.Barrier("via-endpoint", rp.TestInstanceCount)
    finally:
        c.Close()


def test_runner_serves_sync_endpoint(tmp_path, make_oracle):
    out = rn.LocalSimRunner().Run(Context(), _job("ep", [rn.RunGroup("g", 2, endpoint_plan)], _cfg(tmp_path, make_oracle)))
    assert out.Result.Outcome == rn.OUTCOME_SUCCESS, out.Result.Errors
