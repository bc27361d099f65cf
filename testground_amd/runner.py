"""`local:mi355x-sim`: a runner whose instances are simulated peers of one engine (SURVEY §8(f)
rank 3, first form).

Mirrors the reference's runner plugin surface, with the same names and meaning:

  Runner{ID, Run, ConfigType, CompatibleBuilders, CollectOutputs}   pkg/api/runner.go:17-34
  RunInput / RunGroup / RunOutput / CollectionInput                  pkg/api/runner.go:37-115
  Terminatable.TerminateAll                                           pkg/api/runner.go:117-121
  Result{Outcome, Outcomes}, GroupOutcome{Ok, Total} ("ok/total")     pkg/runner/cluster_k8s.go:144-161
  outcome rule: success iff every group has Ok == Total and there is
  at least one group                                                  pkg/runner/cluster_k8s.go:1235-1245
  per-instance run params and outputs dir <outputs>/<plan>/<run>/<group>/<i>
                                                                      pkg/runner/local_exec.go:78-140

Where `local:exec` starts one OS process per instance (local_exec.go:117-166), this runner starts
one thread per instance and gives each a simulated data interface: its datagrams go through the
engine (`PacketBridge`), its network configuration through the sidecar handler
(`sidecar.handler` over `SimNetwork`, TestSidecar = true), its sync calls to the engine's sync
counters (`EngineSyncClient`).  An instance "succeeds" when its plan function returns, as sdk-go's
run.Invoke records success on a nil return and failure on an error or panic.

Simulated time is advanced conservatively, so a run is reproducible: the clock steps the engine
one window only when every live instance is blocked (in `DataPlane.recv`/`sleep` or a sync
barrier) and none of them could go on; an instance inside ConfigureNetwork is never blocked, so a
configuration is applied before the next window is simulated.  Replies sent at a delivery's time
need the engine's lookahead to cover one window, which `Run` sets.
"""
from __future__ import annotations

import dataclasses
import io
import json
import os
import queue
import tarfile
import tempfile
import threading
import time
from typing import Callable, Dict, List, Optional, Tuple

from .bridge import NativeBridge, PacketBridge
from .engine import LIB_PATH, EngineError
from .sidecar import Context, NetClient, SimReactor, SyncClient, handler
from .sync_service import SyncService

OUTCOME_UNKNOWN = "unknown"     # pkg/task/task.go:25-28
OUTCOME_SUCCESS = "success"
OUTCOME_FAILURE = "failure"
OUTCOME_CANCELED = "canceled"


@dataclasses.dataclass
class RunGroup:
    """api.RunGroup (runner.go:65-85).  ArtifactPath is the plan: a callable taking a `PlanEnv`,
    or a "module:function" string naming one (the exec:py builder's artifact)."""
    ID: str
    Instances: int
    ArtifactPath: object = None
    Parameters: Dict[str, str] = dataclasses.field(default_factory=dict)


@dataclasses.dataclass
class RunInput:
    """api.RunInput (runner.go:37-63)."""
    RunID: str
    TestPlan: str
    TestCase: str
    TotalInstances: int
    Groups: List[RunGroup]
    RunnerConfig: Optional["LocalSimRunnerCfg"] = None
    DisableMetrics: bool = False


@dataclasses.dataclass
class GroupOutcome:
    Ok: int = 0
    Total: int = 0

    def __str__(self) -> str:
        return f"{self.Ok}/{self.Total}"


@dataclasses.dataclass
class Result:
    Outcome: str = OUTCOME_UNKNOWN
    Outcomes: Dict[str, GroupOutcome] = dataclasses.field(default_factory=dict)
    Errors: Dict[str, str] = dataclasses.field(default_factory=dict)  # "<group>[<i>]" -> error
    SimulatedNs: int = 0

    def StringOutcomes(self) -> str:
        return " ".join(f"{g}:{o}" for g, o in sorted(self.Outcomes.items()))

    def __str__(self) -> str:
        return f"outcome = {self.Outcome} ({self.StringOutcomes()})"


@dataclasses.dataclass
class RunOutput:
    """api.RunOutput (runner.go:87-101)."""
    RunID: str
    Result: Result


@dataclasses.dataclass
class CollectionInput:
    """api.CollectionInput (runner.go:103-115)."""
    RunID: str
    TestPlan: str
    RunnerID: str = "local:mi355x-sim"


@dataclasses.dataclass
class RunParams:
    """The subset of sdk-go runtime.RunParams the runner fills per instance (local_exec.go:82-90,
    :125-131)."""
    TestPlan: str
    TestCase: str
    TestRun: str
    TestInstanceCount: int
    TestGroupID: str
    TestGroupInstanceCount: int
    TestInstanceParams: Dict[str, str]
    TestOutputsPath: str
    TestSidecar: bool = True
    TestSubnet: str = "16.0.0.0/8"
    TestStartTime: float = 0.0
    # the run's sync endpoint (sdk-go runenv SYNC_SERVICE_HOST/PORT, set by local_common.go:77-82's
    # sync-service container in the reference): out-of-process plan code reaches the run's sync
    # counters through it (sync_service.SyncServiceClient)
    SyncServiceHost: str = ""
    SyncServicePort: int = 0


@dataclasses.dataclass
class LocalSimRunnerCfg:
    """Runner configuration (the manifest's [runners."local:mi355x-sim"] table)."""
    outputs_dir: str = ""
    window_ticks: int = 1000
    tick_ns: int = 1000
    seed: int = 0x7E576A0D00000001
    queue_limit: int = 0
    max_instances: int = 1 << 20
    run_timeout_s: float = 120.0
    max_sim_ns: int = 3600 * 10**9
    # engine_factory(n_peers, **engine kwargs) -> engine; default: the HIP engine (engine.Engine)
    engine_factory: Optional[Callable] = None
    sync_service: bool = True  # serve the run's sync counters on a loopback port (sync_service.py)


def _make_bridge(engine, n: int, cfg):
    """The native bridge (libtgsim's tgsim_bridge_*): always with the HIP engine, which needs the
    library anyway (a failure to load it is the run's failure).  An engine_factory engine (the
    oracle in the CPU tests) falls back to the Python PacketBridge when libtgsim.so is absent or
    cannot be loaded on this host (no HIP runtime)."""
    if cfg.engine_factory is None:
        return NativeBridge(engine, n, cfg.window_ticks, cfg.tick_ns)
    if LIB_PATH.exists():
        try:
            return NativeBridge(engine, n, cfg.window_ticks, cfg.tick_ns)
        except (OSError, AttributeError, EngineError):
            pass
    return PacketBridge(engine, n, cfg.window_ticks, cfg.tick_ns)


class _Clock:
    """Conservative time advance: steps the bridge one window when every live instance is blocked
    and no blocked instance is ready to continue."""

    def __init__(self, bridge: PacketBridge, lock: threading.Lock, n: int, ctx: Context, max_sim_ns: int):
        self.bridge = bridge
        self.lock = lock
        self.ctx = ctx
        self.max_sim_ns = max_sim_ns
        self._mu = threading.Lock()
        self.cv = threading.Condition(self._mu)                            # the clock waits here
        self.pcv = [threading.Condition(self._mu) for _ in range(n)]       # instance p waits here
        self.live = set(range(n))
        self.waiting: Dict[int, Callable[[], bool]] = {}
        self.inbox: List[List[Tuple[int, int, bytes, int]]] = [[] for _ in range(n)]
        self.error: Optional[BaseException] = None

    def now_ns(self) -> int:
        return self.bridge.now_tick * self.bridge.tick_ns

    def block(self, peer: int, ready: Callable[[], bool]) -> None:
        with self.cv:
            self.waiting[peer] = ready
            self.cv.notify_all()
            try:
                while not ready():
                    if self.error is not None:
                        raise RuntimeError(f"simulation stopped: {self.error}")
                    if self.ctx.done():
                        raise TimeoutError(f"instance {peer}: {self.ctx.err()}")
                    self.pcv[peer].wait(timeout=0.05)
            finally:
                del self.waiting[peer]

    def kick(self) -> None:
        """Wakes every blocked instance to re-check (after a sync signal)."""
        with self.cv:
            for c in self.pcv:
                c.notify()
            self.cv.notify_all()

    def finish(self, peer: int) -> None:
        with self.cv:
            self.live.discard(peer)
            self.cv.notify_all()

    def _fail(self, e: BaseException) -> None:
        """Stops the clock with `e`, surfaced to every instance (called with the lock held)."""
        self.error = e
        for c in self.pcv:
            c.notify()

    def run(self) -> None:
        with self.cv:
            while self.live and not self.ctx.done():
                try:  # readiness checks call into the engine (barrier polls) and may raise too
                    if (len(self.waiting) < len(self.live)
                            or any(r() for r in self.waiting.values())):
                        self.cv.wait(timeout=0.005)
                        continue
                    if self.now_ns() >= self.max_sim_ns:
                        self._fail(TimeoutError(f"simulated time reached {self.max_sim_ns} ns"))
                        return
                    with self.lock:
                        self.bridge.step()
                        for p in range(self.bridge.n):
                            for t_ns, src, _seq, data, flags in self.bridge.recv(p):
                                self.inbox[p].append((t_ns, src, data, flags))
                    for p, r in self.waiting.items():  # wake only the instances that can go on
                        if r():
                            self.pcv[p].notify()
                except BaseException as e:  # noqa: BLE001 - surfaced to every instance
                    self._fail(e)
                    return


class DataPlane:
    """An instance's simulated data interface: datagrams to other instances by instance index."""

    def __init__(self, clock: _Clock, peer: int):
        self._c = clock
        self.peer = peer

    def now_ns(self) -> int:
        """Start of the next window to be simulated (the earliest time a send can leave at)."""
        return self._c.now_ns()

    def send(self, dst: int, data: bytes, at_ns: Optional[int] = None) -> int:
        """Sends one datagram at at_ns (default: now_ns()); returns its sequence number.  A time
        already simulated (a reply to a delivery that arrived less than one window after it was
        sent, on a link shorter than the window) leaves at now_ns(): the clock cannot go back, so
        links shorter than `window_ticks` see their replies rounded up to the next window."""
        b = self._c.bridge
        with self._c.lock:
            at = None if at_ns is None else max(-(-int(at_ns) // b.tick_ns), b.now_tick)
            return b.send(self.peer, dst, data, at_tick=at)

    def recv(self, timeout_ns: Optional[int] = None) -> List[Tuple[int, int, bytes, int]]:
        """Blocks until at least one datagram has arrived, or simulated time passes timeout_ns
        from now; returns [(t_ns, src, payload, flags)] in delivery order (may be empty)."""
        box = self._c.inbox[self.peer]
        deadline = None if timeout_ns is None else self.now_ns() + int(timeout_ns)
        self._c.block(self.peer, lambda: bool(box) or (deadline is not None and self._c.now_ns() >= deadline))
        with self._c.cv:
            out = list(box)
            box.clear()
        return out

    def sleep(self, ns: int) -> None:
        deadline = self.now_ns() + int(ns)
        self._c.block(self.peer, lambda: self._c.now_ns() >= deadline)


class ClockedSync:
    """The instance's view of the sync client: barriers block through the clock."""

    def __init__(self, inner: SyncClient, clock: _Clock, peer: int):
        self.inner = inner
        self._c = clock
        self.peer = peer

    def SignalEntry(self, ctx: Context, state: str) -> int:
        seq = self.inner.SignalEntry(ctx, state)
        self._c.kick()
        return seq

    def Barrier(self, ctx: Context, state: str, target: int) -> None:
        self._c.block(self.peer, lambda: self.inner._reached(state, target))

    def SignalAndWait(self, ctx: Context, state: str, target: int) -> int:
        seq = self.SignalEntry(ctx, state)
        self.Barrier(ctx, state, target)
        return seq

    def Publish(self, ctx: Context, topic: str, payload) -> int:
        return self.inner.Publish(ctx, topic, payload)

    def Subscribe(self, ctx: Context, topic: str) -> "ClockedSubscription":
        return ClockedSubscription(self.inner.Subscribe(ctx, topic), self._c, self.peer)

    def PublishSubscribe(self, ctx: Context, topic: str, payload) -> "ClockedSubscription":
        """sdk-go PublishSubscribe (pingpong.go:225): publish, then subscribe from the start."""
        self.Publish(ctx, topic, payload)
        return self.Subscribe(ctx, topic)


class ClockedSubscription:
    """A topic subscription whose blocking get() waits through the clock (so simulated time can
    advance, and the run's context cancels it) instead of blocking a thread the clock cannot see."""

    def __init__(self, q: "queue.Queue", clock: "_Clock", peer: int):
        self._q = q
        self._c = clock
        self._peer = peer

    def get(self, block: bool = True, timeout: Optional[float] = None):
        if block:
            self._c.block(self._peer, lambda: not self._q.empty())
        return self._q.get_nowait()

    def get_nowait(self):
        return self._q.get_nowait()

    def empty(self) -> bool:
        return self._q.empty()

    def qsize(self) -> int:
        return self._q.qsize()


@dataclasses.dataclass
class PlanEnv:
    """What a plan function receives: its run params, sdk-go-shaped clients and data interface."""
    runenv: RunParams
    seq: int          # global instance index = simulated peer
    group_seq: int    # index within the group
    hostname: str
    ctx: Context
    sync: ClockedSync
    net: NetClient
    data: DataPlane


def _resolve(artifact) -> Callable[[PlanEnv], None]:
    if callable(artifact):
        return artifact
    if isinstance(artifact, str) and ":" in artifact:
        import importlib
        mod, fn = artifact.split(":", 1)
        return getattr(importlib.import_module(mod), fn)
    raise ValueError(f"artifact {artifact!r} is not a plan callable or 'module:function'")


HEALTH_OK = "ok"                 # pkg/api/healthcheck.go:20-35
HEALTH_FAILED = "failed"
HEALTH_ABORTED = "aborted"
HEALTH_OMITTED = "omitted"
HEALTH_UNNECESSARY = "unnecessary"


@dataclasses.dataclass
class HealthcheckItem:
    """api.HealthcheckItem (healthcheck.go:39-47)."""
    Name: str
    Status: str
    Message: str = ""


@dataclasses.dataclass
class HealthcheckReport:
    """api.HealthcheckReport (healthcheck.go:49-56)."""
    Checks: List[HealthcheckItem] = dataclasses.field(default_factory=list)
    Fixes: List[HealthcheckItem] = dataclasses.field(default_factory=list)

    def ChecksSucceeded(self) -> bool:
        return all(c.Status in (HEALTH_OK, HEALTH_OMITTED) for c in self.Checks)


class LocalSimRunner:
    """api.Runner (and api.Healthchecker) for `local:mi355x-sim`."""

    def __init__(self):
        self._lk = threading.Lock()
        self._active: List[Context] = []

    def ID(self) -> str:
        return "local:mi355x-sim"

    def ConfigType(self):
        return LocalSimRunnerCfg

    def CompatibleBuilders(self) -> List[str]:
        return ["exec:py"]

    @staticmethod
    def _outputs_dir(cfg: LocalSimRunnerCfg) -> str:
        return cfg.outputs_dir or os.path.join(tempfile.gettempdir(), "testground", "local_mi355x_sim")

    def Run(self, ctx: Context, job: RunInput, ow=None) -> RunOutput:
        cfg = job.RunnerConfig or LocalSimRunnerCfg()
        n = sum(g.Instances for g in job.Groups)
        if n != job.TotalInstances:
            raise ValueError(f"groups hold {n} instances, TotalInstances is {job.TotalInstances}")
        if not 0 < n <= cfg.max_instances:
            raise ValueError(f"{n} instances: this runner takes 1..{cfg.max_instances}")
        plans = {g.ID: _resolve(g.ArtifactPath) for g in job.Groups}

        kw = dict(seed=cfg.seed, tick_ns=cfg.tick_ns, queue_limit=cfg.queue_limit,
                  lookahead_ns=cfg.window_ticks * cfg.tick_ns)
        if cfg.engine_factory is None:
            from .engine import Engine  # the HIP engine; raises if the extension is missing
            engine = Engine(n, **kw)
        else:
            engine = cfg.engine_factory(n, **kw)

        run_ctx = Context(timeout=cfg.run_timeout_s)
        with self._lk:
            self._active.append(run_ctx)
        result = Result(Outcomes={g.ID: GroupOutcome(0, g.Instances) for g in job.Groups})
        reactor = SimReactor(engine, n)
        sync_client = reactor.Client
        service = SyncService(sync_client) if cfg.sync_service else None
        svc_host, svc_port = service.address if service else ("", 0)
        bridge = _make_bridge(engine, n, cfg)
        reactor.on_link_removed(bridge.link_removed)
        clock = _Clock(bridge, reactor.lock, n, run_ctx, cfg.max_sim_ns)
        run_dir = os.path.join(self._outputs_dir(cfg), job.TestPlan, job.RunID)
        threads: List[threading.Thread] = []
        res_lk = threading.Lock()
        try:
            reactor.Handle(run_ctx, handler)   # the sidecar, one handler per instance
            clock_t = threading.Thread(target=clock.run, daemon=True)

            def instance(peer: int, gseq: int, g: RunGroup) -> None:
                tag = f"{g.ID}[{gseq:03d}]"
                try:
                    odir = os.path.join(run_dir, g.ID, str(gseq))
                    os.makedirs(odir, exist_ok=True)
                    rp = RunParams(job.TestPlan, job.TestCase, job.RunID, n, g.ID, g.Instances,
                                   dict(g.Parameters), odir, TestStartTime=time.time(),
                                   SyncServiceHost=svc_host, SyncServicePort=svc_port)
                    env = PlanEnv(rp, peer, gseq, reactor.hostname(peer), run_ctx,
                                  ClockedSync(sync_client, clock, peer), reactor.net_client(peer),
                                  DataPlane(clock, peer))
                    plans[g.ID](env)
                    with res_lk:
                        result.Outcomes[g.ID].Ok += 1
                except BaseException as e:  # noqa: BLE001 - recorded as the instance's failure
                    with res_lk:
                        result.Errors[tag] = f"{type(e).__name__}: {e}"
                    if ow is not None:
                        ow.write(f"{tag} failed: {e}\n")
                finally:
                    clock.finish(peer)

            peer = 0
            for g in job.Groups:
                for i in range(g.Instances):
                    t = threading.Thread(target=instance, args=(peer, i, g), daemon=True)
                    threads.append(t)
                    peer += 1
            for t in threads:
                t.start()
            clock_t.start()
            deadline = time.monotonic() + max(0.0, cfg.run_timeout_s)  # one deadline for the whole run
            for t in threads:
                t.join(max(0.0, deadline - time.monotonic()))
            canceled = run_ctx.done() or any(t.is_alive() for t in threads)
            run_ctx.cancel()
            clock_t.join(timeout=5)
        finally:
            run_ctx.cancel()
            if service is not None:
                service.close()
            reactor.Close()
            with self._lk:
                if run_ctx in self._active:
                    self._active.remove(run_ctx)

        result.SimulatedNs = clock.now_ns()
        if reactor.errors:
            for i, e in enumerate(reactor.errors):
                result.Errors[f"sidecar[{i}]"] = str(e)
        ok = bool(result.Outcomes) and all(o.Ok == o.Total for o in result.Outcomes.values())
        result.Outcome = OUTCOME_SUCCESS if ok and not reactor.errors else (
            OUTCOME_CANCELED if canceled else OUTCOME_FAILURE)
        os.makedirs(run_dir, exist_ok=True)
        with open(os.path.join(run_dir, "run.json"), "w") as f:
            json.dump({"outcome": result.Outcome, "outcomes": {g: str(o) for g, o in result.Outcomes.items()},
                       "errors": result.Errors, "simulated_ns": result.SimulatedNs,
                       "engine_stats": engine.stats()}, f, indent=1,
                      default=lambda o: o.tolist() if hasattr(o, "tolist") else int(o))
        if cfg.engine_factory is None:
            engine.close()
        if ow is not None:
            ow.write(f"{result}\n")
        return RunOutput(job.RunID, result)

    def CollectOutputs(self, ctx: Context, inp: CollectionInput, ow: io.BufferedIOBase,
                       cfg: Optional[LocalSimRunnerCfg] = None) -> None:
        """Writes a gzipped tar of the run's outputs (<run>/<group>/<i>/...) to ow, as the local
        runners' gzipRunOutputs does."""
        run_dir = os.path.join(self._outputs_dir(cfg or LocalSimRunnerCfg()), inp.TestPlan, inp.RunID)
        if not os.path.isdir(run_dir):
            raise FileNotFoundError(f"no outputs for run {inp.RunID} under {run_dir}")
        with tarfile.open(fileobj=ow, mode="w:gz") as tar:
            tar.add(run_dir, arcname=inp.RunID)

    def Healthcheck(self, ctx: Context, fix: bool = False, cfg: Optional[LocalSimRunnerCfg] = None,
                    ow=None) -> HealthcheckReport:
        """api.Healthchecker (healthcheck.go:13-15).  Checks, as the local runners' helper does
        (Enlist check + fix, local_exec.go:49-72): the outputs directory (fixed by creating it),
        the engine library and an engine on a GPU (both need manual fixing: build the extension,
        run on a box with an MI355X)."""
        cfg = cfg or LocalSimRunnerCfg()
        rep = HealthcheckReport()

        def outputs():
            d = self._outputs_dir(cfg)
            return (HEALTH_OK, d) if os.path.isdir(d) else (HEALTH_FAILED, f"{d} does not exist")

        def library():
            if cfg.engine_factory is not None:  # the run falls back to the Python bridge without it
                return HEALTH_OMITTED, "engine_factory configured (libtgsim.so optional)"
            from .engine import load_library
            try:
                load_library()
                return HEALTH_OK, "libtgsim.so loaded"
            except (OSError, RuntimeError) as e:  # EngineUnavailable is a RuntimeError
                return HEALTH_FAILED, str(e)

        def engine():
            try:
                if cfg.engine_factory is None:
                    from .engine import Engine
                    e = Engine(1, tick_ns=cfg.tick_ns)
                else:
                    e = cfg.engine_factory(1, tick_ns=cfg.tick_ns)
                e.close()
                return HEALTH_OK, "engine created"
            except Exception as e:  # noqa: BLE001 - reported in the check
                return HEALTH_FAILED, str(e)

        def fix_outputs():
            os.makedirs(self._outputs_dir(cfg), exist_ok=True)

        for name, check, fixer in (("outputs-dir", outputs, fix_outputs), ("engine-library", library, None),
                                   ("engine-device", engine, None)):
            status, msg = check()
            rep.Checks.append(HealthcheckItem(name, status, msg))
            if not fix:
                continue
            if status in (HEALTH_OK, HEALTH_OMITTED):
                rep.Fixes.append(HealthcheckItem(name, HEALTH_UNNECESSARY))
            elif fixer is None:
                rep.Fixes.append(HealthcheckItem(name, HEALTH_FAILED, "requires manual fixing"))
            else:
                try:
                    fixer()
                    rep.Fixes.append(HealthcheckItem(name, HEALTH_OK))
                except OSError as e:
                    rep.Fixes.append(HealthcheckItem(name, HEALTH_FAILED, str(e)))
        if ow is not None:
            for c in rep.Checks:
                ow.write(f"check {c.Name}: {c.Status} {c.Message}\n")
        return rep

    def TerminateAll(self, ctx: Context, ow=None) -> None:
        with self._lk:
            for c in self._active:
                c.cancel()
