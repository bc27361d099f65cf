"""Mirror of the reference sidecar's instance handling (pkg/sidecar) over the engine.

The reference's plugin surface is kept with the same names, argument meaning and errors:

  Network{ConfigureNetwork, ListActive, Close}     pkg/sidecar/instance.go:37-42
  Reactor{Handle, Close}, InstanceHandler          pkg/sidecar/instance.go:16-23
  Instance{Hostname, Client, RunEnv, Network}      pkg/sidecar/instance.go:25-60
  handler                                          pkg/sidecar/sidecar_handler.go:15-83
  MockReactor / MockNetwork                        pkg/sidecar/mock.go:27-118

plus the sdk-go pieces the handler and the plans talk to: an in-memory sync client (the role of
sync.NewInmemClient, used by mock.go:41) and network.Client (WaitNetworkInitialized,
ConfigureNetwork).  ``SimNetwork`` is the new implementation of ``Network``: one per simulated
instance, all funnelled into one engine handle (the C engine is not re-entrant, so calls are
serialised with a lock, as INTEGRATION.md's Go binding does).
"""
from __future__ import annotations

import copy
import dataclasses
import queue
import threading
import time
from typing import Callable, Dict, List, Optional

from .abi import SYNC_STATES
from .engine import EngineError
from .network import Config

DEFAULT_DATA_NETWORK = "default"   # sidecar_handler.go:11
NET_INIT_STATE = "network-initialized"  # sidecar_handler.go:39


class Context:
    """Minimal context.Context: cancellation plus an optional deadline."""

    def __init__(self, timeout: Optional[float] = None):
        self._done = threading.Event()
        self._deadline = time.monotonic() + timeout if timeout else None

    def cancel(self) -> None:
        self._done.set()

    def done(self) -> bool:
        if self._deadline is not None and time.monotonic() > self._deadline:
            self._done.set()
        return self._done.is_set()

    def err(self) -> Optional[str]:
        return "context canceled" if self.done() else None


class SyncClient:
    """In-memory sync service: signal (1-based sequence numbers), barrier, pub/sub topics."""

    def __init__(self):
        self._cv = threading.Condition()
        self._counts: Dict[str, int] = {}
        self._topics: Dict[str, List] = {}
        self._subs: Dict[str, List[queue.Queue]] = {}

    def SignalEntry(self, ctx: Context, state: str) -> int:
        with self._cv:
            self._counts[state] = self._counts.get(state, 0) + 1
            self._cv.notify_all()
            return self._counts[state]

    def _reached(self, state: str, target: int) -> bool:
        with self._cv:
            return self._counts.get(state, 0) >= target

    def Barrier(self, ctx: Context, state: str, target: int) -> None:
        with self._cv:
            while self._counts.get(state, 0) < target:
                if ctx.done():
                    raise TimeoutError(f"barrier {state!r}: {ctx.err()}")
                self._cv.wait(timeout=0.05)

    def SignalAndWait(self, ctx: Context, state: str, target: int) -> int:
        seq = self.SignalEntry(ctx, state)
        self.Barrier(ctx, state, target)
        return seq

    def Publish(self, ctx: Context, topic: str, payload) -> int:
        # sdk-go serialises the payload onto the topic: subscribers get a copy, and the publisher
        # may change its own object afterwards (pingpong.go:190-192 reuses its Config)
        payload = copy.deepcopy(payload)
        with self._cv:
            self._topics.setdefault(topic, []).append(payload)
            for q in self._subs.get(topic, []):
                q.put(payload)
            return len(self._topics[topic])

    def Subscribe(self, ctx: Context, topic: str) -> "queue.Queue":
        q: queue.Queue = queue.Queue(maxsize=0)
        with self._cv:
            for p in self._topics.get(topic, []):  # subscribers see the whole topic history
                q.put(p)
            self._subs.setdefault(topic, []).append(q)
        return q

    def PublishAndWait(self, ctx: Context, topic: str, payload, state: str, target: int) -> int:
        seq = self.Publish(ctx, topic, payload)
        self.Barrier(ctx, state, target)
        return seq

    def Close(self) -> None:
        pass


class EngineSyncClient(SyncClient):
    """Sync client whose signal and barrier counters are the engine's sync counters
    (tgsim_signal / tgsim_barrier_poll, K7): the states the handler signals
    (`network-initialized`, sidecar_handler.go:40-44; callback states, :75-80) and the plans'
    barriers live beside the simulated network instead of in a Redis-backed sync service.
    Pub/sub topics stay in memory (the handler's `network:<hostname>` subscription, :49).

    State names map to the engine's device counters (abi.SYNC_STATES of them) in first-use order,
    so every process of a sharded run must touch its states in the same order; `reduce`, when
    given, sums a state's count over the shards (ShardedStepper.barrier does it with an RCCL
    all-reduce).  The reference's sync service has no state limit, so a run that names more states
    than the engine holds (e.g. one callback state per instance, splitbrain/main.go:113, at more
    than 65,536 instances) keeps the rest in this client's in-memory counters; that works for a
    single engine, while a sharded run (`reduce`) refuses the extra state with a clear error."""

    def __init__(self, engine, lock: Optional[threading.Lock] = None,
                 reduce: Optional[Callable[[int, int], bool]] = None, n_slots: Optional[int] = None):
        super().__init__()
        self.engine = engine
        self.lock = lock or threading.Lock()
        self.reduce = reduce
        self.n_slots = n_slots if n_slots is not None else SYNC_STATES
        self._ids: Dict[str, int] = {}

    def state_id(self, state: str) -> Optional[int]:
        """The engine counter of `state`, or None when it lives in the in-memory counters."""
        with self._cv:
            if state not in self._ids:
                if len(self._ids) >= self.n_slots:
                    if self.reduce is not None:
                        raise RuntimeError(f"sync state {state!r}: all {self.n_slots} engine sync counters are "
                                           "in use and a sharded run cannot sum in-memory counters")
                    return None
                self._ids[state] = len(self._ids)
            return self._ids[state]

    def SignalEntry(self, ctx: Context, state: str) -> int:
        sid = self.state_id(state)
        if sid is None:
            return super().SignalEntry(ctx, state)
        with self.lock:
            seq = self.engine.signal(sid, 1)
        with self._cv:
            self._cv.notify_all()
        return seq

    def _reached(self, state: str, target: int) -> bool:
        sid = self.state_id(state)
        if sid is None:
            return super()._reached(state, target)
        if self.reduce is not None:
            return self.reduce(sid, target)
        with self.lock:
            return self.engine.barrier_poll(sid, target)

    def Barrier(self, ctx: Context, state: str, target: int) -> None:
        while not self._reached(state, target):
            if ctx.done():
                raise TimeoutError(f"barrier {state!r}: {ctx.err()}")
            with self._cv:
                self._cv.wait(timeout=0.01)


@dataclasses.dataclass
class RunEnv:
    TestInstanceCount: int = 1
    TestSidecar: bool = True
    TestRun: str = "run"
    TestSubnet: str = "16.0.0.0/8"


class NetClient:
    """sdk-go network.Client as used by the plans (pingpong.go:21-22, splitbrain/main.go:73-74)."""

    def __init__(self, sync_client: SyncClient, runenv: RunEnv, hostname: str, ip: Optional[str] = None):
        self.sync = sync_client
        self.runenv = runenv
        self.hostname = hostname
        self._ip = ip  # the data-network address (sdk-go reads it from the interface)

    def GetDataNetworkIP(self) -> str:
        """MustGetDataNetworkIP (pingpong.go:83): the instance's current data-network address."""
        if self._ip is None:
            raise RuntimeError("no data network address")
        return self._ip

    def WaitNetworkInitialized(self, ctx: Context) -> None:
        self.sync.Barrier(ctx, NET_INIT_STATE, self.runenv.TestInstanceCount)

    def ConfigureNetwork(self, ctx: Context, config: Config) -> None:
        if not config.CallbackState:  # pinned by sidecar_test.go:59
            raise ValueError("failed to configure network; no callback state provided")
        target = config.CallbackTarget or self.runenv.TestInstanceCount
        # sdk-go serialises the config onto the topic, so the sidecar gets a copy and the caller
        # may change its own object afterwards (plans/network/pingpong.go:191-194 does)
        self.sync.PublishAndWait(ctx, "network:" + self.hostname, copy.deepcopy(config),
                                 config.CallbackState, target)
        if config.IPv4 is not None and config.Enable:
            from .network import _ipnet
            import ipaddress
            self._ip = str(ipaddress.IPv4Address(_ipnet(config.IPv4)[0]))


class Network:
    """sidecar.Network (instance.go:37-42)."""

    def ConfigureNetwork(self, ctx: Context, cfg: Config) -> None:
        raise NotImplementedError

    def ListActive(self) -> List[str]:
        raise NotImplementedError

    def Close(self) -> None:
        raise NotImplementedError


class MockNetwork(Network):
    """mock.go:88-118: records every config; closed networks refuse configuration."""

    def __init__(self):
        self.Active: Dict[str, Config] = {"default": Config()}
        self.Configured: List[Config] = []
        self.Closed = False
        self.L = threading.Lock()

    def Close(self) -> None:
        self.Closed = True

    def ConfigureNetwork(self, ctx: Context, cfg: Config) -> None:
        if self.Closed:
            raise RuntimeError("mock network is closed.")
        with self.L:
            self.Configured.append(cfg)
            self.Active[cfg.Network] = cfg

    def ListActive(self) -> List[str]:
        return list(self.Active)


class SimNetwork(Network):
    """sidecar.Network backed by the engine: the instance is simulated peer `peer`.  The engine
    applies DockerNetwork.ConfigureNetwork's order of operations and errors (docker_network.go:51-148);
    the config is copied into engine state and never mutated (sidecar_test.go:91-92)."""

    def __init__(self, engine, peer: int, lock: threading.Lock,
                 on_link_removed: Optional[Callable[[int], None]] = None):
        self.engine = engine
        self.peer = peer
        self.lock = lock
        # called (under the lock) when a config removed the data link: the packet bridge then
        # resolves the packets the engine flushed or purged with it (tgsim_bridge_link_removed)
        self.on_link_removed = on_link_removed
        self.active: Dict[str, bool] = {DEFAULT_DATA_NETWORK: True}
        self.closed = False

    def ConfigureNetwork(self, ctx: Context, cfg: Config) -> None:
        if self.closed:
            raise RuntimeError("network is closed")
        with self.lock:
            gen = self.engine.link_generation(self.peer) if self.on_link_removed else 0
            self.engine.configure(self.peer, cfg)
            if self.on_link_removed and self.engine.link_generation(self.peer) != gen:
                self.on_link_removed(self.peer)
        self.active[cfg.Network] = bool(cfg.Enable)

    def ListActive(self) -> List[str]:
        return [n for n, on in self.active.items() if on]

    def Close(self) -> None:
        self.closed = True


@dataclasses.dataclass
class Instance:
    """instance.go:25-60."""
    Hostname: str
    Client: SyncClient
    RunEnv: RunEnv
    Network: Network

    def Close(self) -> None:
        self.Network.Close()


InstanceHandler = Callable[[Context, Instance], None]


class HandlerError(RuntimeError):
    pass


def handler(ctx: Context, instance: Instance) -> None:
    """sidecar_handler.go:15-83: configure the default network, wait for every sidecar, then
    apply each config published on network:<hostname> and signal its callback state."""
    try:
        instance.Network.ConfigureNetwork(ctx, Config(Network=DEFAULT_DATA_NETWORK, Enable=True))
        instance.Client.SignalAndWait(ctx, NET_INIT_STATE, instance.RunEnv.TestInstanceCount)
        changes = instance.Client.Subscribe(ctx, "network:" + instance.Hostname)
        while not ctx.done():
            try:
                cfg = changes.get(timeout=0.05)
            except queue.Empty:
                continue
            try:
                instance.Network.ConfigureNetwork(ctx, cfg)
            except (EngineError, RuntimeError) as e:
                raise HandlerError(f"failed to update network {cfg.Network}: {e}") from e
            if cfg.CallbackState:
                instance.Client.SignalEntry(ctx, cfg.CallbackState)
    finally:
        instance.Close()


class Reactor:
    """sidecar.Reactor (instance.go:18-23)."""

    def Handle(self, ctx: Context, h: InstanceHandler) -> None:
        raise NotImplementedError

    def Close(self) -> None:
        pass


class MockReactor(Reactor):
    """mock.go:27-73: a single instance with a MockNetwork and an in-memory sync client."""

    def __init__(self, hostname: str = "mock-host"):
        self.RunEnv = RunEnv(TestInstanceCount=1)
        self.Network = MockNetwork()
        self.Client = SyncClient()
        self.Hostname = hostname

    def Handle(self, ctx: Context, h: InstanceHandler) -> None:
        h(ctx, Instance(self.Hostname, self.Client, self.RunEnv, self.Network))


class SimReactor(Reactor):
    """The `mi355x-sim` reactor: one Instance per simulated peer, all on one engine, each served
    by `handler` on its own thread (the docker reactor runs one goroutine per container,
    pkg/docker/manager.go:154-178)."""

    def __init__(self, engine, n_instances: int, client: Optional[SyncClient] = None):
        self.engine = engine
        self.n = n_instances
        self.lock = threading.Lock()
        self.Client = client if client is not None else EngineSyncClient(engine, self.lock)
        self.RunEnv = RunEnv(TestInstanceCount=n_instances)
        self.threads: List[threading.Thread] = []
        self.errors: List[BaseException] = []
        self.networks = [SimNetwork(engine, p, self.lock) for p in range(n_instances)]

    def hostname(self, peer: int) -> str:
        return f"instance-{peer}"

    def Handle(self, ctx: Context, h: InstanceHandler) -> None:
        def run(p):
            try:
                h(ctx, Instance(self.hostname(p), self.Client, self.RunEnv, self.networks[p]))
            except BaseException as e:  # noqa: BLE001 - reported to the caller
                self.errors.append(e)

        for p in range(self.n):
            t = threading.Thread(target=run, args=(p,), daemon=True)
            t.start()
            self.threads.append(t)

    def on_link_removed(self, fn: Callable[[int], None]) -> None:
        """Routes every instance's link removals to fn (the runner's packet bridge)."""
        for nw in self.networks:
            nw.on_link_removed = fn

    def net_client(self, peer: int) -> NetClient:
        import ipaddress
        base = int(getattr(self.engine, "subnet_base", 0) or (16 << 24))
        return NetClient(self.Client, self.RunEnv, self.hostname(peer), str(ipaddress.IPv4Address(base + 2 + peer)))

    def Close(self) -> None:
        for t in self.threads:
            t.join(timeout=5)


def snapshot(cfg: Config) -> Config:
    """Deep copy used by tests to check configs pass through unmodified."""
    return copy.deepcopy(cfg)
