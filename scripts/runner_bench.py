"""Throughput of the local:mi355x-sim runner on the HIP engine: N instances, each sends K datagrams
of 100 B to random instances over a C3-style shaped link, then receives for 200 simulated ms.
Prints one JSON line (wall seconds, datagrams sent and delivered, windows simulated)."""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from testground_amd import network as nw
from testground_amd import runner as rn
from testground_amd.sidecar import Context

ap = argparse.ArgumentParser()
ap.add_argument("--instances", type=int, default=256)
ap.add_argument("--per-instance", type=int, default=200)
args = ap.parse_args()
delivered = [0] * args.instances


def plan(env: rn.PlanEnv) -> None:
    env.net.WaitNetworkInitialized(env.ctx)
    env.net.ConfigureNetwork(env.ctx, nw.Config(
        Network="default", Enable=True, CallbackState="shaped",
        Default=nw.LinkShape(Latency=20 * nw.Millisecond, Jitter=5 * nw.Millisecond, Loss=1.0,
                             Bandwidth=100 * 10**6)))
    rng = random.Random(env.seq)
    n = env.runenv.TestInstanceCount
    for _ in range(args.per_instance):
        d = rng.randrange(n - 1)
        env.data.send(d + (d >= env.seq), b"x" * 100)
    end = env.data.now_ns() + 200 * nw.Millisecond
    while env.data.now_ns() < end:
        delivered[env.seq] += len(env.data.recv(timeout_ns=end - env.data.now_ns()))


cfg = rn.LocalSimRunnerCfg(run_timeout_s=300)
job = rn.RunInput("bench", "bench", "runner", args.instances, [rn.RunGroup("all", args.instances, plan)], cfg)
t0 = time.perf_counter()
out = rn.LocalSimRunner().Run(Context(), job)
wall = time.perf_counter() - t0
sent = args.instances * args.per_instance
print(json.dumps({"outcome": out.Result.Outcome, "instances": args.instances, "sent": sent,
                  "delivered": sum(delivered), "wall_s": round(wall, 3),
                  "datagrams_per_s": round(sent / wall), "simulated_ms": out.Result.SimulatedNs / 1e6,
                  "errors": dict(list(out.Result.Errors.items())[:3])}))
