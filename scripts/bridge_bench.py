"""Datagrams/s through the packet bridge (host payload bookkeeping + HIP engine), C3-like traffic:
n instances, `per` datagrams of 100 B per 1-ms window to uniform destinations, 100 Mbit/s links."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from testground_amd import network as nw  # noqa: E402
from testground_amd.bridge import PacketBridge  # noqa: E402
from testground_amd.engine import Engine  # noqa: E402

n, per, windows = 1000, 50_000, 20
torch.cuda.init()
e = Engine(n, lookahead_ns=1_000_000)
for i in range(n):
    e.configure(i, nw.Config(Network="default", Enable=True,
                             Default=nw.LinkShape(Latency=5 * nw.Millisecond, Bandwidth=10**8)))
b = PacketBridge(e, n, 1000)
rng = np.random.default_rng(0)
payload = bytes(100)
src = rng.integers(0, n, per * windows)
dst = (src + 1 + rng.integers(0, n - 1, per * windows)) % n
tick = rng.integers(0, 1000, per * windows)
t0 = time.perf_counter()
t_send = 0.0
for w in range(windows):
    ts = time.perf_counter()
    base = b.now_tick
    for k in range(w * per, (w + 1) * per):
        b.send(int(src[k]), int(dst[k]), payload, at_tick=base + int(tick[k]))
    t_send += time.perf_counter() - ts
    b.step()
for _ in range(10):
    b.step()
el = time.perf_counter() - t0
got = sum(len(b.recv(i)) for i in range(n))
print(f"bridge: {per * windows} datagrams sent, {got} delivered, {el:.2f} s wall "
      f"({per * windows / el / 1e3:.0f} k datagrams/s; {t_send:.2f} s in send())")
