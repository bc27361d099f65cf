"""Packet bridge (testground_amd/bridge.py): real payloads through the engine.  CPU tests drive it
over the CPU oracle (the checker), the GPU test over the HIP engine and compares the two."""
import socket
import struct
import time

import numpy as np
import pytest

from testground_amd import abi
from testground_amd import network as nw
from testground_amd import workloads as wl
from testground_amd.bridge import PacketBridge, UdpFront, _flip_bit

WINDOW = 1000  # ticks of 1 us; the engine's lookahead covers one window (replies at delivery time)


def pingpong(bridge, rounds=3):
    """pingpong.go:116-183 over the bridge: each side writes its id, echoes the other's id on
    receipt at the delivery time, and records the round trip when its own id comes back."""
    rtts = {0: [], 1: []}
    sent_at = {}
    for i in (0, 1):
        sent_at[i] = bridge.now_tick
        bridge.send(i, 1 - i, bytes([i]))
    for _ in range(2_000):
        bridge.step()
        for me in (0, 1):
            for t_ns, src, _seq, data, _f in bridge.recv(me):
                at = -(-t_ns // 1000)
                if data[0] == me:  # own id came back
                    rtts[me].append(t_ns - sent_at[me] * 1000)
                    if len(rtts[me]) < rounds:
                        sent_at[me] = at
                        bridge.send(me, 1 - me, bytes([me]), at_tick=at)
                else:
                    bridge.send(me, src, data, at_tick=at)  # echo
        if all(len(r) >= rounds for r in rtts.values()):
            return rtts
    raise AssertionError(f"ping-pong did not finish: {rtts}")


def test_bridge_pingpong_rtt(make_oracle):
    """plans/network/pingpong.go:185: RTT in [200, 215] ms at 100 ms latency and 1 MiB/s."""
    e = make_oracle(2, lookahead_ns=WINDOW * 1000)
    for i in (0, 1):
        e.configure(i, wl.pingpong_config(100 * nw.Millisecond))
    rtts = pingpong(PacketBridge(e, 2, WINDOW))
    for me in (0, 1):
        assert all(200 * nw.Millisecond <= r <= 215 * nw.Millisecond for r in rtts[me]), rtts


def test_bridge_payloads_follow_verdicts(make_oracle):
    """Every payload arrives as sent, once per scheduled copy, with exactly one bit flipped iff
    the copy is corrupted; lost or queue-full datagrams never arrive and leave nothing behind."""
    n = 4
    e = make_oracle(n, lookahead_ns=WINDOW * 1000, queue_limit=64)
    shape = nw.LinkShape(Latency=2 * nw.Millisecond, Jitter=1 * nw.Millisecond, Loss=20.0,
                         Duplicate=30.0, Corrupt=40.0, Bandwidth=10**7)
    for i in range(n):
        e.configure(i, nw.Config(Network="default", Enable=True, Default=shape))
    b = PacketBridge(e, n, WINDOW)
    rng = np.random.default_rng(1)
    sent = {}
    for w in range(20):
        for _ in range(60):
            src = int(rng.integers(0, n))
            dst = int((src + 1 + rng.integers(0, n - 1)) % n)
            data = rng.bytes(int(rng.integers(1, 1400)))
            seq = b.send(src, dst, data, at_tick=b.now_tick + int(rng.integers(0, WINDOW)))
            sent[(src, seq)] = (dst, data)
        b.step()
    for _ in range(10):
        b.step()
    assert b.in_flight() == 0
    got = {}
    for peer in range(n):
        for _t, src, seq, data, flags in b.recv(peer):
            dst, orig = sent[(src, seq)]
            assert dst == peer and len(data) == len(orig)
            if flags & abi.FLAG_CORRUPT:
                assert data == _flip_bit(orig, src, seq, flags & abi.FLAG_DUP)
            diff = sum(bin(x ^ y).count("1") for x, y in zip(orig, data))
            assert diff == (1 if flags & abi.FLAG_CORRUPT else 0)
            got[(src, seq)] = got.get((src, seq), 0) + 1
    v = np.concatenate(b.verdicts)
    scheduled = int(((v & 15) == abi.V_SCHEDULED).sum() + ((v >> 4) == abi.V_SCHEDULED).sum())
    assert sum(got.values()) == scheduled > 0
    assert ((v & 15) == abi.V_LOSS).any() and ((v >> 4) == abi.V_SCHEDULED).any()
    assert max(got.values()) == 2


def test_udp_front(make_oracle):
    """Real UDP sockets: instance 0 sends a datagram for instance 1 to the bridge; after the
    simulated latency it arrives at instance 1's socket from the bridge with a source header."""
    e = make_oracle(2, lookahead_ns=WINDOW * 1000)
    for i in (0, 1):
        e.configure(i, nw.Config(Network="default", Enable=True, Default=nw.LinkShape(Latency=3 * nw.Millisecond)))
    front = UdpFront(PacketBridge(e, 2, WINDOW))
    socks = []
    try:
        for i in (0, 1):
            s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
            s.bind(("127.0.0.1", 0))
            s.settimeout(5)
            front.register(i, s.getsockname())
            socks.append(s)
        socks[0].sendto(struct.pack("!I", 1) + b"hello over tgsim", front.addr)
        time.sleep(0.05)  # let the datagram reach the bridge's socket
        delivered = sum(front.pump() for _ in range(6))
        assert delivered == 1
        msg, addr = socks[1].recvfrom(65536)
        assert addr == front.addr and struct.unpack("!I", msg[:4])[0] == 0 and msg[4:] == b"hello over tgsim"
    finally:
        front.close()
        for s in socks:
            s.close()


@pytest.mark.gpu
def test_bridge_pingpong_gpu_equals_oracle(make_oracle):
    """The same ping-pong through the HIP engine: identical round-trip times to the oracle's."""
    import torch

    from testground_amd.engine import Engine

    if torch.cuda.is_available():
        torch.cuda.init()
    res = []
    for e in (Engine(2, lookahead_ns=WINDOW * 1000), make_oracle(2, lookahead_ns=WINDOW * 1000)):
        for i in (0, 1):
            e.configure(i, wl.pingpong_config(100 * nw.Millisecond))
        res.append(pingpong(PacketBridge(e, 2, WINDOW)))
    assert res[0] == res[1]
    assert all(200 * nw.Millisecond <= r <= 215 * nw.Millisecond for r in res[0][0])
