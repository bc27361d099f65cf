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


def _native_available():
    from testground_amd.engine import LIB_PATH
    return LIB_PATH.exists()


native = pytest.mark.skipif(not _native_available(), reason="libtgsim.so not built (run __graft_entry__.build())")


def _lossy_pair(make_oracle, n):
    shape = nw.LinkShape(Latency=2 * nw.Millisecond, Jitter=1 * nw.Millisecond, Loss=20.0,
                         Duplicate=30.0, Corrupt=40.0, Bandwidth=10**7)
    out = []
    for _ in range(2):
        e = make_oracle(n, lookahead_ns=WINDOW * 1000, queue_limit=64)
        for i in range(n):
            e.configure(i, nw.Config(Network="default", Enable=True, Default=shape))
        out.append(e)
    return out


@native
def test_native_bridge_equals_python_bridge(make_oracle):
    """The C++ bridge (tgsim_bridge_*) and the Python PacketBridge, each over its own oracle engine
    fed the same datagrams: identical deliveries per destination (time, source, sequence number,
    payload bytes incl. duplicates and the flipped bit of corrupted copies, flags)."""
    from testground_amd.bridge import NativeBridge

    n = 6
    ep, en = _lossy_pair(make_oracle, n)
    bp, bn = PacketBridge(ep, n, WINDOW), NativeBridge(en, n, WINDOW)
    rng = np.random.default_rng(7)
    for w in range(25):
        k = 80
        src = rng.integers(0, n, k)
        dst = (src + 1 + rng.integers(0, n - 1, k)) % n
        lens = rng.integers(0, 900, k)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        data = rng.bytes(int(off[-1]))
        ticks = bp.now_tick + rng.integers(0, 2 * WINDOW, k)
        seq_n = bn.send_many(src, dst, data, off, ticks)
        seq_p = [bp.send(int(s), int(d), data[int(off[i]):int(off[i + 1])], at_tick=int(ticks[i]))
                 for i, (s, d) in enumerate(zip(src, dst))]
        assert list(seq_n) == seq_p
        assert bp.step() == bn.step()
        if w % 5 == 4:
            for peer in range(n):
                assert bp.recv(peer) == bn.recv(peer), (w, peer)
    for _ in range(10):
        bp.step()
        bn.step()
    for peer in range(n):
        assert bp.recv(peer) == bn.recv(peer)
    assert bp.in_flight() == bn.in_flight() == 0


@native
def test_native_udp_front(make_oracle):
    """The C UDP front end (recvmmsg/sendmmsg) over the native bridge: datagrams from registered
    instance sockets cross the simulated link and reach the destination socket with a source
    header."""
    from testground_amd.bridge import NativeBridge, NativeUdpFront

    n = 3
    e = make_oracle(n, lookahead_ns=WINDOW * 1000)
    for i in range(n):
        e.configure(i, nw.Config(Network="default", Enable=True, Default=nw.LinkShape(Latency=3 * nw.Millisecond)))
    front = NativeUdpFront(NativeBridge(e, n, WINDOW))
    socks = []
    try:
        for i in range(n):
            s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
            s.bind(("127.0.0.1", 0))
            s.settimeout(5)
            front.register(i, s.getsockname())
            socks.append(s)
        for k in range(50):
            socks[0].sendto(struct.pack("!I", 1 + k % 2) + b"msg%03d" % k, front.addr)
        socks[2].sendto(struct.pack("!I", 0) + b"back", front.addr)
        time.sleep(0.05)
        delivered = sum(front.pump() for _ in range(6))
        assert delivered == 51
        got1 = sorted(socks[1].recvfrom(65536)[0] for _ in range(25))
        assert got1 == sorted(struct.pack("!I", 0) + b"msg%03d" % k for k in range(0, 50, 2))
        msg, addr = socks[0].recvfrom(65536)
        assert addr == front.addr and msg == struct.pack("!I", 2) + b"back"
    finally:
        front.close()
        for s in socks:
            s.close()


@pytest.mark.gpu
def test_native_bridge_gpu_equals_oracle(make_oracle):
    """The native bridge over the HIP engine delivers exactly what the Python bridge delivers over
    the oracle (payloads, duplicates, corrupted bits, times)."""
    import torch

    from testground_amd.bridge import NativeBridge
    from testground_amd.engine import Engine

    if torch.cuda.is_available():
        torch.cuda.init()
    n = 6
    shape = nw.LinkShape(Latency=2 * nw.Millisecond, Jitter=1 * nw.Millisecond, Loss=20.0,
                         Duplicate=30.0, Corrupt=40.0, Bandwidth=10**7)
    eg = Engine(n, lookahead_ns=WINDOW * 1000, queue_limit=64)
    ec = make_oracle(n, lookahead_ns=WINDOW * 1000, queue_limit=64)
    for e in (eg, ec):
        for i in range(n):
            e.configure(i, nw.Config(Network="default", Enable=True, Default=shape))
    bn, bp = NativeBridge(eg, n, WINDOW), PacketBridge(ec, n, WINDOW)
    rng = np.random.default_rng(9)
    for w in range(20):
        k = 100
        src = rng.integers(0, n, k)
        dst = (src + 1 + rng.integers(0, n - 1, k)) % n
        lens = rng.integers(1, 900, k)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        data = rng.bytes(int(off[-1]))
        bn.send_many(src, dst, data, off)
        for i, (s, d) in enumerate(zip(src, dst)):
            bp.send(int(s), int(d), data[int(off[i]):int(off[i + 1])])
        assert bn.step() == bp.step()
    for peer in range(n):
        assert bn.recv(peer) == bp.recv(peer)


@native
def test_bridge_link_removal_resolves_queued_packets(make_oracle):
    """a scheduled datagram can vanish inside the engine when a link goes away: its
    sender is disconnected (the netem queue is flushed, docker_network.go:65-75) or its destination
    is re-addressed (in-flight packets find no port, :77-88).  The sidecar's SimNetwork sees the
    engine's link generation change and tells the bridge, which resolves exactly those datagrams:
    after draining, nothing is left in flight, on the C++ bridge and on the Python one, and both
    delivered the same datagrams."""
    import ipaddress

    from testground_amd.bridge import NativeBridge
    from testground_amd.sidecar import Context, SimNetwork
    import threading

    n = 6
    shape = nw.LinkShape(Latency=20 * nw.Millisecond, Jitter=5 * nw.Millisecond, Loss=5.0, Duplicate=20.0,
                         Bandwidth=10**7)
    engines = [make_oracle(n, lookahead_ns=WINDOW * 1000, queue_limit=256) for _ in range(2)]
    for e in engines:
        for i in range(n):
            e.configure(i, nw.Config(Network="default", Enable=True, Default=shape))
    bp, bn = PacketBridge(engines[0], n, WINDOW), NativeBridge(engines[1], n, WINDOW)
    nets = [[SimNetwork(e, p, threading.Lock(), on_link_removed=b.link_removed) for p in range(n)]
            for e, b in ((engines[0], bp), (engines[1], bn))]
    rng = np.random.default_rng(3)
    ctx = Context()
    for w in range(16):
        k = 60
        src = rng.integers(0, n, k)
        dst = (src + 1 + rng.integers(0, n - 1, k)) % n
        off = np.concatenate([[0], np.cumsum(rng.integers(1, 300, k))]).astype(np.uint64)
        data = rng.bytes(int(off[-1]))
        ticks = bp.now_tick + rng.integers(0, 3 * WINDOW, k)
        bn.send_many(src, dst, data, off, ticks)
        for i, (s, d) in enumerate(zip(src, dst)):
            bp.send(int(s), int(d), data[int(off[i]):int(off[i + 1])], at_tick=int(ticks[i]))
        if w == 6:  # peer 2 disconnects with its queue full of traffic
            for ns in nets:
                ns[2].ConfigureNetwork(ctx, nw.Config(Network="default", Enable=False))
        if w == 9:  # peer 4 moves to a new address while traffic towards it is queued everywhere
            ip = (str(ipaddress.IPv4Address((16 << 24) + 0x100 + 4)), 8)
            for ns in nets:
                ns[4].ConfigureNetwork(ctx, nw.Config(Network="default", Enable=True, IPv4=ip, Default=shape))
        if w == 12:  # peer 2 comes back
            for ns in nets:
                ns[2].ConfigureNetwork(ctx, nw.Config(Network="default", Enable=True, Default=shape))
        assert bp.step() == bn.step()
    for _ in range(40):
        bp.step()
        bn.step()
    for e in engines:
        st = e.stats()
        assert st["flushed"] > 0 and st["lost_in_flight"] > 0, st  # the scenario removed queued packets
        assert e.link_generation(2) == 1 and e.link_generation(4) == 1 and e.link_generation(0) == 0
    for peer in range(n):
        assert bp.recv(peer) == bn.recv(peer)
    assert bp.in_flight() == bn.in_flight() == 0


@native
def test_native_udp_front_headerless(make_oracle):
    """TUN/TAP is not available on the GPU box (no /dev/net/tun, no CAP_NET_ADMIN, user namespaces
    disabled: DESIGN.md §9), so unmodified UDP code reaches the engine through per-peer data-address
    sockets of the front end (tgsim_udp_front_bind_peer): an instance sends a plain datagram to the
    peer's address and the peer's recvfrom returns the payload unchanged with the SENDER's data
    address as the source, after the simulated link's delay.  No header either way."""
    from testground_amd.bridge import NativeBridge, NativeUdpFront

    n = 3
    e = make_oracle(n, lookahead_ns=WINDOW * 1000)
    for i in range(n):
        e.configure(i, nw.Config(Network="default", Enable=True, Default=nw.LinkShape(Latency=3 * nw.Millisecond)))
    b = NativeBridge(e, n, WINDOW)
    front = NativeUdpFront(b)
    socks, vaddr = [], []
    try:
        for i in range(n):
            s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
            s.bind(("127.0.0.1", 0))
            s.settimeout(5)
            front.register(i, s.getsockname())
            socks.append(s)
            vaddr.append(front.bind_peer(i))
        for k in range(20):  # plain datagrams, addressed by the peer's data address only
            socks[0].sendto(b"ping%02d" % k, vaddr[1 + k % 2])
        socks[2].sendto(b"pong", vaddr[0])
        time.sleep(0.05)
        t0 = b.now_tick
        delivered = sum(front.pump() for _ in range(6))
        assert delivered == 21
        got1 = sorted(socks[1].recvfrom(65536) for _ in range(10))
        assert [m for m, _ in got1] == sorted(b"ping%02d" % k for k in range(0, 20, 2))
        assert all(addr == vaddr[0] for _, addr in got1)  # the source's data address, no header
        msg, addr = socks[0].recvfrom(65536)
        assert msg == b"pong" and addr == vaddr[2]
        assert b.now_tick - t0 == 6 * WINDOW and b.in_flight() == 0
    finally:
        front.close()
        for s in socks:
            s.close()


@native
def test_unmodified_udp_echo_program_through_front_end(make_oracle):
    """an unmodified UDP program (tests/udp_echo_server.py, a separate process that
    only binds a port and echoes what it receives to the sender's address) is instance 1; instance 0's
    client sends plain datagrams to instance 1's data address.  Both directions cross the simulated
    3 ms link through the C front end (recvmmsg -> engine window -> sendmmsg), with no framing: the
    echo program sees instance 0's data address as the sender and replies to it, and the client gets
    every payload back from instance 1's data address, no earlier than one simulated round trip.
    (TCP plans stay out of reach: no TUN/TAP or capabilities on the GPU box)"""
    import subprocess
    import sys
    from pathlib import Path

    from testground_amd.bridge import NativeBridge, NativeUdpFront

    n, lat_ms = 2, 3
    e = make_oracle(n, lookahead_ns=WINDOW * 1000)
    for i in range(n):
        e.configure(i, nw.Config(Network="default", Enable=True, Default=nw.LinkShape(Latency=lat_ms * nw.Millisecond)))
    b = NativeBridge(e, n, WINDOW)
    front = NativeUdpFront(b)
    msgs = [b"echo-%03d" % k + bytes(range(k % 7)) for k in range(10)]
    echo = subprocess.Popen([sys.executable, str(Path(__file__).with_name("udp_echo_server.py")), "0", str(len(msgs))],
                            stdout=subprocess.PIPE, text=True)
    cli = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        echo_port = int(echo.stdout.readline())
        cli.bind(("127.0.0.1", 0))
        cli.setblocking(False)
        front.register(0, cli.getsockname())
        front.register(1, ("127.0.0.1", echo_port))
        vaddr = [front.bind_peer(i) for i in range(n)]
        for m in msgs:
            cli.sendto(m, vaddr[1])
        time.sleep(0.05)
        got, first_at = [], None
        for w in range(400):
            front.pump()
            time.sleep(0.002)  # the echo program answers in wall-clock time
            while True:
                try:
                    data, addr = cli.recvfrom(65536)
                except BlockingIOError:
                    break
                assert addr == vaddr[1]  # from the echo instance's data address, no header
                got.append(data)
                first_at = first_at if first_at is not None else w + 1
            if len(got) == len(msgs):
                break
        assert sorted(got) == sorted(msgs)
        assert first_at >= 2 * lat_ms * 1000 // WINDOW  # a simulated round trip at least
        assert echo.wait(timeout=10) == 0  # it saw all its datagrams
    finally:
        echo.kill()
        cli.close()
        front.close()
