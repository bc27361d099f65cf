"""Packet bridge: real payloads through the simulated network.

In the reference a plan's packets cross the kernel data path of its container's data interface
(veth → FIB → netem → HTB → bridge; `pkg/runner/local_docker.go:706-721`, `pkg/sidecar/link.go`).
Here the payload bytes stay on the host and only the 16-byte packet record goes to the engine
(`tgsim_submit`); every delivery the engine drains is injected back into the destination's inbox
with its payload, so what a receiver sees is exactly what the engine decided:

* scheduled  → delivered at the engine's delivery time;
* duplicated → delivered twice (the clone carries FLAG_DUP);
* corrupted  → delivered with one bit flipped (netem's corrupt flips one random bit of the
  packet; the bit is chosen from (src, seq, clone) so runs are reproducible);
* dropped / filtered / queue-full → never delivered (the verdict bytes say why).

`UdpFront` puts real sockets in front of it: each instance owns a UDP socket on 127.0.0.1, sends
datagrams to the bridge's port with a 4-byte destination header, and receives what the engine
delivered with a 4-byte source header.  Time is simulated: the bridge advances the engine one
window per `step()`; pacing the windows against a wall clock is the runner's business.

A receiver that replies at a delivery's time needs the engine's lookahead to cover one window
(`lookahead_ns >= window_ticks * tick_ns`): deliveries then reach the inbox one window ahead, before
the window that contains them is simulated.

Packet lengths seen by netem and HTB are the IP datagram's: payload + 28 bytes of IPv4 and UDP
headers (`len` is a u16, so payloads up to 65,507 bytes).
"""
from __future__ import annotations

import ctypes as C
import socket
import struct
from collections import deque
from typing import Deque, Dict, List, Optional, Tuple

import numpy as np

from . import abi

IP_UDP_HEADER = 28
MAX_PAYLOAD = 0xFFFF - IP_UDP_HEADER


def _flip_bit(data: bytes, src: int, seq: int, clone: int) -> bytes:
    if not data:
        return data
    h = (src * 0x9E3779B1 ^ seq * 0x85EBCA77 ^ clone * 0xC2B2AE3D) & 0xFFFFFFFF
    h ^= h >> 15
    h = (h * 0x2C1B3C6D) & 0xFFFFFFFF
    h ^= h >> 12
    bit = h % (8 * len(data))
    b = bytearray(data)
    b[bit >> 3] ^= 1 << (bit & 7)
    return bytes(b)


class PacketBridge:
    """Host side of the packet path for n_peers instances on one engine (HIP or oracle)."""

    def __init__(self, engine, n_peers: int, window_ticks: int = 1000, tick_ns: int = 1000):
        if not 0 < window_ticks <= 0xFFFF:
            raise ValueError("window_ticks must fit the u16 tick field (1..65535)")
        self.engine = engine
        self.n = n_peers
        self.window = window_ticks
        self.tick_ns = tick_ns
        self.now_tick = int(engine.stats()["now_tick"])  # start of the next window
        self._seq = np.zeros(n_peers, dtype=np.uint64)
        self._pending: List[Tuple[int, int, int, int, int]] = []  # src, dst, seq, len, absolute tick
        self._payload: Dict[Tuple[int, int], bytes] = {}  # (src, seq) -> bytes, until delivered or dropped
        self._copies: Dict[Tuple[int, int], int] = {}     # deliveries still possible per packet
        self._dst: Dict[Tuple[int, int], int] = {}        # destination of each packet in flight
        self.inbox: List[Deque[Tuple[int, int, int, bytes, int]]] = [deque() for _ in range(n_peers)]
        self.verdicts: List[np.ndarray] = []

    def send(self, src: int, dst: int, data: bytes, at_tick: Optional[int] = None) -> int:
        """Queues one datagram from src to dst (dst may be abi.EXTERNAL) at absolute tick at_tick
        (default: the start of the next window; any later tick waits for its window).  Returns its
        sequence number."""
        if not (0 <= src < self.n) or (dst != abi.EXTERNAL and not 0 <= dst < self.n):
            raise ValueError(f"bad instance {src} -> {dst}")
        if len(data) > MAX_PAYLOAD:
            raise ValueError(f"payload of {len(data)} bytes exceeds {MAX_PAYLOAD}")
        t = self.now_tick if at_tick is None else int(at_tick)
        if t < self.now_tick:
            raise ValueError(f"tick {t} is before the next window (tick {self.now_tick})")
        seq = int(self._seq[src])
        if seq > 0xFFFFFFFF:
            raise OverflowError("sequence numbers exhausted for this source")
        self._seq[src] += 1
        self._pending.append((src, dst, seq, len(data) + IP_UDP_HEADER, t))
        self._payload[(src, seq)] = bytes(data)
        self._dst[(src, seq)] = dst
        return seq

    def step(self) -> int:
        """Simulates one window: submits the queued records, steps the engine, injects every
        delivery into its destination's inbox.  Returns the number of deliveries injected."""
        end = self.now_tick + self.window
        sent = [p for p in self._pending if p[4] < end]
        self._pending = [p for p in self._pending if p[4] >= end]
        if sent:
            pk = np.zeros(len(sent), dtype=abi.PKT_DTYPE)
            a = np.array(sent, dtype=np.uint64)
            pk["src"], pk["dst"], pk["seq"], pk["len"] = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
            pk["tick"] = a[:, 4] - self.now_tick
            self.engine.submit(pk)
        self.engine.step(self.window)
        self.now_tick += self.window
        v = self.engine.verdicts() if sent else np.zeros(0, dtype=np.uint8)
        self.verdicts.append(v)
        for (src, _dst, seq, _len, _t), vb in zip(sent, v):
            n = int((vb & 15) == abi.V_SCHEDULED) + int((vb >> 4) == abi.V_SCHEDULED)
            if n:
                self._copies[(src, seq)] = n
            else:  # dropped, filtered or queue-full: no copy will ever arrive
                self._payload.pop((src, seq), None)
                self._dst.pop((src, seq), None)
        d = self.engine.drain()
        for r in d:
            src, seq, flags = int(r["src"]), int(r["seq"]), int(r["flags"])
            data = self._payload[(src, seq)]
            clone = flags & abi.FLAG_DUP
            if flags & abi.FLAG_CORRUPT:
                data = _flip_bit(data, src, seq, clone)
            self.inbox[int(r["dst"])].append((int(r["t_ns"]), src, seq, data, flags))
            left = self._copies[(src, seq)] - 1
            if left:
                self._copies[(src, seq)] = left
            else:
                del self._copies[(src, seq)]
                del self._payload[(src, seq)]
                del self._dst[(src, seq)]
        return len(d)

    def link_removed(self, peer: int) -> int:
        """peer's data link was removed (engine.link_generation changed after a ConfigureNetwork):
        the packets already handed to the engine that peer sent, or that were addressed to it, are
        flushed or purged by the engine without a delivery (docker_network.go:65-88), so they are
        resolved as lost here.  Packets due in a later window stay queued.  Returns the count."""
        gone = [k for k in self._copies if k[0] == peer or self._dst[k] == peer]
        for k in gone:
            del self._copies[k]
            del self._payload[k]
            del self._dst[k]
        return len(gone)

    def recv(self, peer: int) -> List[Tuple[int, int, int, bytes, int]]:
        """Everything delivered to peer so far: (t_ns, src, seq, payload, flags), in delivery order."""
        out = list(self.inbox[peer])
        self.inbox[peer].clear()
        return out

    def in_flight(self) -> int:
        """Datagrams sent and not yet delivered (or known lost)."""
        return len(self._payload)


class TgsimMsg(C.Structure):
    _fields_ = [("t_ns", C.c_uint64), ("src", C.c_uint32), ("dst", C.c_uint32), ("seq", C.c_uint32),
                ("flags", C.c_uint16), ("_pad", C.c_uint16), ("off", C.c_uint64), ("len", C.c_uint32),
                ("_pad2", C.c_uint32)]


class EngineOps(C.Structure):
    _fields_ = [("submit", C.c_void_p), ("step", C.c_void_p), ("verdicts", C.c_void_p), ("drain", C.c_void_p)]


MSG_DTYPE = np.dtype([("t_ns", "<u8"), ("src", "<u4"), ("dst", "<u4"), ("seq", "<u4"), ("flags", "<u2"),
                      ("_pad", "<u2"), ("off", "<u8"), ("len", "<u4"), ("_pad2", "<u4")])
assert MSG_DTYPE.itemsize == C.sizeof(TgsimMsg) == 40


def _declare_bridge(lib: C.CDLL) -> None:
    vp = C.c_void_p
    for name, res, args in (
            ("tgsim_bridge_create", C.c_int, [vp, vp, C.c_uint32, C.c_uint32, C.c_uint64, C.POINTER(vp)]),
            ("tgsim_bridge_destroy", None, [vp]),
            ("tgsim_bridge_send", C.c_int64, [vp, C.c_size_t, vp, vp, vp, vp, vp, vp]),
            ("tgsim_bridge_step", C.c_int64, [vp]),
            ("tgsim_bridge_recv", C.c_int64, [vp, C.c_uint32, vp, C.c_size_t, vp, C.c_size_t]),
            ("tgsim_bridge_pending", C.c_int64, [vp, C.c_uint32]),
            ("tgsim_bridge_in_flight", C.c_int64, [vp]),
            ("tgsim_bridge_now_tick", C.c_uint64, [vp]),
            ("tgsim_bridge_link_removed", C.c_int64, [vp, C.c_uint32]),
            ("tgsim_udp_front_create", C.c_int, [vp, C.c_uint16, C.POINTER(vp)]),
            ("tgsim_udp_front_port", C.c_int, [vp]),
            ("tgsim_udp_front_register", C.c_int, [vp, C.c_uint32, C.c_uint32, C.c_uint16]),
            ("tgsim_udp_front_bind_peer", C.c_int, [vp, C.c_uint32, C.c_uint32, C.c_uint16]),
            ("tgsim_udp_front_pump", C.c_int64, [vp]),
            ("tgsim_udp_front_destroy", None, [vp])):
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


class NativeBridge:
    """The packet bridge in libtgsim (tgsim_bridge_*: C++ payload arena, per-source sequence
    windows, per-destination FIFOs), with PacketBridge's interface.  It drives the HIP engine
    directly, or any engine-shaped library (the oracle in the CPU tests) through an ops table."""

    ALL = 0xFFFFFFFF

    def __init__(self, engine, n_peers: int, window_ticks: int = 1000, tick_ns: int = 1000):
        from .engine import EngineError, load_library
        self._err = EngineError
        self._lib = load_library()
        _declare_bridge(self._lib)
        self.engine = engine
        self.n = n_peers
        self.window = window_ticks
        self.tick_ns = tick_ns
        ops = None
        if engine._p != "tgsim_":  # another library's engine: call it through its own functions
            f = lambda name: C.cast(getattr(engine._lib, engine._p + name), C.c_void_p).value  # noqa: E731
            self._ops = EngineOps(f("submit"), f("step"), f("verdicts"), f("drain"))
            ops = C.byref(self._ops)
        h = C.c_void_p()
        rc = self._lib.tgsim_bridge_create(engine._h, ops, n_peers, window_ticks, int(engine.stats()["now_tick"]),
                                           C.byref(h))
        if rc:
            raise self._err(rc, "tgsim_bridge_create")
        self._h = h
        self._buf = np.empty(1 << 20, dtype=np.uint8)

    def _chk(self, rc: int, what: str) -> int:
        if rc < 0:
            raise self._err(rc, what)
        return rc

    @property
    def now_tick(self) -> int:
        return int(self._lib.tgsim_bridge_now_tick(self._h))

    def send_many(self, src, dst, payloads: bytes, off, ticks=None) -> np.ndarray:
        """Batch send: datagram i is payloads[off[i]:off[i+1]] from src[i] to dst[i]."""
        src = np.ascontiguousarray(src, dtype=np.uint32)
        dst = np.ascontiguousarray(dst, dtype=np.uint32)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        data = np.frombuffer(payloads, dtype=np.uint8) if len(payloads) else np.zeros(1, dtype=np.uint8)
        t = None if ticks is None else np.ascontiguousarray(ticks, dtype=np.uint64)
        seq = np.empty(len(src), dtype=np.uint32)
        self._chk(self._lib.tgsim_bridge_send(self._h, len(src), src.ctypes.data, dst.ctypes.data, data.ctypes.data,
                                              off.ctypes.data, None if t is None else t.ctypes.data,
                                              seq.ctypes.data), "tgsim_bridge_send")
        return seq

    def send(self, src: int, dst: int, data: bytes, at_tick: Optional[int] = None) -> int:
        if len(data) > MAX_PAYLOAD:
            raise ValueError(f"payload of {len(data)} bytes exceeds {MAX_PAYLOAD}")
        t = None if at_tick is None else [int(at_tick)]
        if t is not None and t[0] < self.now_tick:
            raise ValueError(f"tick {t[0]} is before the next window (tick {self.now_tick})")
        return int(self.send_many([src], [dst], bytes(data), [0, len(data)], t)[0])

    def step(self) -> int:
        return self._chk(self._lib.tgsim_bridge_step(self._h), "tgsim_bridge_step")

    def recv_raw(self, peer: int = ALL):
        """Everything queued for peer (ALL: every peer, by destination): (messages, payload bytes)."""
        n = self._chk(self._lib.tgsim_bridge_pending(self._h, peer), "tgsim_bridge_pending")
        msgs = np.empty(max(n, 1), dtype=MSG_DTYPE)
        out, got = [], 0
        while got < n:
            k = self._chk(self._lib.tgsim_bridge_recv(self._h, peer, msgs[got:].ctypes.data, n - got,
                                                      self._buf.ctypes.data, len(self._buf)), "tgsim_bridge_recv")
            if k == 0:  # the next payload does not fit: grow the buffer
                self._buf = np.empty(2 * len(self._buf), dtype=np.uint8)
                continue
            m = msgs[got:got + k].copy()
            end = int(m["off"][-1] + m["len"][-1])
            out.append((m, self._buf[:end].tobytes()))
            got += k
        return out

    def recv_into(self, msgs: np.ndarray, buf: np.ndarray, peer: int = ALL) -> int:
        """Moves up to len(msgs) queued deliveries (and their payloads, into buf) out of the bridge;
        returns how many.  Zero-copy for the caller: no Python object per datagram."""
        return self._chk(self._lib.tgsim_bridge_recv(self._h, peer, msgs.ctypes.data, len(msgs), buf.ctypes.data,
                                                     len(buf)), "tgsim_bridge_recv")

    def recv(self, peer: int) -> List[Tuple[int, int, int, bytes, int]]:
        """Everything delivered to peer so far: (t_ns, src, seq, payload, flags), in delivery order."""
        res = []
        for m, data in self.recv_raw(peer):
            for r in m:
                o = int(r["off"])
                res.append((int(r["t_ns"]), int(r["src"]), int(r["seq"]), data[o:o + int(r["len"])], int(r["flags"])))
        return res

    def in_flight(self) -> int:
        return self._chk(self._lib.tgsim_bridge_in_flight(self._h), "tgsim_bridge_in_flight")

    def link_removed(self, peer: int) -> int:
        return self._chk(self._lib.tgsim_bridge_link_removed(self._h, peer), "tgsim_bridge_link_removed")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.tgsim_bridge_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NativeUdpFront:
    """tgsim_udp_front_*: the UDP front end in C (recvmmsg/sendmmsg), over a NativeBridge."""

    def __init__(self, bridge: NativeBridge, port: int = 0):
        self.bridge = bridge
        self._lib = bridge._lib
        h = C.c_void_p()
        bridge._chk(self._lib.tgsim_udp_front_create(bridge._h, port, C.byref(h)), "tgsim_udp_front_create")
        self._h = h
        self.addr = ("127.0.0.1", self._lib.tgsim_udp_front_port(h))

    def register(self, peer: int, addr: Tuple[str, int]) -> None:
        import ipaddress
        self.bridge._chk(self._lib.tgsim_udp_front_register(self._h, peer, int(ipaddress.IPv4Address(addr[0])), addr[1]),
                         "tgsim_udp_front_register")

    def bind_peer(self, peer: int, addr: Tuple[str, int] = ("127.0.0.1", 0)) -> Tuple[str, int]:
        """Header-less mode: a front-end socket at addr stands for peer's data address (plain
        datagrams sent to it go to peer; peer's deliveries come from it).  Returns the bound address."""
        import ipaddress
        port = self.bridge._chk(self._lib.tgsim_udp_front_bind_peer(self._h, peer, int(ipaddress.IPv4Address(addr[0])),
                                                                     addr[1]), "tgsim_udp_front_bind_peer")
        return (addr[0], port)

    def pump(self) -> int:
        return self.bridge._chk(self._lib.tgsim_udp_front_pump(self._h), "tgsim_udp_front_pump")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.tgsim_udp_front_destroy(self._h)
            self._h = None


class UdpFront:
    """Real UDP sockets in front of a PacketBridge: instance i sends to `bridge_addr` with a
    4-byte big-endian destination header; `pump()` moves what arrived into the bridge, steps one
    window, and sends each delivery to the destination's registered address with a 4-byte source
    header."""

    HDR = struct.Struct("!I")

    def __init__(self, bridge: PacketBridge, host: str = "127.0.0.1"):
        self.bridge = bridge
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind((host, 0))
        self.sock.setblocking(False)
        self.addr = self.sock.getsockname()
        self._peer_addr: Dict[int, Tuple[str, int]] = {}
        self._by_addr: Dict[Tuple[str, int], int] = {}

    def register(self, peer: int, addr: Tuple[str, int]) -> None:
        self._peer_addr[peer] = addr
        self._by_addr[addr] = peer

    def pump(self) -> int:
        while True:
            try:
                msg, addr = self.sock.recvfrom(65536)
            except BlockingIOError:
                break
            src = self._by_addr.get(addr)
            if src is None or len(msg) < self.HDR.size:
                continue  # not an instance of this run
            (dst,) = self.HDR.unpack_from(msg)
            self.bridge.send(src, dst, msg[self.HDR.size:])
        n = self.bridge.step()
        for peer, addr in self._peer_addr.items():
            for _t, src, _seq, data, _f in self.bridge.recv(peer):
                self.sock.sendto(self.HDR.pack(src) + data, addr)
        return n

    def close(self) -> None:
        self.sock.close()
