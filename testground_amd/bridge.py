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
        return len(d)

    def recv(self, peer: int) -> List[Tuple[int, int, int, bytes, int]]:
        """Everything delivered to peer so far: (t_ns, src, seq, payload, flags), in delivery order."""
        out = list(self.inbox[peer])
        self.inbox[peer].clear()
        return out

    def in_flight(self) -> int:
        """Datagrams sent and not yet delivered (or known lost)."""
        return len(self._payload)


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
