"""Local sync-service endpoint: the plans' sync API across processes, backed by
the engine's device sync counters.

The reference's plans reach a separate sync service through sdk-go (`sync.Client`: SignalEntry,
Barrier, SignalAndWait, Publish, Subscribe); the sidecar handler uses the same calls to signal
`network-initialized` and a ConfigureNetwork's callback state
(`/root/reference/pkg/sidecar/sidecar_handler.go:40-44`, `:75-80`) and is handed the service's
address by the runner (`pkg/runner/local_common.go:77-82`).  Here the service is a loopback TCP
endpoint in the runner's process; its signal and barrier counters are the engine's (K7,
`tgsim_signal` / `tgsim_barrier_poll`, through `sidecar.EngineSyncClient`), so an out-of-process plan
that signals and waits meets the simulated network's own counters, and pub/sub topics are kept in
the service's memory.

Wire format (this engine's own; the sdk-go protocol is not in the reference, so it is parity-unpinned):
one JSON object per line each way.  Requests carry an `id` echoed by the reply:

    {"id": 1, "op": "signal_entry", "state": "s"}                 -> {"id": 1, "seq": 3}
    {"id": 2, "op": "barrier", "state": "s", "target": 4}        -> {"id": 2, "ok": true}   (when reached)
    {"id": 3, "op": "signal_and_wait", "state": "s", "target": 4} -> {"id": 3, "seq": 2}
    {"id": 4, "op": "publish", "topic": "t", "payload": ...}      -> {"id": 4, "seq": 1}
    {"id": 5, "op": "subscribe", "topic": "t"}                    -> {"id": 5, "payload": ...} per entry,
                                                                     the topic's history first
A barrier that is not reached within its `timeout_s` (default 60 s) answers {"id": .., "error": ..};
so does an unknown op.  One connection serves one plan instance; a subscription takes a connection
of its own (as a Subscribe returns a channel in sdk-go)."""
from __future__ import annotations

import json
import queue
import socket
import socketserver
import threading
from typing import Any, Optional, Tuple

from .sidecar import Context, SyncClient


class SyncService:
    """Serves `sync` (a sidecar.SyncClient, normally an EngineSyncClient over the engine's counters)
    on a loopback TCP port until close()."""

    def __init__(self, sync: SyncClient, host: str = "127.0.0.1", port: int = 0):
        self.sync = sync
        service = self

        class Handler(socketserver.StreamRequestHandler):
            def handle(self) -> None:
                for line in self.rfile:
                    if not line.strip():
                        continue
                    try:
                        req = json.loads(line)
                    except ValueError:
                        self._send({"error": "malformed request"})
                        continue
                    if req.get("op") == "subscribe":
                        service._stream(self, req)
                        return  # the connection belongs to the subscription from now on
                    self._send(service._serve(req))

            def _send(self, obj: Any) -> None:
                self.wfile.write((json.dumps(obj) + "\n").encode())
                self.wfile.flush()

        class Server(socketserver.ThreadingTCPServer):
            daemon_threads = True
            allow_reuse_address = True

        self._server = Server((host, port), Handler)
        self.address: Tuple[str, int] = self._server.server_address[:2]
        self._closing = threading.Event()
        self._thread = threading.Thread(target=self._server.serve_forever, kwargs={"poll_interval": 0.05},
                                        daemon=True)
        self._thread.start()

    def _serve(self, req: dict) -> dict:
        rid, op = req.get("id"), req.get("op")
        ctx = Context(timeout=float(req.get("timeout_s", 60.0)))
        try:
            if op == "signal_entry":
                return {"id": rid, "seq": self.sync.SignalEntry(ctx, req["state"])}
            if op == "barrier":
                self.sync.Barrier(ctx, req["state"], int(req["target"]))
                return {"id": rid, "ok": True}
            if op == "signal_and_wait":
                return {"id": rid, "seq": self.sync.SignalAndWait(ctx, req["state"], int(req["target"]))}
            if op == "publish":
                return {"id": rid, "seq": self.sync.Publish(ctx, req["topic"], req.get("payload"))}
            return {"id": rid, "error": f"unknown op {op!r}"}
        except (KeyError, TypeError, ValueError) as exc:
            return {"id": rid, "error": f"bad request: {exc}"}
        except TimeoutError as exc:
            return {"id": rid, "error": str(exc)}

    def _stream(self, handler, req: dict) -> None:
        rid = req.get("id")
        q = self.sync.Subscribe(Context(), req["topic"])
        while not self._closing.is_set():
            try:
                payload = q.get(timeout=0.05)
            except queue.Empty:
                continue
            try:
                handler._send({"id": rid, "payload": payload})
            except OSError:
                return  # the subscriber went away

    def close(self) -> None:
        self._closing.set()
        self._server.shutdown()
        self._server.server_close()
        self._thread.join(timeout=5)


class SyncServiceClient:
    """The plan side (sdk-go `sync.Client`'s calls, same names and meaning) over a SyncService's
    address; what an out-of-process plan links against instead of sdk-go."""

    def __init__(self, address: Tuple[str, int], timeout_s: float = 60.0):
        self.address = tuple(address)
        self.timeout_s = timeout_s
        self._sock = socket.create_connection(self.address, timeout=timeout_s + 5)
        self._rf = self._sock.makefile("rb")
        self._lock = threading.Lock()
        self._next = 0

    def _call(self, **req) -> dict:
        with self._lock:
            self._next += 1
            req["id"] = self._next
            req.setdefault("timeout_s", self.timeout_s)
            self._sock.sendall((json.dumps(req) + "\n").encode())
            line = self._rf.readline()
        if not line:
            raise ConnectionError("sync service closed the connection")
        rep = json.loads(line)
        if "error" in rep:
            raise RuntimeError(f"sync service: {rep['error']}")
        return rep

    def SignalEntry(self, state: str) -> int:
        return int(self._call(op="signal_entry", state=state)["seq"])

    def Barrier(self, state: str, target: int) -> None:
        self._call(op="barrier", state=state, target=int(target))

    def SignalAndWait(self, state: str, target: int) -> int:
        return int(self._call(op="signal_and_wait", state=state, target=int(target))["seq"])

    def Publish(self, topic: str, payload: Any) -> int:
        return int(self._call(op="publish", topic=topic, payload=payload)["seq"])

    def Subscribe(self, topic: str) -> "queue.Queue":
        """The topic's entries, its history first, on a queue fed by a connection of its own."""
        out: queue.Queue = queue.Queue()
        sock = socket.create_connection(self.address, timeout=None)
        sock.sendall((json.dumps({"id": 0, "op": "subscribe", "topic": topic}) + "\n").encode())
        rf = sock.makefile("rb")

        def pump() -> None:
            for line in rf:
                out.put(json.loads(line)["payload"])

        threading.Thread(target=pump, daemon=True).start()
        self._subs = getattr(self, "_subs", []) + [sock]
        return out

    def Close(self) -> None:
        for s in getattr(self, "_subs", []):
            s.close()
        self._rf.close()
        self._sock.close()
