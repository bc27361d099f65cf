"""A plan instance as its own process, with nothing of the engine in it: a UDP socket and the sync
client (testground_amd.sync_service.SyncServiceClient, the sdk-go `sync.Client` calls over the local
sync endpoint).  It publishes its data port, waits at `network-initialized` for all instances
(sdk-go WaitNetworkInitialized: the sidecar signals it once the instance's network is set up,
sidecar_handler.go:40-44), sends its datagrams to the other instance's data address, receives the
other's, then meets the others at `done` (SignalAndWait) and prints what it saw as JSON.
usage: sync_plan.py SYNC_HOST SYNC_PORT INSTANCE N PEER_HOST PEER_PORT N_MSGS"""
import json
import socket
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from testground_amd.sync_service import SyncServiceClient  # noqa: E402

host, port, me, n, peer_host, peer_port, n_msgs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), \
    sys.argv[5], int(sys.argv[6]), int(sys.argv[7])
s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
s.bind(("127.0.0.1", 0))
sync = SyncServiceClient((host, port), timeout_s=120)
sync.Publish("ports", {"instance": me, "port": s.getsockname()[1]})
sync.Barrier("network-initialized", n)
for k in range(n_msgs):
    s.sendto(b"from-%d-msg-%03d" % (me, k), (peer_host, peer_port))
got, deadline = [], time.time() + 60
s.settimeout(0.5)
while len(got) < n_msgs and time.time() < deadline:
    try:
        data, addr = s.recvfrom(65536)
    except socket.timeout:
        continue
    got.append((data.decode(), list(addr)))
seq = sync.SignalAndWait("done", n)
print(json.dumps({"instance": me, "got": got, "done_seq": seq}), flush=True)
sync.Close()
