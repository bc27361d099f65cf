"""A plain UDP echo server with no knowledge of the engine: binds 127.0.0.1:<port> (0 = any), prints
the bound port, then sends every datagram back to where it came from (up to <count> datagrams).  The
bridge tests run it as a separate process, the way a plan's unmodified UDP code would run."""
import socket
import sys

port = int(sys.argv[1]) if len(sys.argv) > 1 else 0
count = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 30
s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
s.bind(("127.0.0.1", port))
print(s.getsockname()[1], flush=True)
for _ in range(count):
    data, addr = s.recvfrom(65536)
    s.sendto(data, addr)
