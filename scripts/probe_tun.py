"""Probe: can a plan's packets be captured with TUN/TAP on this host?

Prints one JSON object: whether /dev/net/tun exists and opens, whether TUNSETIFF creates an
interface (needs CAP_NET_ADMIN in the owning user namespace), the effective capability mask, and
whether a user + network namespace (unshare -Urn) is allowed.  Run it plainly and under
`unshare -Urn` (an unprivileged namespace in which this process holds CAP_NET_ADMIN)."""
import errno
import fcntl
import json
import os
import struct

TUNSETIFF = 0x400454CA
IFF_TUN, IFF_NO_PI = 0x0001, 0x1000


def cap_eff():
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("CapEff:"):
                v = int(line.split()[1], 16)
                return {"hex": hex(v), "cap_net_admin": bool(v & (1 << 12)), "cap_net_raw": bool(v & (1 << 13))}
    return None


def try_tun():
    out = {"dev_exists": os.path.exists("/dev/net/tun")}
    try:
        fd = os.open("/dev/net/tun", os.O_RDWR)
    except OSError as e:
        out["open"] = f"{errno.errorcode.get(e.errno, e.errno)}: {e.strerror}"
        return out
    out["open"] = "ok"
    try:
        fcntl.ioctl(fd, TUNSETIFF, struct.pack("16sH", b"tgsim0", IFF_TUN | IFF_NO_PI))
        out["tunsetiff"] = "ok"
    except OSError as e:
        out["tunsetiff"] = f"{errno.errorcode.get(e.errno, e.errno)}: {e.strerror}"
    os.close(fd)
    return out


def main():
    res = {"uid": os.getuid(), "in_userns": open("/proc/self/uid_map").read().split(), "cap_eff": cap_eff(),
           "tun": try_tun()}
    try:
        with open("/proc/sys/user/max_user_namespaces") as f:
            res["max_user_namespaces"] = int(f.read())
    except OSError as e:
        res["max_user_namespaces"] = str(e)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
