"""Loopback ping-pong between two processes pinned to idle cores: round-trip time when the peer blocks in
recv (wakes from idle) vs when it spins on a non-blocking socket, plus the cpuidle states the kernel offers."""
import glob
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from gpushare_scheduler_extender_amd.utils.cpuset import plan  # noqa: E402


def idle_states(cpu):
    out = []
    for d in sorted(glob.glob(f"/sys/devices/system/cpu/cpu{cpu}/cpuidle/state*")):
        try:
            name = open(f"{d}/name").read().strip()
            lat = int(open(f"{d}/latency").read())
            dis = open(f"{d}/disable").read().strip()
            usage = int(open(f"{d}/usage").read())
        except OSError:
            continue
        out.append({"name": name, "latency_us": lat, "disabled": dis, "usage": usage})
    return out


def server(sock, spin):
    conn, _ = sock.accept()
    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    if spin:
        conn.setblocking(False)
    while True:
        try:
            b = conn.recv(64)
        except BlockingIOError:
            continue
        if not b:
            return
        conn.sendall(b)


def main():
    p = plan(["a", "b"], {}, "spread")
    res = {"cpus": p, "idle_states": idle_states(p["b"][0])}
    for spin in (0, 1):
        ls = socket.socket()
        ls.bind(("127.0.0.1", 0))
        ls.listen(1)
        port = ls.getsockname()[1]
        pid = os.fork()
        if pid == 0:
            os.sched_setaffinity(0, set(p["b"]))
            server(ls, spin)
            os._exit(0)
        os.sched_setaffinity(0, set(p["a"]))
        c = socket.create_connection(("127.0.0.1", port))
        c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        for gap_us in (0, 200):
            rtts = []
            for _ in range(2000):
                if gap_us:
                    t = time.perf_counter() + gap_us * 1e-6
                    while time.perf_counter() < t:
                        pass
                t0 = time.perf_counter()
                c.sendall(b"x")
                c.recv(64)
                rtts.append(time.perf_counter() - t0)
            rtts.sort()
            res[f"spin{spin}_gap{gap_us}us"] = {"p50_us": round(rtts[1000] * 1e6, 1), "p99_us": round(rtts[1980] * 1e6, 1)}
        c.close()
        os.waitpid(pid, 0)
        ls.close()
    print(json.dumps(res))


main()
