"""Per-CPU load and interrupt rate over a short window (which CPUs are busy before the bench starts)."""
import json
import os
import sys
import time


def stat():
    out = {}
    with open("/proc/stat") as f:
        for ln in f:
            if ln.startswith("cpu") and ln[3].isdigit():
                p = ln.split()
                v = list(map(int, p[1:]))
                out[int(p[0][3:])] = (sum(v), v[3] + v[4])
    return out


def irqs():
    with open("/proc/interrupts") as f:
        hdr = f.readline().split()
        tot = [0] * len(hdr)
        for ln in f:
            p = ln.split()
            for i in range(len(hdr)):
                if i + 1 < len(p) and p[i + 1].isdigit():
                    tot[i] += int(p[i + 1])
    return {int(h[3:]): t for h, t in zip(hdr, tot)}


window = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
s0, i0 = stat(), irqs()
time.sleep(window)
s1, i1 = stat(), irqs()
busy = {c: 1 - (s1[c][1] - s0[c][1]) / max(1, s1[c][0] - s0[c][0]) for c in s1}
irq = {c: (i1.get(c, 0) - i0.get(c, 0)) / window for c in i1}
allowed = sorted(os.sched_getaffinity(0))
top = sorted(busy, key=lambda c: -busy[c])[:16]
print(json.dumps({"ncpu": len(s1), "allowed": len(allowed), "busy_mean": sum(busy.values()) / len(busy),
                  "busiest": {c: round(busy[c], 3) for c in top},
                  "cpu0_7_busy": {c: round(busy[c], 3) for c in range(8)},
                  "irq_per_s_top": {c: round(irq[c]) for c in sorted(irq, key=lambda c: -irq[c])[:12]},
                  "irq_cpu0_7": {c: round(irq.get(c, 0)) for c in range(8)}}))
