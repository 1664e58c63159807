#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counters (rocpd SQLite): per kernel, per counter, value per dispatch (summed over SEs)."""
import collections
import sqlite3
import sys


def short(name: str) -> str:
    n = name.split("(")[0]
    return n if len(n) <= 70 else n[:67] + "..."


def summary(db: str) -> str:
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection")
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    names = {}
    for disp, kn, cn, v, d in rows:
        per[disp][cn] += v
        dur[disp] = d
        names[disp] = short(kn)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for disp, cs in per.items():
        for cn, v in cs.items():
            agg[names[disp]][cn].append(v)
        agg[names[disp]]["duration_us"].append(dur[disp] / 1e3)
    counters = sorted({cn for k in agg.values() for cn in k})
    out = ["| kernel | dispatches | " + " | ".join(counters) + " |", "|---|---:|" + "---:|" * len(counters)]
    for kn, cs in sorted(agg.items(), key=lambda kv: -sum(kv[1]["duration_us"])):
        n = len(cs["duration_us"])
        vals = [f"{sum(cs[cn]) / max(1, len(cs[cn])):.4g}" for cn in counters]
        out.append(f"| `{kn}` | {n} | " + " | ".join(vals) + " |")
    return "\n".join(out)


if __name__ == "__main__":
    print(summary(sys.argv[1]))
