#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite (rocpd) database: per-kernel dispatch count / total / avg / min / max (us)."""
import sqlite3
import sys


def summary(db: str) -> str:
    c = sqlite3.connect(db)
    q = """select s.kernel_name, count(*), sum(d.end-d.start), avg(d.end-d.start), min(d.end-d.start),
                  max(d.end-d.start), max(s.arch_vgpr_count), max(s.accum_vgpr_count), max(d.group_segment_size)
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           group by s.kernel_name order by 3 desc"""
    rows = list(c.execute(q))
    tot = sum(r[2] for r in rows) or 1
    out = ["| kernel | calls | total us | avg us | min us | max us | % | vgpr | agpr | lds B |",
           "|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|"]
    for name, n, s, a, mn, mx, v, ag, lds in rows:
        nm = name.replace(".kd", "")
        out.append(f"| `{nm}` | {n} | {s/1e3:.1f} | {a/1e3:.2f} | {mn/1e3:.2f} | {mx/1e3:.2f} | {100*s/tot:.1f} | "
                   f"{v} | {ag} | {lds} |")
    return "\n".join(out)


if __name__ == "__main__":
    print(summary(sys.argv[1]))
