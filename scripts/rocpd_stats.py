"""Kernel statistics (calls, total / mean / min / max / p50 us) from a rocprofv3 rocpd SQLite database.

    python scripts/rocpd_stats.py gpurun_out/<tag>/prof/bench_results.db > profiles/<tag>/rocprof_kernels.md
"""
import sqlite3
import statistics
import sys


def main(path: str) -> int:
    db = sqlite3.connect(path)
    rows = db.execute("select s.display_name, d.end - d.start from rocpd_kernel_dispatch d "
                      "join rocpd_info_kernel_symbol s on s.id = d.kernel_id").fetchall()
    by: dict[str, list[int]] = {}
    for name, ns in rows:
        by.setdefault(name, []).append(ns)
    total = sum(sum(v) for v in by.values()) or 1
    print("| kernel | calls | total us | % | mean us | p50 us | min us | max us |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"| `{name[:70]}` | {len(v)} | {sum(v) / 1e3:.1f} | {100 * sum(v) / total:.1f} | "
              f"{statistics.mean(v) / 1e3:.2f} | {statistics.median(v) / 1e3:.2f} | {min(v) / 1e3:.2f} | {max(v) / 1e3:.2f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
