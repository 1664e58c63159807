"""Per-wave critical path from ``bench.py --dump-timings`` (scheduler timeline, CLOCK_MONOTONIC like the wave's t0):
when the scheduler first / last saw a pod of the wave, finished filtering the last one, and the last bind returned,
next to the wave's bound / running / total marks.  Medians over the waves, in ms from the wave's start."""
import json
import statistics
import sys


def main(path):
    waves = json.load(open(path))
    cols = {k: [] for k in ("first_seen", "last_seen", "last_filtered", "last_bound", "filter_span_per_pod_us",
                            "filter_rtt_us", "bind_rtt_us", "t_bound", "t_run", "t_total")}
    for w in waves:
        t0, pods = w["t0"], w["pods"]
        seen = sorted(p["seen"] - t0 for p in pods)
        filt = sorted(p["filtered"] - t0 for p in pods)
        bound = sorted(p["bound"] - t0 for p in pods)
        cols["first_seen"].append(seen[0] * 1e3)
        cols["last_seen"].append(seen[-1] * 1e3)
        cols["last_filtered"].append(filt[-1] * 1e3)
        cols["last_bound"].append(bound[-1] * 1e3)
        cols["filter_span_per_pod_us"].append((filt[-1] - filt[0]) / max(1, len(pods) - 1) * 1e6)
        cols["filter_rtt_us"].append(statistics.median(p["filter_rtt"] for p in pods) * 1e6)
        cols["bind_rtt_us"].append(statistics.median(p["bind_rtt"] for p in pods) * 1e6)
        for k in ("t_bound", "t_run", "t_total"):
            cols[k].append(w[k] * 1e3)
    print(json.dumps({k: round(statistics.median(v), 3) for k, v in cols.items()}))


if __name__ == "__main__":
    main(sys.argv[1])
