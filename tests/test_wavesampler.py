"""gsxtools/wavesampler.py: per-wave run-delay / pressure attribution of bench.py's timed waves."""
import os
import time

from gsxtools.wavesampler import Sampler, attribute


def _data(rows, names=("rank0", "plugin")):
    return {"names": list(names), "interval": 0.002, "samples": rows}


def test_slow_wave_is_blamed_on_the_process_that_waited_for_a_cpu():
    # samples every 1 ms: [t, run-delay ns per process..., psi cpu/io/memory us]
    rows = []
    rd_plugin = 0
    for i in range(100):
        t = i * 0.001
        if 50 <= i < 60:
            rd_plugin += 800_000  # the plugin's threads waited 0.8 ms of every 1 ms in the slow wave
        rows.append([t, 0, rd_plugin, 0, 0, 0])
    waves = [(0.001 * k, 0.001) for k in range(0, 40, 2)] + [(0.050, 0.010)]  # 20 x 1 ms, then one 10 ms wave
    out = attribute(_data(rows), waves)
    assert len(out["slow_waves"]) == 1
    slow = out["slow_waves"][0]
    assert slow["wave"] == 20 and slow["blame"] == "plugin" and slow["x_p50"] >= 5
    assert slow["run_delay_ms"]["plugin"] >= 7.0
    assert len(out["run_delay_ms_each"]["plugin"]) == 21


def test_host_pressure_and_off_cpu_waits_are_told_apart():
    rows = []
    psi = 0
    for i in range(100):
        if 50 <= i < 60:
            psi += 900  # us of CPU pressure per 1 ms sample: every task stalled
        rows.append([i * 0.001, 0, 0, psi, 0, 0])
    waves = [(0.001 * k, 0.001) for k in range(0, 40, 2)] + [(0.050, 0.010)]
    slow = attribute(_data(rows), waves)["slow_waves"][0]
    assert slow["blame"] == "host (cpu pressure)"
    rows = [[i * 0.001, 0, 0, None, None, None] for i in range(100)]  # no PSI on this kernel, nobody waited
    slow = attribute(_data(rows), waves)["slow_waves"][0]
    assert slow["blame"].startswith("unattributed")


def test_sampler_process_records_this_process(tmp_path):
    s = Sampler({"me": os.getpid()}, str(tmp_path / "w.json"), interval=0.001)
    assert s.wait_ready()
    t0 = time.perf_counter()
    x = 0
    while time.perf_counter() - t0 < 0.05:  # some CPU for the sampler to see
        x += 1
    data = s.stop()
    assert data and data["names"] == ["me"] and len(data["samples"]) >= 10
    ts = [r[0] for r in data["samples"]]
    assert ts == sorted(ts) and ts[0] <= t0 + 0.02
