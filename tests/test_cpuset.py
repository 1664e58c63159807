"""CPU placement of the bench's control-plane processes (utils/cpuset.py)."""
import multiprocessing as mp
import os

from gpushare_scheduler_extender_amd.utils import cpuset


def test_sample_load_covers_every_cpu():
    load = cpuset.sample_load(0.05)
    assert load, "/proc/stat unreadable"
    assert set(os.sched_getaffinity(0)) <= set(load)
    assert all(0.0 <= v <= 1.0 for v in load.values())


def test_idle_cores_first_and_cpu0_last():
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < 4:
        return
    busy = allowed[1]
    load = {c: 0.0 for c in allowed}
    load[busy] = 0.9  # another job's thread
    order = cpuset.physical_cpus(allowed, load)
    assert sorted(order) == allowed
    primary = order[:len(set(order))]
    # the busy CPU's core comes after every idle core; CPU 0's core comes after the idle cores too
    idx = {c: i for i, c in enumerate(primary)}
    idle_cores = [c for c in primary if load[c] < cpuset.IDLE and c != 0]
    if busy in idx and idle_cores:
        assert all(idx[c] < idx[busy] for c in idle_cores if c in idx)
    if 0 in idx and idle_cores:
        assert all(idx[c] < idx[0] for c in idle_cores if c in idx)


def test_plan_modes_disjoint_slots():
    names = ["a", "b", "c"]
    for mode in ("spread", "static"):
        p = cpuset.plan(names, {"b": 2}, mode, load={} if mode == "spread" else None)
        if not p:
            continue  # fewer CPUs than slots
        flat = [c for n in names for c in p[n]]
        assert len(flat) == len(set(flat)) == 4
    assert cpuset.plan(names, {}, "none") == {}
    c = cpuset.plan(names, {"b": 2}, "compact")
    assert c["a"] == c["b"] == c["c"]


def _child(key, q):
    q.put(cpuset.shared_plan(["x", "y"], {"y": 2}, "spread", key))


def test_shared_plan_is_computed_once_per_key():
    key = f"test-{os.getpid()}"
    try:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=_child, args=(key, q)) for _ in range(3)]
        for p in ps:
            p.start()
        got = [q.get(timeout=60) for _ in ps]
        for p in ps:
            p.join(60)
        assert got[0] == got[1] == got[2]
        assert cpuset.shared_plan(["x", "y"], {"y": 2}, "spread", key) == got[0]
    finally:
        cpuset.forget_shared_plan(key)
    assert not os.path.exists(os.path.join(__import__("tempfile").gettempdir(), f"gsx-cpuplan-{key}.json"))


def test_order_cores_prefers_a_domain_that_fits(monkeypatch):
    # two L3 domains of 4 cores (CPU n and its SMT sibling n + 100); domain A has one busy core
    dom = {c: (0,) if c < 4 else (4,) for c in range(8)}
    monkeypatch.setattr(cpuset, "_group_key", lambda c: dom[c % 100])
    cores = [(c, c + 100) for c in range(8)]
    load = {c: 0.0 for core in cores for c in core}
    load[102] = 0.5  # the sibling of CPU 2 belongs to another job
    got = cpuset._order_cores(cores, load, need=4)
    # domain B (4..7) holds all 4 needed cores idle: it comes first; CPU 0's core comes last
    assert [c[0] for c in got[:4]] == [4, 5, 6, 7]
    assert got[-1] == (0, 100)
    assert got.index((2, 102)) > got.index((1, 101))  # busy core after the idle ones
    # need 6: no domain fits, the one with the most idle cores comes first (B: 4 idle vs A: 2 without CPU 0)
    got = cpuset._order_cores(cores, load, need=6)
    assert [c[0] for c in got[:4]] == [4, 5, 6, 7]


def test_order_cores_least_busy_domain_when_none_is_idle(monkeypatch):
    monkeypatch.setattr(cpuset, "_group_key", lambda c: (8,) if c % 100 < 12 else (12,))
    cores = [(c, c + 100) for c in range(8, 16)]
    load = {c: 0.0 for core in cores for c in core}
    for c in range(8, 12):
        load[c] = 0.06  # domain A: every core a little busy
    load[12] = 0.9  # domain B: one core taken by another job
    assert [c[0] for c in cpuset._order_cores(cores, load, need=4)[:4]] == [8, 9, 10, 11]
    assert [c[0] for c in cpuset._order_cores(cores, load, need=3)[:3]] == [13, 14, 15]


def test_n8_plan_degrades_to_unpinned_on_a_16_cpu_cgroup(monkeypatch, caplog):
    """the N = 8 bench asks for more CPUs (29) than a 16-CPU share of an 8-GPU node may give; the plan
    comes back empty -- nothing pinned -- with a warning, and the run goes on (bench.py pins nothing with {})."""
    import logging
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    names, widths, _ = bench.cpu_slots(8)
    asked = sum(widths.get(n, 1) for n in names)
    assert asked == 29, (asked, widths)
    allowed = list(range(100, 116))  # a 16-CPU cgroup, SMT pairs (100,101), (102,103), ...
    monkeypatch.setattr(cpuset.os, "sched_getaffinity", lambda pid: set(allowed))
    monkeypatch.setattr(cpuset, "_cores", lambda cpus: [(c, c + 1) for c in sorted(cpus) if c % 2 == 0])
    monkeypatch.setattr(cpuset, "_group_key", lambda cpu: (0,))
    with caplog.at_level(logging.WARNING, logger="gsx.cpuset"):
        assert cpuset.plan(names, widths, "spread", load={c: 0.0 for c in allowed}, smt=True) == {}
        assert cpuset.plan(names, widths, "spread", load={c: 0.0 for c in allowed}, smt=False) == {}
    assert sum("not pinning" in r.message for r in caplog.records) == 2
    # the N = 1 plan (10 CPUs) still fits such a share
    n1, w1, _ = bench.cpu_slots(1)
    p = cpuset.plan(n1, w1, "spread", load={c: 0.0 for c in allowed}, smt=True)
    assert p and sum(len(v) for v in p.values()) == sum(w1.get(n, 1) for n in n1)
    cpuset.pin_self(None)  # an empty slot pins nothing (bench.py with the degraded plan)
