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
