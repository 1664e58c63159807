"""The swap / guard / exchange / publication protocol under a deterministic scheduler.

tests/interleave.py runs the device plugin's Allocate path, its physical guard, the PodResources reconciler with its
exchanges and holds, the physical publication and the extender's native ledger in one thread, with every apiserver
call, extender call, sleep, PodResources answer and watch delivery a gate a seeded scheduler opens.  Every schedule
is checked step by step (no GPU runs past its capacity) and once drained (annotations = what runs, no holds, the
ledger = the annotations, nothing unaccounted, no Allocate failed, every bound pod admitted).

The mutation tests re-introduce known bug classes -- round 5's controller freeing a terminating pod's share, no
physical guard, no lingering of force-deleted pods' shares, and bugs this harness found in round 6 (an exchange's
step 2 re-applied over a partner served since -- two defences now, the matcher skipping partners and the finish
accepting a partner served on the fields step 2 gave it, removed together; an Allocate failing kubelet's pod because
the pod it matched was deleted meanwhile) -- and require the harness to find each within a few hundred schedules.
The schedules that found bugs are replayed as regressions.

``GSX_INTERLEAVE_SEEDS`` (default 200) sets schedules per scenario; the sweep logged under profiles/r06_interleave
ran 10000 per scenario.
"""
import os

import pytest

from tests import interleave as il

SEEDS = int(os.environ.get("GSX_INTERLEAVE_SEEDS", "200"))


@pytest.mark.parametrize("scenario", sorted(il.SCENARIOS))
def test_every_schedule_keeps_the_gpus_within_capacity_and_converges(scenario):
    n = SEEDS // 3 if scenario == "batch-faults" else SEEDS  # (four times the steps of the others)
    r = il.sweep(scenario, range(n))
    assert not r["violations"], "\n".join(r["violations"][:3])
    assert r["runs"] == n
    # the schedules exercise the protocol, not an idle node
    assert r["swaps"] > n // 4 and r["holds"] > 0 and r["moves"] > 0, r
    if il.SCENARIOS[scenario].faults:
        assert r["faults"] > n, r


@pytest.mark.parametrize("scenario", ["swap-graceful", "swap-force"])
def test_every_schedule_one_departure_from_the_fair_order_is_clean(scenario):
    # exhaustive, not sampled: each of the first 40 steps, each other action enabled there
    r = il.systematic(scenario, bound=1, window=40)
    assert not r["violations"], "\n".join(r["violations"][:3])
    assert r["runs"] > 150, r


def test_a_schedule_replays_from_its_seed():
    a = il.run_one("churn", 7)
    b = il.run_one("churn", 7)
    assert a.trace == b.trace and a.steps == b.steps > 50


@pytest.mark.parametrize("scenario,seed", [
    ("batch-faults", 1914),   # a partner served on the fields step 2 gave it, then step 2 re-applied (ASSIGNED=false)
    ("batch-faults", 15378),  # the guard's move failing kubelet's pod on an apiserver 500
    ("swap-graceful", 25),    # the first bug the harness found: a stale exchange payload over a served pod
])
def test_the_schedules_that_found_bugs_stay_clean(scenario, seed):
    il.run_one(scenario, seed)


def test_the_physical_guard_and_lingering_are_exercised():
    r = il.sweep("force-grace", range(200))
    assert not r["violations"], r["violations"][:2]
    assert r["guards"] > 0 and r["lingered"] > 0, r


@pytest.mark.parametrize("mutation,scenario,what", [
    ("serve_partner,strict_finish", "swap-graceful", "annotated"),
    ("fail_on_gone", "swap-force", "Allocate failed"),
    ("no_linger", "force-grace", "runs"),
    ("no_guard", "force-grace", "runs"),
    ("free_on_deleting", "slow-stop", "promise"),
])
def test_the_harness_finds_each_known_bug_class(mutation, scenario, what):
    found = None
    for seed in range(400):
        try:
            il.run_one(scenario, seed, mutation)
        except il.Violation as e:
            found = str(e)
            break
    assert found is not None, f"{mutation}: no violation in 400 schedules of {scenario}"
    assert what in found.split("\n", 1)[0], found


def test_unknown_mutations_are_refused():
    with pytest.raises(ValueError, match="unknown mutations"):
        il.Harness(il.SCENARIOS["churn"], 0, "no_such_bug")
