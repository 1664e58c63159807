"""The device plugin on a quiet node costs (almost) no CPU.  Round 4's serving thread left a
deferred wake-up standing and then took the state lock for empty passes ~500k times a second until the next event:
10-25 % of a CPU at one pod a second.  gsxtools/plugincpu.py measures idle and trickle phases of the real process."""
import asyncio

from gsxtools.plugincpu import run


def test_plugin_cpu_idle_and_at_a_trickle_of_pods():
    out = asyncio.run(run(gpus=8, idle=2.0, trickle=4.0, rate=2.0))
    assert out["trickle"]["pods"] >= 6
    assert out["idle"]["total_pct"] < 2.0, out
    assert out["trickle"]["total_pct"] < 5.0, out
    assert out["trickle"]["threads_pct"].get("gsx-dp-serve", 0.0) < 2.0, out
