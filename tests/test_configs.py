"""BASELINE.json configurations 1-5 and the hardware-partition scenario (6) through the whole stack (sim/configs.py): CPU plumbing and, on MI355X,
real device sizes, the HBM arena and hardware-verified CU partitions."""
import pytest

from gpushare_scheduler_extender_amd.sim import configs


@pytest.mark.parametrize("k", sorted(configs.CONFIGS))
def test_baseline_config_cpu(k, tmp_path):
    assert configs.main(["--only", str(k), "--json-out", str(tmp_path / "r.json")]) == 0


@pytest.mark.gpu
def test_baseline_configs_on_mi355x(tmp_path):
    out = tmp_path / "r.json"
    rc = configs.main(["--gpu", "--json-out", str(out)])
    import json

    rep = json.loads(out.read_text())
    assert rc == 0, rep
    assert rep["2"]["hbm_arena"] and rep["2"]["bad_stamps"] == 0
    assert rep["5"]["probe_cus_per_pod"] == [64] * 4 and rep["5"]["probe_disjoint"]
