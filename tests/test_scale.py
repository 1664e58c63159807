"""Cluster scale: 5,000 nodes x 8 devices with 10,000 resident pods sync through paginated
LISTs and filter at full NodeNames in bounded time; pods keep binding under churn (gsxtools/scale.py)."""
import json

from gsxtools import scale


def test_5000_nodes_sync_filter_and_churn(tmp_path):
    out = tmp_path / "scale.json"
    assert scale.main(["--nodes", "5000", "--churn-batches", "3", "--batch", "200", "--filter-reps", "50",
                       "--json-out", str(out)]) == 0
    r = json.loads(out.read_text())["5000"]
    assert r["devices"] == 40000 and r["resident_pods"] == 10000
    # the initial LIST came in pages (limit=500): 10,000 pods -> 20 pages, 5,000 nodes -> 10 pages
    assert r["pod_list_pages"] >= 20 and r["node_list_pages"] >= 10
    assert r["extender_ready_s"] < 20.0
    f = r["filter_full_nodenames"]
    assert f["nodes_passed"] == 5000  # every node has a free device for a 64 GiB pod
    assert f["p99_ms"] < 50.0  # O(nodes x devices) with incremental counters, no per-pod re-summing
    assert r["churn"]["pods_per_s"] > 100
    assert r["extender_rss_mib_after_sync"] < 1024
