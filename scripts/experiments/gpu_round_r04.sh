#!/bin/bash
# Round-4 GPU session: the GPU test suite, smoke(), and the driver's N=1 command three times (BENCH evidence).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_round}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest -m gpu rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || { echo "smoke rc=$rc"; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $i rc=$rc"; tail -20 $OUT/bench.$i.log; exit $rc; }
  tail -1 $OUT/bench.$i.log > $OUT/bench.$i.json
  python -c "
import json; d=json.load(open('$OUT/bench.$i.json')); na=d.get('node_agent') or {}; g=((d.get('plugin') or {}).get('grpc') or {})
print('bench', $i, d['value'], d['wave_pods_per_s'], d['config'].get('node_agent'), na.get('plugin_calls_mean_ms'), g.get('handler_us'), d.get('latency_sweep_pods_per_s'), d.get('busy_pct'))"
done
