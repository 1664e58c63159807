#!/bin/bash
# GPU tests (tightened assertions, concurrency test, configs via the gRPC plugin), smoke, 3 driver benches.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02c}
mkdir -p $OUT
ok() { rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/gpu_tests.log | tail -45
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
ok $rc || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 --json-out $OUT/bench$i.json > $OUT/bench$i.log 2>&1; rc=$?
  [ $rc -eq 0 ] || exit $rc
  python -c "
import json; d=json.load(open('$OUT/bench$i.json'))
print($i, d['value'], d['wave_pods_per_s'], d['wave_ms_max'], d['node_agent'].get('max_ms'))"
done
exit 0
