#!/bin/bash
# Round-2 GPU session: gpu tests, smoke, cluster-scale harness, the driver's bench command x3, rocprof stats.
# Every GPU step has its own time limit; the script stops at the first fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02s}
mkdir -p $OUT
ok() { rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $OUT/gpu_tests.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
ok $rc || exit $rc
timeout -k 10 600 python -m gsxtools.scale --json-out $OUT/scale.json > $OUT/scale.log 2>&1; rc=$?
echo "scale rc=$rc"; cut -c1-300 $OUT/scale.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $OUT/bench$i.json > $OUT/bench$i.log 2>&1; rc=$?
  echo "bench $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "
import json; d=json.load(open('$OUT/bench$i.json'))
print($i, d['value'], d['wave_pods_per_s'], d['p50_bind_latency_ms'], d['p99_bind_latency_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --sweep 0 > $OUT/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -2 $OUT/prof.log
exit 0
