#!/bin/bash
# Short confirmation of the tree on one MI355X: gpu tests, smoke, the driver's N=1 command (x2, the second with the
# sweep and plugin rows), default K/W, rocprof of the driver's command.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_confirm}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
for i in 1 2; do
  sw=0; [ $i -eq 2 ] && sw=1
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep $sw --json-out $OUT/bench$i.json > $OUT/bench$i.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/bench$i.json'))
print('bench', $i, d['value'], d['wave_pods_per_s']['p50'], d['p50_bind_latency_ms'], d['p99_bind_latency_ms'], (d.get('device_plugin_path_native_kubelet') or {}).get('pods_per_s'))"
done
timeout -k 10 600 python bench.py --gpus 1 --sweep 0 --json-out $OUT/bench_default.json > $OUT/bench_default.log 2>&1 || exit $?
python -c "
import json; d=json.load(open('$OUT/bench_default.json')); print('bench default', d['value'], d['wave_pods_per_s'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --sweep 0 > $OUT/prof.log 2>&1 || exit $?
echo "rocprof ok"
