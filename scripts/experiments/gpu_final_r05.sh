#!/bin/bash
# Round-5 closing GPU session on the final tree: pytest -m gpu, smoke(), the driver's N = 1 command five times,
# and a rocprofv3 kernel trace of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_final}
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
print('bench', $i, d['value'], d['wave_pods_per_s'], round(max(w[2] for w in d['wave_ms_each']), 2), na.get('plugin_calls_mean_ms'), g.get('handler_us', {}).get('allocate'), d.get('latency_sweep_pods_per_s'), d.get('busy_pct'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --sweep 0 > $OUT/prof.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; tail -20 $OUT/prof.log; exit $rc; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
timeout -k 10 300 python -m gsxtools.plugincpu --gpus 8 --idle 30 --trickle 30 --json-out $OUT/plugincpu.json > $OUT/plugincpu.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "plugincpu rc=$rc"; tail -20 $OUT/plugincpu.log; exit $rc; }
cat $OUT/plugincpu.json
