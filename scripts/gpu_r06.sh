#!/bin/bash
# Round-6 GPU session: pytest -m gpu (slice B now through the sample image's run.sh), smoke(), the driver's N = 1
# bench command three times, and a rocprofv3 kernel trace of it.  Every GPU step under its own timeout, chained so
# that the first failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06}
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
import json; d=json.load(open('$OUT/bench.$i.json'))
print('bench', $i, d['value'], d['wave_pods_per_s'], round(max(w[2] for w in d['wave_ms_each']), 2), d.get('latency_sweep_pods_per_s'), d.get('open_loop_knee_pods_per_s'), (d.get('open_loop') or {}).get('bound_stage'))"
done
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --sweep 0 --open-loop 0 > $OUT/prof.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; tail -20 $OUT/prof.log; exit $rc; }
  find $OUT/prof -name "*kernel_stats.csv" | head -3
fi
exit 0
