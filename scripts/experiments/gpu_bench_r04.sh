#!/bin/bash
# The driver's N=1 command, RUNS times back to back (BENCH evidence: value and its spread).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_bench}
mkdir -p $OUT
for i in $(seq 1 ${RUNS:-5}); do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 ${EXTRA:-} > $OUT/bench.$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $i rc=$rc"; tail -20 $OUT/bench.$i.log; exit $rc; }
  tail -1 $OUT/bench.$i.log > $OUT/bench.$i.json
  python -c "
import json; d=json.load(open('$OUT/bench.$i.json')); na=d.get('node_agent') or {}; g=((d.get('plugin') or {}).get('grpc') or {})
print('bench', $i, d['value'], d['wave_pods_per_s'], [w[2] for w in d['wave_ms_each']], na.get('plugin_calls_mean_ms'), g.get('handler_us', {}).get('allocate'), d.get('latency_sweep_pods_per_s'), d.get('busy_pct'))"
done
