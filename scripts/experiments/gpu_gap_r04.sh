#!/bin/bash
# Where an admission's time goes at N = 8 (fake devices): the node agent's encode of GetPreferredAllocation, the two
# round trips, and the gap between one admission's end and the next one's calls.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_gap
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 400 python bench.py --gpus 8 --devices fake --steps 20 --warmup 5 --sweep 0 --json-out $OUT/n8.$i.json \
    > $OUT/n8.$i.log 2>&1 || { echo "bench $i failed"; tail -20 $OUT/n8.$i.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/n8.$i.json')); g=d['plugin']['grpc']
print($i, d['value'], d['wave_pods_per_s']['p50'], d['node_agent']['plugin_calls_mean_ms'], g.get('handler_us'), g.get('wait_ms'), g.get('lock_wait'), d.get('busy_threads_pct'))"
done
