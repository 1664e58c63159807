#!/bin/bash
# Fake-device N = 8 on one node with the latency sweep (1 / 2 / 5 ms per apiserver request) on the plugin path.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_sweep8
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 600 python bench.py --gpus 8 --devices fake --steps 20 --warmup 5 --json-out $OUT/n8.$i.json \
    > $OUT/n8.$i.log 2>&1 || { echo "n8 $i failed"; tail -20 $OUT/n8.$i.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/n8.$i.json'))
print('n8', $i, d['value'], d['wave_pods_per_s']['p50'], d['node_agent'].get('mismatch'), d['node_agent'].get('failed'), d.get('latency_sweep_pods_per_s'))"
done
