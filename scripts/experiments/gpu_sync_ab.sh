#!/bin/bash
# A/B of the admission completion wait: event spin (default) vs hipStreamSynchronize (GSX_SYNC_SPIN=0).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export PYTHONPATH=$PWD
OUT=gpurun_out/${TAG:-syncab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
tail -1 $OUT/gpu_tests.log
for v in 0 1; do
  GSX_SYNC_SPIN=$v timeout -k 10 120 python scripts/experiments/admit_probe.py > $OUT/probe_$v.json 2> $OUT/probe_$v.err || exit $?
  echo "probe spin=$v"; head -c 600 $OUT/probe_$v.json; echo
done
for i in 1 2; do
  for v in 0 1; do
    GSX_SYNC_SPIN=$v timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 --json-out $OUT/b_${v}_$i.json \
      > $OUT/b_${v}_$i.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/b_${v}_$i.json')); print('spin=$v', $i, d['value'], d['wave_pods_per_s']['p50'], d['node_agent']['mean_ms']['runtime'])"
  done
done
