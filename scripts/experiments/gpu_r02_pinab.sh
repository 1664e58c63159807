#!/bin/bash
# A/B of CPU slot widths for the pinned control plane, interleaved on one box (bench.py --pin-widths).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02ab}
mkdir -p $OUT
A='{"extender": 2, "node-agent": 2}'
B='{"rank0": 2, "extender": 3, "scheduler": 2, "node-agent": 3}'
C='{"extender": 2, "node-agent": 2, "scheduler": 2}'
for i in 1 2 3; do
  for v in A B C; do
    w="${!v}"
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 --pin-widths "$w" --json-out $OUT/$v$i.json > $OUT/$v$i.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/$v$i.json'))
print('$v', $i, d['value'], d['wave_pods_per_s']['p50'], d['cpu_pinning'])"
  done
done
