#!/bin/bash
# Interleaved A/B of the one-launch admission (default) vs two launches (GSX_ADMIT_ONE_LAUNCH=0), driver's N=1 command.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-onelaunch}
mkdir -p $OUT
for i in 1 2 3; do
  for v in 0 1; do
    GSX_ADMIT_ONE_LAUNCH=$v timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 \
      --json-out $OUT/b_${v}_$i.json > $OUT/b_${v}_$i.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/b_${v}_$i.json')); print('one_launch=$v', $i, d['value'], d['wave_pods_per_s']['p50'], d['node_agent']['mean_ms']['runtime'], d['agents'][0]['bad_stamps'])"
  done
done
