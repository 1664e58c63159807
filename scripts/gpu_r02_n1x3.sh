#!/bin/bash
# The driver's N=1 command three times back to back (plus the sweep on the last run).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02n1}
mkdir -p $OUT
for i in 1 2 3; do
  sw=0; [ $i -eq 3 ] && sw=1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep $sw --json-out $OUT/b$i.json > $OUT/b$i.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/b$i.json'))
print($i, d['value'], d['wave_pods_per_s']['p50'], d['timed_region_ms'], d['p50_bind_latency_ms'], d['cpu_pinning'])"
done
