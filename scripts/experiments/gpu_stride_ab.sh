#!/bin/bash
# A/B of the HBM stamp stride (1 MiB = 2 stamps per 2 MiB carve unit, 2 MiB = one per unit), interleaved, the
# driver's N=1 command otherwise.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-stride}
mkdir -p $OUT
for i in 1 2 3; do
  for s in 1048576 2097152; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 --stamp-stride $s \
      --json-out $OUT/b_${s}_$i.json > $OUT/b_${s}_$i.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/b_${s}_$i.json')); na=d['node_agent']
print('$s', $i, d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], na.get('mean_ms') or na.get('max_ms'))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --sweep 0 --stamp-stride 2097152 > $OUT/prof.log 2>&1 || exit $?
echo rocprof ok
