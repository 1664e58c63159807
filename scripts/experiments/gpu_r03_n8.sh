#!/bin/bash
# N = 8 fake-device rehearsal on the 1-GPU box, twice, with every wave's phase times (where do slow waves go?)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_n8}
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 8 --steps 40 --warmup 5 --devices fake --sweep 0 \
    --json-out $OUT/n8_$i.json > $OUT/n8_$i.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/n8_$i.json'))
print('n8', $i, d['value'], d['wave_pods_per_s'], d['wave_ms_max'])
print([w[2] for w in d['wave_ms_each']])"
done
