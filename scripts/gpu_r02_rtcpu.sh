#!/bin/bash
# GPU 0's runtime endpoint on its own SMT thread (split, default) vs sharing rank 0's thread (shared), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02rt}
mkdir -p $OUT
for i in 1 2 3; do
  for m in shared split; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 --runtime-cpu $m \
      --json-out $OUT/${m}_$i.json > $OUT/${m}_$i.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/${m}_$i.json'))
print('$m', $i, d['value'], d['wave_ms_p50'], d['node_agent']['mean_ms'], d['cpu_pinning']['rank0'])"
  done
done
