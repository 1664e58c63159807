#!/bin/bash
# Does an idle GPU slow the first bench? The driver's N=1 command with and without a GPU clock warm-up, each run
# after 20 s of idle GPU (as after pytest / smoke), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02wm}
mkdir -p $OUT
for i in 1 2 3; do
  for w in 0 300; do
    sleep 20
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 --gpu-warm-ms $w \
      --json-out $OUT/w${w}_$i.json > $OUT/w${w}_$i.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/w${w}_$i.json'))
print('warm', $w, $i, d['value'], d['wave_ms_p50'], 'admit p50', d['node_agent']['admit_p50_ms'])"
  done
done
