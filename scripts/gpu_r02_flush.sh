#!/bin/bash
# Fake apiserver watch flush policy A/B: per loop iteration (default) vs per request; N=1 (GPU) and N=8 (gloo,
# fake devices), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02fl}
mkdir -p $OUT
for rep in 1 2; do
  for m in iteration request; do
    GSX_FAKEAPI_WATCH_FLUSH=$m timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 \
      --json-out $OUT/n1_${m}_$rep.json > $OUT/n1_${m}_$rep.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/n1_${m}_$rep.json'))
print('n1', '$m', $rep, d['value'], d['wave_ms_p50'], d['wave_pods_per_s']['p50'])"
    GSX_FAKEAPI_WATCH_FLUSH=$m timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port 29508 bench.py --gpus 8 --steps 20 --warmup 5 --devices fake \
      --sweep 0 --json-out $OUT/n8_${m}_$rep.json > $OUT/n8_${m}_$rep.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/n8_${m}_$rep.json'))
print('n8', '$m', $rep, d['value'], d['wave_ms_p50'], d['wave_pods_per_s']['p50'], 'busy', d['apiserver'].get('busy_ms'))"
  done
done
