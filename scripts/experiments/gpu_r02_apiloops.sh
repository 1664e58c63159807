#!/bin/bash
# Fake kube-apiserver event loops x CPUs at N=8 (gloo ranks, fake devices): 1x1 (default), 2x2, 4x4; interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02al}
mkdir -p $OUT
n=${N:-8}
ranks=""
for r in $(seq 1 $((n - 1))); do ranks="$ranks, \"rank$r\": 2"; done
for rep in 1 2; do
  for v in 1 2 4; do
    w="{\"apiserver\": $v, \"extender\": 2, \"scheduler\": 2, \"node-agent\": 2$ranks}"
    GSX_FAKEAPI_THREADS=$v timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 --devices fake \
      --sweep 0 --pin-widths "$w" --json-out $OUT/t${v}_$rep.json > $OUT/t${v}_$rep.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/t${v}_$rep.json'))
print('threads', $v, 'rep', $rep, d['value'], d['wave_ms_p50'], 'api', d['extender']['api_latency_mean_ms'], d['apiserver'].get('loops'), d['apiserver']['lock'])"
  done
done
