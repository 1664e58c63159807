#!/bin/bash
# N-rank rehearsal of the driver's scaling bench on the 1-GPU box: gloo ranks with fake devices (no rank
# touches the GPU), CPU-pinned control plane as in the real run; N = 1, 2, 4, 8.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02reh}
mkdir -p $OUT
for n in 1 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 --devices fake --sweep 0 \
    --json-out $OUT/n$n.json > $OUT/n$n.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/n$n.json'))
print($n, d['value'], d['wave_pods_per_s'], d['wave_ms_p50'], d['p50_bind_latency_ms'], d['node_agent'].get('max_ms'), d['cpu_s'])"
done
