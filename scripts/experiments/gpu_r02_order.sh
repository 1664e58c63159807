#!/bin/bash
# Where the N-GPU wave spends its time: gloo ranks with fake devices (no rank touches the GPU), N = 4, 8;
# prints the extender's bind-order waits and apiserver round trips next to the wave times.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02ord}
mkdir -p $OUT
for n in ${NS:-4 8 8}; do
  i=$((${i:-0} + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 --devices fake --sweep 0 \
    --json-out $OUT/n${n}_$i.json > $OUT/n${n}_$i.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/n${n}_$i.json'))
print($n, d['value'], d['wave_ms_p50'], 'bind p50', d['p50_bind_latency_ms'], 'rtt', d['p50_bind_rtt_ms'])
print('   extender', d['extender'])
print('   timed', d['timed_region_ms'])
print('   apiserver busy', d['apiserver'].get('busy_ms'), 'lock hold', d['apiserver']['lock']['hold_ms'])"
done
