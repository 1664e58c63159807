#!/bin/bash
# Round 3: bind-order chain (strict vs relaxed) at N = 8 fake devices x apiserver latency, the device-plugin path
# breakdown (shipped gRPC plugin behind the kubelet stand-in, and behind a faithful kubelet), on the GPU box's CPUs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_orders}
mkdir -p $OUT
for o in strict relaxed; do
  for ms in 0 2 5; do
    timeout -k 10 300 python bench.py --gpus 8 --steps 20 --warmup 5 --devices fake --sweep 0 --bind-order $o \
      --api-latency-ms $ms --json-out $OUT/n8_${o}_${ms}.json > $OUT/n8_${o}_${ms}.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/n8_${o}_${ms}.json'))
print('n8', '$o', $ms, d['value'], d['wave_ms_p50'], d['extender']['bind_order_waits'])"
  done
done
for k in standin faithful; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --node-agent plugin --kubelet $k --sweep 0 \
    --json-out $OUT/plugin_$k.json > $OUT/plugin_$k.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/plugin_$k.json')); na=d['node_agent']
print('plugin', '$k', d['value'], na.get('admit_p50_ms'), na.get('breakdown_ms'), na.get('plugin_breakdown_ms'), na.get('reconcile'))"
done
timeout -k 10 300 python -m gsxtools.configs --only 3 --faithful --api-latency-ms 5 \
  --json-out $OUT/config3_faithful_5ms.json > $OUT/config3_faithful.log 2>&1 || exit $?
tail -2 $OUT/config3_faithful.log
