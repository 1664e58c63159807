#!/bin/bash
# A/B of the kubelet + device-plugin path on one MI355X: the driver's N=1 command shape (20 timed waves after 5
# warmup) with the compiled node agent's in-process matcher (native) and with the shipped plugin process behind
# gRPC (native-plugin), 3 runs each, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_ab}
mkdir -p $OUT
for i in 1 2 3; do
  for na in ${AGENTS:-native native-plugin}; do
    timeout -k 10 300 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARM:-5} --sweep 0 --node-agent $na \
      ${EXTRA:-} --json-out $OUT/$na.$i.json > $OUT/$na.$i.log 2>&1 || { echo "bench $na $i failed"; tail -20 $OUT/$na.$i.log; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/$na.$i.json')); na=d['node_agent']
g=((d.get('plugin') or {}).get('grpc') or {})
print('$na', $i, d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], na.get('plugin_calls_mean_ms'), na.get('mean_ms'), g.get('handler_us'), d.get('busy_pct'))"
  done
done
