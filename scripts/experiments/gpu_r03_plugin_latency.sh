#!/bin/bash
# The shipped plugin process behind the compiled kubelet stand-in at 0 / 1 / 2 / 5 ms apiserver latency (N = 1):
# kubelet admits serially, and each Allocate waits for the plugin's ASSIGNED patch to the apiserver.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_plat}
mkdir -p $OUT
for ms in 0 1 2 5; do
  for na in native-plugin native; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 60 --warmup 5 --sweep 0 --node-agent $na --api-latency-ms $ms \
      --json-out $OUT/${na}_$ms.json > $OUT/${na}_$ms.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/${na}_$ms.json')); na=d['node_agent']
print('$na', $ms, d['value'], d['wave_pods_per_s']['p50'], na.get('plugin_calls_mean_ms'), na['mean_ms'])"
  done
done
