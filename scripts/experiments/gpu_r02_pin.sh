#!/bin/bash
# Run-to-run spread of the driver's bench command under each CPU placement (bench.py --pin), 3 runs each,
# plus the shipped gRPC device-plugin path (--node-agent plugin).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02pin}
mkdir -p $OUT
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpus')" > $OUT/cpus.txt
for mode in spread none compact; do
  for i in 1 2 3; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --pin $mode --sweep 0 --json-out $OUT/$mode$i.json > $OUT/$mode$i.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/$mode$i.json'))
print('$mode', $i, d['value'], d['wave_pods_per_s'], d['p50_bind_latency_ms'])"
  done
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --node-agent plugin --json-out $OUT/plugin.json > $OUT/plugin.log 2>&1 || exit $?
python -c "
import json; d=json.load(open('$OUT/plugin.json'))
print('plugin', d['value'], d['wave_pods_per_s'], d['p50_bind_latency_ms'], d['node_agent'])"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $OUT/default.json > $OUT/default.log 2>&1 || exit $?
python -c "
import json; d=json.load(open('$OUT/default.json'))
print('default+sweep', d['value'], d['wave_pods_per_s'])
for r in d['latency_sweep']: print(r)
for r in d['reference_client']: print(r)"
