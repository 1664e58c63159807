#!/bin/bash
# The default 1-GPU bench REPS times in a row on one box (run-to-run variance).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rep
for i in $(seq 1 ${REPS:-3}); do
  timeout -k 10 300 python bench.py --json-out gpurun_out/rep/b$i.json > gpurun_out/rep/b$i.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/rep/b$i.json'))
print($i, d['value'], d['ms_per_step'], d['wave_ms'], d['p50_bind_latency_ms'], d['node_agent']['max_ms'])"
done
