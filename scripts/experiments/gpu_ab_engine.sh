#!/bin/bash
# Balanced A/B of the extender engine alone (_engine .so): current build vs ab_old/, in ABBA order
# so run-position drift on the box cancels.  Node agent and kernels are the current build in every run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
N=gpushare_scheduler_extender_amd/_native
mkdir -p gpurun_out/abe ab_new
cp $N/_engine*.so ab_new/
i=0
for v in new old old new new old old new new old old new; do
  i=$((i + 1))
  cp ab_$v/_engine*.so $N/
  timeout -k 10 300 python bench.py --json-out gpurun_out/abe/${i}_$v.json > gpurun_out/abe/${i}_$v.log 2>&1 || { tail -5 gpurun_out/abe/${i}_$v.log; cp ab_new/_engine*.so $N/; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/abe/${i}_$v.json'))
print('$i $v', d['value'], d['wave_ms']['total'], d['p50_bind_latency_ms'])"
done
cp ab_new/_engine*.so $N/
