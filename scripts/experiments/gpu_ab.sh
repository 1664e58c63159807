#!/bin/bash
# A/B of the 1-GPU bench on one box: current binaries vs those in ab_old/ (engine / node agent / kernels),
# swapped in per variant.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
N=gpushare_scheduler_extender_amd/_native
mkdir -p gpurun_out/ab ab_new
cp $N/_engine*.so $N/gsx-nodeagent $N/libgsx_kernels.so ab_new/
use() {  # use <dir-for-engine> <dir-for-nodeagent> <dir-for-kernels>
  cp $1/_engine*.so $N/ && cp $2/gsx-nodeagent $N/ && cp $3/libgsx_kernels.so $N/
}
run() {
  timeout -k 10 300 python bench.py --json-out gpurun_out/ab/$1.json > gpurun_out/ab/$1.log 2>&1 || { tail -5 gpurun_out/ab/$1.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab/$1.json'))
print('$1', d['value'], d['wave_ms'], d['p50_bind_latency_ms'])"
}
for r in 1 2; do
  use ab_new ab_new ab_new && run new_$r
  use ab_old ab_old ab_old && run old_$r
  use ab_new ab_old ab_new && run oldagent_$r
  use ab_old ab_new ab_old && run oldruntime_$r
done
use ab_new ab_new ab_new
