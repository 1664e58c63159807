#!/bin/bash
# N=4 / N=8 fake-device rehearsal with per-wave p50/max and node-agent stats.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 1 2 4 8 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29800 + RANDOM % 100)) bench.py --gpus $n --steps 50 --warmup 10 --devices fake \
    --json-out gpurun_out/probe_$n.json > gpurun_out/probe_$n.log 2>&1; rc=$?
  echo "fake N=$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "
import json; d=json.load(open('gpurun_out/probe_$n.json'))
print({k: d[k] for k in ['value','ms_per_step','wave_ms','wave_ms_p50','wave_ms_max','p50_bind_rtt_ms','cpu_s','cgroup_timed']})"
done
