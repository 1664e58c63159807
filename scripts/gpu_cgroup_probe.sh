#!/bin/bash
# Is the bench CPU-throttled on the box?  cgroup cpu.max / cpu.stat around one N=8 fake-device run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "nproc=$(nproc)"; cat /proc/self/cgroup
for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat /sys/fs/cgroup/cpuset.cpus.effective; do echo "== $f"; cat $f 2>&1; done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29811 bench.py --gpus 8 --steps 200 --warmup 10 --devices fake \
  --json-out gpurun_out/cg_8.json > gpurun_out/cg_8.log 2>&1; rc=$?
echo "fake N=8 rc=$rc"
echo "== after"; cat /sys/fs/cgroup/cpu.stat 2>&1
python -c "
import json; d=json.load(open('gpurun_out/cg_8.json'))
print({k: d[k] for k in ['value','ms_per_step','wave_ms_p50','wave_ms_max','node_agent','apiserver']})"
