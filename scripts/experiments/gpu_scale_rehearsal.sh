#!/bin/bash
# Rehearse the driver's N=1,2,4,8 scaling run on the GPU box's CPUs with fake devices
# (ranks never touch the GPU), plus one real 1-GPU run for reference.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "nproc=$(nproc)" > gpurun_out/scale.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --json-out gpurun_out/scale_gpu1.json >> gpurun_out/scale.log 2>&1; rc=$?
echo "gpu N=1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for n in 1 2 4 8; do
  for mode in rank node; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29600 + n)) bench.py --gpus $n --steps 30 --warmup 3 --devices fake --agent $mode \
      --json-out gpurun_out/scale_fake_${mode}_$n.json >> gpurun_out/scale.log 2>&1; rc=$?
    echo "fake N=$n $mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python - <<'PY'
import json
for f in ["scale_gpu1"] + [f"scale_fake_{m}_{n}" for n in (1, 2, 4, 8) for m in ("rank", "node")]:
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["wave_ms"], d["p50_bind_latency_ms"], d.get("cpu_s"))
PY
