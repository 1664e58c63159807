#!/bin/bash
# A/B of the control-plane stand-ins on the GPU box's CPUs (fake devices, N=1 and N=8) + real-GPU N=1.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "nproc=$(nproc)" > gpurun_out/ab.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --json-out gpurun_out/ab_gpu1.json >> gpurun_out/ab.log 2>&1; rc=$?
echo "gpu N=1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for n in 1 8; do
  for s in native python; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29700 + n)) bench.py --gpus $n --steps 30 --warmup 5 --devices fake --scheduler $s \
      --json-out gpurun_out/ab_${s}_$n.json >> gpurun_out/ab.log 2>&1; rc=$?
    echo "fake N=$n $s rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python - <<'PY'
import json
for f in ["ab_gpu1"] + [f"ab_{s}_{n}" for n in (1, 8) for s in ("native", "python")]:
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["wave_ms"], d["p50_bind_latency_ms"], d["p50_bind_rtt_ms"], d.get("cpu_s"))
PY
