#!/bin/bash
# GPU tests, smoke, real-GPU bench (native control plane), then N=1..8 rehearsal with fake devices
# (all-native vs all-python stand-ins) on the box's CPUs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --json-out gpurun_out/nat_gpu1.json > gpurun_out/nat_gpu1.log 2>&1; rc=$?
echo "bench gpu N=1 rc=$rc"; tail -1 gpurun_out/nat_gpu1.log
[ $rc -eq 0 ] || exit $rc
for n in 1 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29700 + n)) bench.py --gpus $n --steps 50 --warmup 10 --devices fake \
    --json-out gpurun_out/nat_fake_$n.json > gpurun_out/nat_fake_$n.log 2>&1; rc=$?
  echo "fake N=$n native rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for n in 1 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29750 + n)) bench.py --gpus $n --steps 50 --warmup 10 --devices fake --apiserver python \
    --scheduler python --node-agent python --json-out gpurun_out/py_fake_$n.json > gpurun_out/py_fake_$n.log 2>&1; rc=$?
  echo "fake N=$n python rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python - <<'PY'
import json
for f in ["nat_gpu1"] + [f"nat_fake_{n}" for n in (1, 2, 4, 8)] + [f"py_fake_{n}" for n in (1, 8)]:
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["wave_ms"], d["p50_bind_latency_ms"], d["p50_bind_rtt_ms"], d.get("cpu_s"))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --inproc > gpurun_out/prof.log 2>&1; echo "rocprof rc=$?"
