#!/bin/bash
# GPU tests + smoke, then the driver's N=1 command on the GPU, then the N-rank rehearsal (gloo ranks, fake devices)
# for N = 1, 2, 4, 8 with the default CPU placement.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02sw}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $OUT/gpu_n1_$i.json > $OUT/gpu_n1_$i.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/gpu_n1_$i.json'))
print('gpu n1', d['value'], d['wave_pods_per_s']['p50'], d['cpu_pinning'])"
done
for n in 1 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 --devices fake --sweep 0 \
    --json-out $OUT/n$n.json > $OUT/n$n.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/n$n.json'))
print('fake n$n', d['value'], d['wave_pods_per_s']['p50'], d['timed_region_ms'])"
done
