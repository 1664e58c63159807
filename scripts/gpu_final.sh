#!/bin/bash
# Final round-2 confirmation: gpu tests, smoke, the driver's N=1 command x3 (sweep on the third), rocprof of the
# bench, N-rank rehearsal (gloo, fake devices) N = 2, 4, 8.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02f2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
for i in 1 2 3; do
  sw=0; [ $i -eq 3 ] && sw=1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep $sw --json-out $OUT/bench$i.json > $OUT/bench$i.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/bench$i.json'))
print('bench', $i, d['value'], d['wave_pods_per_s']['p50'], d['p50_bind_latency_ms'], d['p99_bind_latency_ms'], d['timed_region_ms']['max_over_ranks'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --sweep 0 > $OUT/prof.log 2>&1 || exit $?
echo "rocprof ok"
for n in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 --devices fake --sweep 0 \
    --json-out $OUT/fake_n$n.json > $OUT/fake_n$n.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/fake_n$n.json'))
print('fake n$n', d['value'], d['wave_pods_per_s']['p50'], d['timed_region_ms']['max_over_ranks'])"
done
