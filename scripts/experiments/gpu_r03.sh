#!/bin/bash
# Round-3 GPU pass: gpu tests, smoke, the driver's N=1 bench command x2 + one with the latency sweep and the
# device-plugin path, rocprof of the driver's command, and the fake-device N = 2 / 4 / 8 rehearsal with apiserver
# latency (bench.py launches torchrun itself).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
STAGE=${STAGE:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
  echo "gpu tests rc=$rc"; tail -1 $OUT/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
  tail -1 $OUT/smoke.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  for i in 1 2 3; do
    sw=0; [ $i -eq 3 ] && sw=1
    timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep $sw --json-out $OUT/bench$i.json > $OUT/bench$i.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/bench$i.json'))
print('bench', $i, d['value'], d['wave_pods_per_s']['p50'], d['p50_bind_latency_ms'], d['p99_bind_latency_ms'], d['timed_region_ms']['max_over_ranks'], (d.get('device_plugin_path') or {}).get('pods_per_s'))"
  done
  timeout -k 10 600 python bench.py --gpus 1 --steps 300 --warmup 30 --sweep 0 --json-out $OUT/bench_default.json > $OUT/bench_default.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/bench_default.json'))
print('bench default', d['value'], d['wave_pods_per_s'], d['p50_bind_latency_ms'])"
fi
if [ "$STAGE" = all ] || [ "$STAGE" = prof ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --sweep 0 > $OUT/prof.log 2>&1 || exit $?
  echo "rocprof ok"
fi
if [ "$STAGE" = all ] || [ "$STAGE" = scale ]; then
  for n in 2 4 8; do
    timeout -k 10 600 python bench.py --gpus $n --steps 20 --warmup 5 --devices fake --sweep 1 --sweep-steps 4 \
      --sweep-orders ${SWEEP_ORDERS:-auto} --json-out $OUT/fake_n$n.json > $OUT/fake_n$n.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/fake_n$n.json'))
print('fake n$n', d['value'], d['wave_pods_per_s']['p50'], d['timed_region_ms']['max_over_ranks'])
for r in d['latency_sweep'] or []:
    print('   ', r.get('bind_mode'), r.get('bind_order'), r.get('api_latency_ms'), r.get('pods_per_s'), r.get('bind_order_waits'), r.get('bind_order_wait_ms_per_wave'))"
  done
fi
