#!/bin/bash
# Round-3 closing pass on one MI355X: gpu tests, smoke, the driver's N=1 command (x2, the second with the sweep and
# the plugin rows), default K/W, rocprof of the driver's command, a 100k-pod soak through the headline path and a
# 20k-pod soak through the shipped plugin process, and the N = 2/4/8 rehearsal (fake devices).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
for i in 1 2; do
  sw=0; [ $i -eq 2 ] && sw=1
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep $sw --json-out $OUT/bench$i.json > $OUT/bench$i.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/bench$i.json'))
print('bench', $i, d['value'], d['wave_pods_per_s']['p50'], d['p50_bind_latency_ms'], d['p99_bind_latency_ms'], (d.get('device_plugin_path_native_kubelet') or {}).get('pods_per_s'))"
done
timeout -k 10 600 python bench.py --gpus 1 --sweep 0 --json-out $OUT/bench_default.json > $OUT/bench_default.log 2>&1 || exit $?
python -c "
import json; d=json.load(open('$OUT/bench_default.json')); print('bench default', d['value'], d['wave_pods_per_s'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --sweep 0 > $OUT/prof.log 2>&1 || exit $?
echo "rocprof ok"
timeout -k 10 900 python -u bench.py --gpus 1 --steps 25000 --warmup 5 --sweep 0 --json-out $OUT/soak.json > $OUT/soak.log 2>&1 || exit $?
python -c "
import json; d=json.load(open('$OUT/soak.json'))
print('soak', d['steps'], d['value'], d['wave_pods_per_s'], d['rss_mib'], {k: d['node_agent'].get(k) for k in ('admitted','failed','bad_stamps')})"
GSX_PLUGIN_STATS_DIR=$PWD/$OUT timeout -k 10 900 python -u bench.py --gpus 1 --steps 5000 --warmup 10 --sweep 0 --node-agent native-plugin \
  --json-out $OUT/soak_plugin.json > $OUT/soak_plugin.log 2>&1 || exit $?
python -c "
import json; d=json.load(open('$OUT/soak_plugin.json'))
print('soak plugin', d['steps'], d['value'], d['wave_pods_per_s'], {k: d['node_agent'].get(k) for k in ('admitted','failed','bad_stamps','plugin_calls_mean_ms')})"
for n in 2 4 8; do
  timeout -k 10 600 python bench.py --gpus $n --steps 40 --warmup 5 --devices fake --sweep 0 --json-out $OUT/fake_n$n.json \
    > $OUT/fake_n$n.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/fake_n$n.json')); print('fake n$n', d['value'], d['wave_pods_per_s']['p50'])"
done
