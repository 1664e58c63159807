#!/bin/bash
# Round-5 session 18: the plugin joins the L3-local CPU group (GSX_PIN_LOCAL=6, the default now) vs round 5's group
# of five (GSX_PIN_LOCAL=5), N = 8 fake devices and the driver's N = 1 command, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s18}
mkdir -p $OUT
for c in 0 8 16 24; do echo "cpu$c L3: $(cat /sys/devices/system/cpu/cpu$c/cache/index3/shared_cpu_list)"; done
run() {  # tag local, bench args...
  local tag=$1 loc=$2; shift 2
  GSX_PIN_LOCAL=$loc timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); p=d['cpu_pinning']
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50']['total'], 'na', p.get('node-agent'), 'plugin', p.get('plugin'), 'r0', p.get('rank0'), 'api', p.get('apiserver'))"
}
for rep in 1 2 3; do
  run n8_l5_r$rep 5 --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
  run n8_l6_r$rep 6 --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
done
for rep in 1 2 3; do
  run h_l5_r$rep 5 --gpus 1 --steps 20 --warmup 5 --sweep 0
  run h_l6_r$rep 6 --gpus 1 --steps 20 --warmup 5 --sweep 0
done
