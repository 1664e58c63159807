#!/bin/bash
# Round-5 session 27: the default plan after session 26 -- N = 8 three times, N = 4 and N = 2 once (fake devices,
# the driver's torchrun shape is rehearsed by --devices fake in one process), N = 1 twice (the driver's command).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s27}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); p=d['cpu_pinning']
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50']['total'], 'max', d['wave_ms_max']['total'], 'na', p.get('node-agent'), 'pl', p.get('plugin'))"
}
for rep in 1 2 3; do
  run n8_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
done
run n4 --gpus 4 --devices fake --steps 40 --warmup 5 --sweep 0
run n2 --gpus 2 --devices fake --steps 40 --warmup 5 --sweep 0
run h_r1 --gpus 1 --steps 20 --warmup 5 --sweep 0
run h_r2 --gpus 1 --steps 20 --warmup 5 --sweep 0
