#!/bin/bash
# Round-5 session 16: the wave's teardown split (teardown_ms_mean: /inspect read, DeleteCollection call, informer
# sees every pod gone, ledger empty) at N = 8 fake devices and N = 1.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s16}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json'))
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], d['teardown_ms_mean'], 'busy', d['busy_pct'])"
}
run n8_r1 --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
run n8_r2 --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
run h_r1 --gpus 1 --steps 20 --warmup 5 --sweep 0
# the driver's own command (latency sweep included: 20 waves a point now)
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $OUT/driver.json > $OUT/driver.log 2>&1 || { tail -30 $OUT/driver.log; exit 1; }
python -c "
import json; d=json.load(open('$OUT/driver.json'))
print('driver', d['value'], d['wave_pods_per_s']['p50'], [(r['bind_mode'], r['api_latency_ms'], r['pods_per_s'], r['pods_per_s_p50_wave']) for r in d['latency_sweep']])"
