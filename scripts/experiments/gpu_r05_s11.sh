#!/bin/bash
# Round-5 session 11: the kubelet stand-in on two cores (--pin-widths node-agent 4) vs one, N = 8 fake devices and
# the driver's N = 1 command, interleaved.  Session 10 read the node agent 100 % busy and its threads' run-delay
# 64-102 % of the region at N = 8, with 20 of the 25 us gap between admissions inside the admitting worker's loop.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s11}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); n=d.get('node_agent') or {}; c=n.get('plugin_calls_mean_ms') or {}
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'calls', {k: c.get(k) for k in ('get_preferred','allocate','gap','gap_loop')}, 'rd', d.get('run_delay_pct'), 'busy', d.get('busy_pct'))"
}
for rep in 1 2 3; do
  run n8_w2_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
  run n8_w4_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0 --pin-widths '{"node-agent": 4}'
done
for rep in 1 2; do
  run h_w2_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0
  run h_w4_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0 --pin-widths '{"node-agent": 4}'
done
