#!/bin/bash
# Round-5 session 12: is the N = 8 gap between admissions spent by the worker that kept the admission slot
# (gap_kept / n_gap_kept), or by a worker that had to take the slot after the queue ran dry?
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s12}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); n=d.get('node_agent') or {}; c=n.get('plugin_calls_mean_ms') or {}
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'calls', c)"
}
run n8_r1 --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
run n8_r2 --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0 --pin-widths '{"node-agent": 4}'
