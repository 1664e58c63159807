#!/bin/bash
# Round-5 session 9: rank 0's GPU runtime endpoint on its own CPU (--runtime-cpu split) vs shared, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s9}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); n=d.get('node_agent') or {}; c=n.get('plugin_calls_mean_ms') or {}
print('$tag', d['value'], d['wave_pods_per_s'], d['wave_ms_p50'], 'rd', d['run_delay_pct'], 'gap', c.get('gap'))"
}
for rep in 1 2 3 4; do
  run shared_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0
  run split_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0 --runtime-cpu split
done
