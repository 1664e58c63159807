#!/bin/bash
# Round-5 session 8: the serving thread yields inside its spin (A/B by GSX_PLUGIN_SPIN_US: 1000 with yield vs 0 = block),
# headline on the plugin's one core, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s8}
mkdir -p $OUT
run() {  # tag, env, bench args...
  local tag=$1; local envs=$2; shift 2
  env $envs timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); n=d.get('node_agent') or {}; c=n.get('plugin_calls_mean_ms') or {}
print('$tag', d['value'], d['wave_pods_per_s'], 'busy', d['busy_pct'].get('plugin'), 'rd', d['run_delay_pct'].get('plugin'), d['run_delay_pct'].get('rank0'), 'alloc rtt', c.get('allocate'), 'gap', c.get('gap'))"
}
for rep in 1 2 3; do
  run y_r$rep "GSX_PLUGIN_SPIN_US=1000" --gpus 1 --steps 20 --warmup 5 --sweep 0
  run b_r$rep "GSX_PLUGIN_SPIN_US=0" --gpus 1 --steps 20 --warmup 5 --sweep 0
done
for rep in 1 2; do
  run n8y_r$rep "GSX_PLUGIN_SPIN_US=1000" --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
done
