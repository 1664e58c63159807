#!/bin/bash
# Round-5 session 10: where the kubelet stand-in's gap between admissions goes at N = 8 (gap_loop / gap_list /
# gap_handoff / relock in node_agent.plugin_calls_mean_ms).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s10}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); n=d.get('node_agent') or {}; c=n.get('plugin_calls_mean_ms') or {}
g=((d.get('plugin') or {}).get('grpc') or {}).get('handler_us') or {}
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'calls', c, 'handler', round(g.get('get_preferred', 0), 1), round(g.get('allocate', 0), 1), 'rd', d.get('run_delay_pct'), 'busy', d.get('busy_threads_pct'))"
}
for rep in 1 2; do
  run n8_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
done
run h_r1 --gpus 1 --steps 20 --warmup 5 --sweep 0
