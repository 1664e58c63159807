#!/bin/bash
# Round-5 session 26: at N = 8 the kubelet stand-in is now the busy one (133-136 % of its one core, its threads'
# run-delay 169-188 % of the region, session 25): two cores for it (--pin-widths node-agent 4) vs one, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s26}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); c=d['node_agent']['plugin_calls_mean_ms']; p=d['cpu_pinning']
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'rtt', c['get_preferred'], c['allocate'], 'rd', d['run_delay_pct'].get('node-agent'), 'busy', d['busy_pct'].get('node-agent'), 'na', p.get('node-agent'), 'pl', p.get('plugin'), 'r0', p.get('rank0'))"
}
for rep in 1 2 3; do
  run n8_w2_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
  run n8_w4_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0 --pin-widths '{"node-agent": 4}'
done
