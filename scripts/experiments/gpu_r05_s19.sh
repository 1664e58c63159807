#!/bin/bash
# Round-5 session 19: GetPreferredAllocation in one walk (the size read off the request's tail, a tight picker
# instead of two callback walks) -- A/B against the engine before it (abtools/_engine_old.so), N = 8 fake devices.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s19}
mkdir -p $OUT
SO=gpushare_scheduler_extender_amd/_native/_engine.cpython-310-x86_64-linux-gnu.so
cp $SO abtools/_engine_new.so
use() { cp abtools/_engine_$1.so $SO; }
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; use new; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); n=d.get('node_agent') or {}; c=n.get('plugin_calls_mean_ms') or {}
g=(d.get('plugin') or {}).get('grpc') or {}; h=g.get('handler_us') or {}; p=d['cpu_pinning']
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50']['total'], 'rtt', c.get('get_preferred'), c.get('allocate'), 'handler', round(h.get('get_preferred', 0), 1), round(h.get('allocate', 0), 1), 'na', p.get('node-agent'), 'plugin', p.get('plugin'))"
}
for rep in 1 2 3 4; do
  use old; run n8_old_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
  use new; run n8_new_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
done
use new
