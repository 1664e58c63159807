#!/bin/bash
# Round-5 session 5: wave sampler on / off at N = 1 (the driver's command) and N = 8 (fake devices), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s5}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); w=d.get('wave_attribution') or {}; n=d.get('node_agent') or {}
c=n.get('plugin_calls_mean_ms') or {}
print('$tag', d['value'], d['wave_pods_per_s'], d['busy_pct'].get('plugin'), 'calls', c.get('get_preferred'), c.get('allocate'), c.get('gap'), 'slow', [(s['wave'], s['ms'], s['blame']) for s in (w.get('slow_waves') or [])])"
}
for rep in 1 2 3; do
  run h_ws1_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0
  run h_ws0_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0 --wave-sampler 0
done
for rep in 1 2; do
  run n8_ws1_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
  run n8_ws0_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0 --wave-sampler 0
done
