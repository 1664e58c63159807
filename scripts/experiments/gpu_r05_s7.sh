#!/bin/bash
# Round-5 session 7: short device IDs -- headline, N = 8 fake devices, 8 ranks on one GPU (--share-gpu, real device
# inventory: UUID-derived IDs).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s7}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); n=d.get('node_agent') or {}; c=n.get('plugin_calls_mean_ms') or {}
g=((d.get('plugin') or {}).get('grpc') or {}).get('handler_us') or {}
print('$tag', d['value'], d['wave_pods_per_s'], d['busy_pct'].get('plugin'), 'rtt', c.get('get_preferred'), c.get('allocate'), c.get('gap'), 'handler', round(g.get('get_preferred', 0), 1), round(g.get('allocate', 0), 1), 'mismatch', n.get('mismatch'))"
}
for rep in 1 2; do
  run h_r$rep --gpus 1 --steps 20 --warmup 5
  run n8_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
done
run share8 --gpus 8 --share-gpu --pod-gib 4 --steps 20 --warmup 5 --sweep 0
