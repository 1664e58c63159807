#!/bin/bash
# Round-5 session 13: how much of an admission's two round trips is the kubelet stand-in's own wake-up
# (GSX_H2_CLIENT_SPIN_US=300: its h2 client polls without sleeping for the answer) at N = 8, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s13}
mkdir -p $OUT
run() {  # tag spin, bench args...
  local tag=$1 spin=$2; shift 2
  GSX_H2_CLIENT_SPIN_US=$spin timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); n=d.get('node_agent') or {}; c=n.get('plugin_calls_mean_ms') or {}
g=((d.get('plugin') or {}).get('grpc') or {}).get('handler_us') or {}
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'calls', {k: c.get(k) for k in ('get_preferred','allocate','gap_kept','encode_preferred')}, 'handler', round(g.get('get_preferred', 0), 1), round(g.get('allocate', 0), 1), 'busy', d.get('busy_pct'))"
}
for rep in 1 2; do
  run n8_s0_r$rep 0 --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
  run n8_s300_r$rep 300 --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
done
