#!/bin/bash
# Round-5 session 4: the headline after the serving-thread fix -- wave sampler on / off, the plugin on one core (2 CPUs,
# the new default) vs two (4 CPUs); the one-box 4-rank launch; N = 8 fake devices; the plugin's CPU idle / trickle.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s4}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); w=d.get('wave_attribution') or {}; n=d.get('node_agent') or {}
print('$tag', d['value'], d['wave_pods_per_s'], d['busy_pct'].get('plugin'), 'slow', [(s['wave'], s['ms'], s['blame']) for s in (w.get('slow_waves') or [])], 'mismatch', n.get('mismatch'))"
}
for rep in 1 2; do
  run h_ws1_p2_r$rep --gpus 1 --steps 20 --warmup 5
  run h_ws0_p2_r$rep --gpus 1 --steps 20 --warmup 5 --wave-sampler 0
  run h_ws1_p4_r$rep --gpus 1 --steps 20 --warmup 5 --pin-widths '{"plugin": 4}'
done
run share4 --gpus 4 --share-gpu --pod-gib 8 --steps 20 --warmup 5 --sweep 0
for rep in 1 2; do
  run n8_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
done
timeout -k 10 200 python -m gsxtools.plugincpu --gpus 8 --idle 60 --trickle 60 --json-out $OUT/plugincpu.json \
  > $OUT/plugincpu.log 2>&1 || { tail -20 $OUT/plugincpu.log; exit 1; }
tail -1 $OUT/plugincpu.log
