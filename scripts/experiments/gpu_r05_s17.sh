#!/bin/bash
# Round-5 session 17: the wave driver's BatchClient keeps its helper threads (a wave's creates started and joined up to 15 threads inside the timed wave) -- A/B against the engine before it (abtools/_engine_old.so), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s17}
mkdir -p $OUT
SO=gpushare_scheduler_extender_amd/_native/_engine.cpython-310-x86_64-linux-gnu.so
cp $SO abtools/_engine_new.so
use() { cp abtools/_engine_$1.so $SO; }
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; use new; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); n=d.get('node_agent') or {}; c=n.get('plugin_calls_mean_ms') or {}
g=(d.get('plugin') or {}).get('grpc') or {}; h=g.get('handler_us') or {}; ph=g.get('allocate_phases_us') or {}
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'create', d.get('create_ms_mean'), 'rd', d.get('run_delay_pct', {}).get('rank0'))"
}
for rep in 1 2 3 4; do
  use old; run n8_old_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
  use new; run n8_new_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
done
for rep in 1 2 3; do
  use old; run h_old_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0
  use new; run h_new_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0
done
use new
