#!/bin/bash
# Round-5 sessions 14-15: the plugin's admission path trimmed (one recv per request instead of a second one meeting
# EAGAIN, the GPU's ID prefix resolved once per GetPreferredAllocation, the Allocate journal a shared mapping
# instead of a write(2) per Allocate, no sort of already-ordered IDs) -- A/B against the previous engine build
# (abtools/_engine_old.so), N = 8 fake devices and the driver's N = 1 command, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s14}
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
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50']['total'], 'rtt', c.get('get_preferred'), c.get('allocate'), 'handler', round(h.get('get_preferred', 0), 1), round(h.get('allocate', 0), 1), 'phases', {k: round(v, 1) for k, v in ph.items()})"
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
