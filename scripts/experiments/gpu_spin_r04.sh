#!/bin/bash
# The shipped plugin path (driver command shape, N=1): serving-thread spin 200 us (default) vs 1000 us, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_spin}
mkdir -p $OUT
for i in 1 2 3; do
  for spin in 200 1000; do
    GSX_PLUGIN_SPIN_US=$spin timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 \
      --json-out $OUT/s$spin.$i.json > $OUT/s$spin.$i.log 2>&1 || { echo "bench $spin $i failed"; tail -20 $OUT/s$spin.$i.log; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/s$spin.$i.json')); na=d['node_agent']; g=((d.get('plugin') or {}).get('grpc') or {})
print($spin, $i, d['value'], d['wave_pods_per_s']['p50'], na.get('plugin_calls_mean_ms'), g.get('handler_us'), g.get('lock_wait'), g.get('allocate_phases_us'), d.get('busy_pct'))"
  done
done
