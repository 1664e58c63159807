#!/bin/bash
# Fake-device N = 4 / 8 rehearsal keeping every child's log (node agent + plugin stderr) under
# gpurun_out/r04_scale_logs/<run>/, then the driver's N = 1 command twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_scale_logs
mkdir -p $OUT
run() {  # name n extra...
  local name=$1 n=$2; shift 2
  GSX_LOG_DIR=$OUT/$name timeout -k 10 400 python bench.py --gpus $n --steps 20 --warmup 5 --sweep 0 "$@" \
    --json-out $OUT/$name.json > $OUT/$name.log 2>&1 || { echo "bench $name failed"; tail -20 $OUT/$name.log; return 1; }
  python -c "
import json; d=json.load(open('$OUT/$name.json'))
print('$name', d['value'], d['wave_pods_per_s']['p50'], d['node_agent'].get('mismatch'), d['wave_ms_max'], d.get('busy_pct'))"
}
for i in 1 2 3; do run n4.$i 4 --devices fake || exit 1; done
for i in 1 2 3; do run n8.$i 8 --devices fake || exit 1; done
run n1.drv.1 1 || exit 1
run n1.drv.2 1 || exit 1
