#!/bin/bash
# Round-5 session 29: N = 1 (the driver's command) with rank 0 on one core (default) vs two CPUs vs the extender on
# four CPUs, interleaved: rank 0's threads waited for its CPU 97 % of the region in profiles/r05_final4/bench.1.json.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s29}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); p=d['cpu_pinning']
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'rd', d['run_delay_pct'], 'r0', p.get('rank0'))"
}
for rep in 1 2 3 4; do
  run a_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0
  run b_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0 --pin-widths '{"rank0": 2}'
  run c_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0 --pin-widths '{"extender": 4}'
done
