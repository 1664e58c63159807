#!/bin/bash
# Round-5 session 23: rank 0's pod runtime endpoint on its own SMT thread (--runtime-cpu split) vs sharing rank 0's
# one CPU with the wave driver (default), re-run on the final CPU placement (session 9's A/B was inside the noise),
# with the runtime call's mean in the node agent's breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s23}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json')); n=d.get('node_agent') or {}
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'runtime', n.get('mean_ms', {}).get('runtime'), 'rd', d.get('run_delay_pct', {}).get('rank0'), d['cpu_pinning'].get('rank0'))"
}
for rep in 1 2 3 4; do
  run shared_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0
  run split_r$rep --gpus 1 --steps 20 --warmup 5 --sweep 0 --runtime-cpu split
done
