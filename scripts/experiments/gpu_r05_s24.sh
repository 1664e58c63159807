#!/bin/bash
# Round-5 session 24: the wave's teardown on the final tree (the fake apiserver's DELETED objects without a deep
# copy; teardown_ms_mean) at N = 8 fake devices and N = 1.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s24}
mkdir -p $OUT
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json'))
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'create', d.get('create_ms_mean'), d['teardown_ms_mean'])"
}
for rep in 1 2 3; do
  run n8_r$rep --gpus 8 --devices fake --steps 40 --warmup 5 --sweep 0
done
run h_r1 --gpus 1 --steps 20 --warmup 5 --sweep 0
