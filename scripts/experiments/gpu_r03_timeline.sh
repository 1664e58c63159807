#!/bin/bash
# N = 8 wave critical path (fake devices): scheduler timeline per wave (scripts/experiments/wave_timeline.py)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_tl}
mkdir -p $OUT
for n in 1 8; do
  timeout -k 10 300 python bench.py --gpus $n --devices fake --steps 40 --warmup 5 --sweep 0 \
    --dump-timings $OUT/tim_n$n.json --json-out $OUT/n$n.json > $OUT/n$n.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/n$n.json')); print('n$n', d['value'], d['wave_ms_p50'], d['node_agent']['mean_ms'], d['extender'])"
  python scripts/experiments/wave_timeline.py $OUT/tim_n$n.json
done
