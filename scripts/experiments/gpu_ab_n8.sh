#!/bin/bash
# Interleaved A/B at N = 8 (fake devices) with the wave timeline: CONFIGS is a ';'-separated list of
# name|ENV=... ENV=...|extra bench args
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_ab8}
mkdir -p $OUT
IFS=';' read -ra CFGS <<< "$CONFIGS"
for rep in $(seq 1 ${REPS:-2}); do
  for c in "${CFGS[@]}"; do
    IFS='|' read -r name envs args <<< "$c"
    tag=${name}_r$rep
    env $envs timeout -k 10 300 python bench.py --gpus ${N:-8} --devices ${DEVICES:-fake} --steps ${STEPS:-40} --warmup 5 --sweep 0 \
      $args --dump-timings $OUT/tim_$tag.json --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/$tag.json')); a=d['apiserver']
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'api busy', a['busy_ms'], d['cpu_pinning'].get('rank0'))"
    python scripts/experiments/wave_timeline.py $OUT/tim_$tag.json
  done
done
