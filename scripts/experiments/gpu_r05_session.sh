#!/bin/bash
# Round-5 GPU session: the GPU tests, the driver's headline command, the 4-rank one-box launch (--share-gpu) and an
# interleaved N = 8 fake-device A/B of GetPreferredAllocation (auto vs off).  Every GPU step has its own time limit;
# the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s2}
mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
  tail -2 $OUT/gputests.log
fi
for i in $(seq 1 ${HEADLINE:-2}); do
  for ws in ${SAMPLER:-1}; do
    timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --wave-sampler $ws --json-out $OUT/bench_${i}_ws$ws.json \
      > $OUT/bench_${i}_ws$ws.log 2>&1 || { tail -30 $OUT/bench_${i}_ws$ws.log; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/bench_${i}_ws$ws.json')); w=d.get('wave_attribution') or {}
print('headline ws=$ws', d['value'], d['wave_pods_per_s'], d['busy_pct'], 'slow', w.get('slow_waves'))"
  done
done
if [ "${SHARE:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --gpus 4 --share-gpu --pod-gib 8 --steps 20 --warmup 5 --sweep 0 \
    --json-out $OUT/share4.json > $OUT/share4.log 2>&1 || { tail -30 $OUT/share4.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/share4.json')); print('share4', d['value'], d['per_device_used_gib'], [(a['physical_gpu'], a['admitted'], a['bad_stamps'], a['hbm_total']) for a in d['agents']])"
fi
for rep in $(seq 1 ${REPS:-2}); do
  for pref in auto 0; do
    tag=n8_pref${pref}_r$rep
    GSX_PLUGIN_PREFERRED=$pref timeout -k 10 300 python bench.py --gpus 8 --devices fake --steps 40 --warmup 5 \
      --sweep 0 --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -30 $OUT/$tag.log; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/$tag.json')); n=d['node_agent'] or {}
print('$tag', d['value'], d['wave_pods_per_s'], 'mismatch', n.get('mismatch'), 'failed', n.get('failed'), d['busy_pct'])"
  done
done
