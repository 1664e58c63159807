#!/bin/bash
# A/B of the fake apiserver's loop layout at N = 8 (fake devices: the control plane alone): one loop (default) vs
# a dedicated watch loop + request loops (--watch-loop), the apiserver pinned to as many CPUs as it has loops.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_wl}
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "1 0 1" "3 1 3" "2 1 2"; do
    set -- $cfg
    tag=t$1w$2r$rep
    GSX_FAKEAPI_THREADS=$1 GSX_FAKEAPI_WATCH_LOOP=$2 timeout -k 10 300 python bench.py --gpus 8 --devices fake \
      --steps 40 --warmup 5 --sweep 0 --pin-widths "{\"apiserver\": $3}" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/$tag.json')); a=d['apiserver']
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'busy', a['busy_ms'], 'hold', a['lock']['hold_ms'], 'wait', a['lock']['wait_ms'], d['cpu_pinning'].get('apiserver'))"
  done
done
