#!/bin/bash
# Plugin process CPUs: 2 (one core: its spinning serving thread shares the other SMT thread with the pod feed,
# Python and the commit worker) vs 4, driver command shape N = 1, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_pinw
mkdir -p $OUT
for i in 1 2 3; do
  for w in 2 4; do
    timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 --pin-widths "{\"plugin\": $w}" \
      --json-out $OUT/w$w.$i.json > $OUT/w$w.$i.log 2>&1 || { echo "bench $w $i failed"; tail -20 $OUT/w$w.$i.log; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/w$w.$i.json')); na=d['node_agent']; g=d['plugin']['grpc']
w=[x[2] for x in d['wave_ms_each']]
print($w, $i, d['value'], 'p50', d['wave_pods_per_s']['p50'], 'max wave', max(w), 'n>1ms', sum(x>1 for x in w), 'agent max', na['max_ms'], 'waited', g.get('waited'), g.get('wait_ms'), d['cpu_pinning'].get('plugin'), d.get('busy_threads_pct',{}).get('plugin'))"
  done
done
