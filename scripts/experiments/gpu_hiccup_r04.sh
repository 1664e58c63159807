#!/bin/bash
# The ~1 ms waves of the driver's N = 1 command: per run, the slowest wave next to the node agent's slowest plugin
# call, the plugin's slowest handler and the longest a call waited for its pod's event.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_hiccup
mkdir -p $OUT
for i in 1 2 3 4 5 6; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 --json-out $OUT/b$i.json > $OUT/b$i.log 2>&1 \
    || { echo "bench $i failed"; tail -20 $OUT/b$i.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/b$i.json')); na=d['node_agent']; g=d['plugin']['grpc']
w=[x[2] for x in d['wave_ms_each']]
print($i, d['value'], 'max wave', max(w), 'agent max', na['max_ms'], 'handler', g.get('handler_us'), 'waited', g.get('waited'), g.get('wait_ms'), 'lock', g.get('lock_wait'))"
done
