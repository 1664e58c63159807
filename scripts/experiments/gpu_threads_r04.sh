#!/bin/bash
# Per-thread busy % of the node agent and the plugin (bench.py busy_threads_pct): fake-device N = 8 twice, then the
# driver's N = 1 command twice.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_threads
mkdir -p $OUT
run() {  # name n extra...
  local name=$1 n=$2; shift 2
  timeout -k 10 400 python bench.py --gpus $n --steps 20 --warmup 5 "$@" --json-out $OUT/$name.json > $OUT/$name.log 2>&1 \
    || { echo "bench $name failed"; tail -20 $OUT/$name.log; return 1; }
  python -c "
import json; d=json.load(open('$OUT/$name.json'))
print('$name', d['value'], d['wave_pods_per_s']['p50'], d['node_agent'].get('mismatch'), d.get('busy_pct'), d.get('busy_threads_pct'), d['node_agent'].get('plugin_calls_mean_ms'))"
}
run n8.1 8 --devices fake --sweep 0 || exit 1
run n8.2 8 --devices fake --sweep 0 || exit 1
run n1.1 1 || exit 1
run n1.2 1 || exit 1
