#!/bin/bash
# The kubelet stand-in's h2 client polling without sleeping for its answer (GSX_H2_CLIENT_SPIN_US) vs blocking:
# driver command N = 1 and fake-device N = 8, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_clientspin
mkdir -p $OUT
run() {  # name spin n extra...
  local name=$1 spin=$2 n=$3; shift 3
  GSX_H2_CLIENT_SPIN_US=$spin timeout -k 10 400 python bench.py --gpus $n --steps 20 --warmup 5 "$@" \
    --json-out $OUT/$name.json > $OUT/$name.log 2>&1 || { echo "bench $name failed"; tail -20 $OUT/$name.log; return 1; }
  python -c "
import json; d=json.load(open('$OUT/$name.json'))
print('$name', d['value'], d['wave_pods_per_s']['p50'], d['node_agent'].get('mismatch'), d['node_agent'].get('plugin_calls_mean_ms'), d.get('busy_threads_pct'))"
}
for i in 1 2; do
  for spin in 0 300; do
    run n1.s$spin.$i $spin 1 --sweep 0 || exit 1
    run n8.s$spin.$i $spin 8 --devices fake --sweep 0 || exit 1
  done
done
