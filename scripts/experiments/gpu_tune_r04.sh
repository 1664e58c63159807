#!/bin/bash
# Plugin-path tuning on one MI355X: the driver's N=1 command shape with one knob changed per variant, 2 runs each.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_tune}
mkdir -p $OUT
W4='{"plugin":4}'
run() {  # name i env... -- bench args...
  local name=$1 i=$2; shift 2
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARM:-5} --sweep 0 \
    "$@" --json-out $OUT/$name.$i.json > $OUT/$name.$i.log 2>&1 || { echo "bench $name $i failed"; tail -20 $OUT/$name.$i.log; return 1; }
  python -c "
import json; d=json.load(open('$OUT/$name.$i.json')); na=d['node_agent']; g=(d.get('plugin') or {}).get('grpc') or {}
print('$name', $i, d['value'], d['wave_pods_per_s']['p50'], na.get('plugin_calls_mean_ms'), na.get('mean_ms'), {k: g.get(k) for k in ('slow_preferred','waited','feed_events','passes')})"
}
for i in 1 2; do
  run base $i X=1 -- || exit 1
  run plugin4 $i X=1 -- --pin-widths "$W4" || exit 1
  run spin1000 $i GSX_PLUGIN_SPIN_US=1000 -- || exit 1
  run native $i X=1 -- --node-agent native || exit 1
done
