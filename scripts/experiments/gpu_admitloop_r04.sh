#!/bin/bash
# The kubelet stand-in's admission pipeline: the admission slot handed from worker to worker after each Allocate
# (abtools/gsx-nodeagent_slot_handoff, the previous build) vs one worker admitting back to back while the others
# start the admitted pods (current build).  Driver command shape N = 1 and fake-device N = 8, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_admitloop}
mkdir -p $OUT
run() {  # name bin n extra...
  local name=$1 bin=$2 n=$3; shift 3
  GSX_NODEAGENT_BIN=$bin timeout -k 10 400 python bench.py --gpus $n --steps 20 --warmup 5 --sweep 0 "$@" \
    --json-out $OUT/$name.json > $OUT/$name.log 2>&1 || { echo "bench $name failed"; tail -20 $OUT/$name.log; return 1; }
  python -c "
import json; d=json.load(open('$OUT/$name.json')); w=[x[2] for x in d['wave_ms_each']]
print('$name', d['value'], d['wave_pods_per_s']['p50'], 'max wave', max(w), d['node_agent'].get('mismatch'), d['node_agent'].get('plugin_calls_mean_ms'), d.get('busy_threads_pct',{}).get('node-agent'))"
}
NEW=gpushare_scheduler_extender_amd/_native/gsx-nodeagent
OLD=${OLD:-abtools/gsx-nodeagent_slot_handoff}
for i in 1 2 3; do
  run n1.old.$i $OLD 1 || exit 1
  run n1.new.$i $NEW 1 || exit 1
  run n8.old.$i $OLD 8 --devices fake || exit 1
  run n8.new.$i $NEW 8 --devices fake || exit 1
done
