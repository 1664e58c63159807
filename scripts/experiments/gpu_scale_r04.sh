#!/bin/bash
# Fake-device scaling rehearsal (the ranks use no GPU: --devices fake): N = 1 / 2 / 4 / 8 ranks of the headline
# command on one box, plugin path, 20 timed waves; N = 8 three times, with the fake apiserver on 1 and on 4
# event loops.  Prints value, per-wave p50 and each process's busy % (which process the pipeline waits on).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_scale}
mkdir -p $OUT
show() {
  python -c "
import json; d=json.load(open('$1'))
print('$2', d['value'], d['wave_pods_per_s'], d.get('busy_pct'))"
}
run() {  # name n threads
  timeout -k 10 400 python bench.py --gpus $2 --apiserver-threads $3 --steps ${STEPS:-20} --warmup ${WARM:-5} --sweep 0 \
    --devices fake --json-out $OUT/$1.json > $OUT/$1.log 2>&1 || { echo "bench $1 failed"; tail -20 $OUT/$1.log; return 1; }
  show $OUT/$1.json $1
}
for n in 1 2 4; do run n$n.t1 $n 1 || exit 1; done
for i in 1 2 3; do
  run n8.t1.$i 8 1 || exit 1
  run n8.t4.$i 8 4 || exit 1
done
