#!/bin/bash
# Load-aware CPU placement (spread: idlest physical cores sampled at start) vs topology order (static), the
# driver's N=1 command, interleaved; then one N=8 gloo rehearsal (fake devices) each.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02pl}
mkdir -p $OUT
python scripts/experiments/cpu_probe.py 1 > $OUT/probe0.json
for rep in 1 2 3; do
  for m in static spread smt; do
    extra="--pin $m"; [ $m = smt ] && extra="--pin spread --pin-smt 1"
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 $extra \
      --json-out $OUT/n1_${m}_$rep.json > $OUT/n1_${m}_$rep.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('$OUT/n1_${m}_$rep.json'))
print('n1', '$m', $rep, d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_max']['total'], d['cpu_pinning'])"
  done
done
for m in spread smt; do
  extra="--pin $m"; [ $m = smt ] && extra="--pin spread --pin-smt 1"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29508 bench.py --gpus 8 --steps 20 --warmup 5 --devices fake --sweep 0 $extra \
    --json-out $OUT/n8_$m.json > $OUT/n8_$m.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('$OUT/n8_$m.json'))
print('n8', '$m', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_max']['total'], d['cpu_pinning'])"
done
python scripts/experiments/cpu_probe.py 1 > $OUT/probe1.json
