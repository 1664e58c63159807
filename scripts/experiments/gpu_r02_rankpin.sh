#!/bin/bash
# N=4 / N=8 gloo rehearsal (fake devices): CPU slots of ranks > 0 -- 1 CPU (default), 2 CPUs, unpinned.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02rp}
mkdir -p $OUT
base='"extender": 2, "scheduler": 2, "node-agent": 2'
for n in 4 8; do
  r2=""; r0=""
  for r in $(seq 1 $((n - 1))); do r2="$r2, \"rank$r\": 2"; r0="$r0, \"rank$r\": 0"; done
  for rep in 1 2; do
    for v in R1 R2 R0; do
      case $v in R1) w="{$base}";; R2) w="{$base$r2}";; R0) w="{$base$r0}";; esac
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 --devices fake --sweep 0 \
        --pin-widths "$w" --json-out $OUT/n${n}_$v$rep.json > $OUT/n${n}_$v$rep.log 2>&1 || exit $?
      python -c "
import json; d=json.load(open('$OUT/n${n}_$v$rep.json'))
print($n, '$v', $rep, d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_max']['total'], d['node_agent'].get('max_ms'))"
    done
  done
done
