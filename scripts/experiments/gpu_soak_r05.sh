#!/bin/bash
# Round 5 plugin-path soak (the mapped Allocate journal grows and rotates throughout): the driver's N = 1 command shape for 25,000 timed waves (100,000 pods), then
# fake-device N = 8 for 4,000 waves (128,000 pods).  Failed admissions, swaps and each process's RSS at the start
# and end of the timed region are in the BENCH lines.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_soak}
mkdir -p $OUT
timeout -k 10 900 python bench.py --gpus 1 --steps 25000 --warmup 10 --sweep 0 --json-out $OUT/n1.json > $OUT/n1.log 2>&1 \
  || { echo "n1 soak failed"; tail -20 $OUT/n1.log; exit 1; }
python -c "
import json; d=json.load(open('$OUT/n1.json')); na=d['node_agent']; g=d['plugin']['grpc']
print('n1', d['value'], d['wave_pods_per_s'], na.get('admitted'), na.get('failed'), na.get('mismatch'), d.get('rss_mib'), g.get('fast_allocate'), g.get('slow_allocate'))"
timeout -k 10 900 python bench.py --gpus 8 --devices fake --steps 4000 --warmup 10 --sweep 0 --json-out $OUT/n8.json > $OUT/n8.log 2>&1 \
  || { echo "n8 soak failed"; tail -20 $OUT/n8.log; exit 1; }
python -c "
import json; d=json.load(open('$OUT/n8.json')); na=d['node_agent']; g=d['plugin']['grpc']
print('n8', d['value'], d['wave_pods_per_s'], na.get('admitted'), na.get('failed'), na.get('mismatch'), d.get('rss_mib'), g.get('fast_allocate'), g.get('slow_allocate'))"
