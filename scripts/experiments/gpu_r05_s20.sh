#!/bin/bash
# Round-5 session 20: the real-GPU multi-rank path on the final tree -- 4 and 8 ranks sharing GPU 0 (--share-gpu,
# gloo only), each rank's HBM arena stamped and verified by its own runtime endpoint.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s20}
mkdir -p $OUT
run() {  # tag nproc, bench args...
  local tag=$1 np=$2; shift 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port $((29500 + np)) bench.py --gpus $np "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 \
    || { tail -30 $OUT/$tag.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$tag.json'))
print('$tag', d['value'], d['wave_pods_per_s']['p50'], d['wave_ms_p50'], 'bad', [a.get('bad_stamps') for a in d.get('agents', [])], 'hbm', [a.get('hbm_total') for a in d.get('agents', [])][:2], d['config'].get('collectives'))"
}
run share4 4 --share-gpu --pod-gib 8 --steps 20 --warmup 5 --sweep 0
run share8 8 --share-gpu --pod-gib 4 --steps 20 --warmup 5 --sweep 0
