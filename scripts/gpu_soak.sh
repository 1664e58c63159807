#!/bin/bash
# Soak on one MI355X: gpu tests, smoke, the driver's N=1 bench, then 100k pods (25,000 waves of 4 x 64 GiB) through
# the whole stack with resident memory of every control-plane process sampled at the start and end of the timed region.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-soak}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sweep 0 --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || exit $?
python -c "
import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['wave_pods_per_s']['p50'], d['p50_bind_latency_ms'])"
timeout -k 10 900 python -u bench.py --gpus 1 --steps ${SOAK_STEPS:-25000} --warmup 5 --sweep 0 --json-out $OUT/soak.json \
  > $OUT/soak.log 2>&1 || exit $?
python -c "
import json; d=json.load(open('$OUT/soak.json'))
print('soak', d['steps'], d['value'], d['wave_pods_per_s'], d['p50_bind_latency_ms'], d['p99_bind_latency_ms'])
print('rss', d['rss_mib']); print('agents', d['agents']); print('node_agent', {k: d['node_agent'].get(k) for k in ('admitted','failed','bad_stamps','conflicts')})
print('extender', d['extender'])"
