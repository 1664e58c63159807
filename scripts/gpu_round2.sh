#!/bin/bash
# GPU session: gpu tests, smoke, bench (N=1), rocprof (inproc), isolation scenarios.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 600 python bench.py --steps 30 --warmup 3 --json-out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench1.log | cut -c1-400
ok $rc || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 2 --inproc > gpurun_out/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"
ok $rc || exit $rc
timeout -k 10 900 python -m gpushare_scheduler_extender_amd.sim.isolation --seconds 6 --json-out gpurun_out/isolation.json > gpurun_out/isolation.log 2>&1; rc=$?
echo "isolation rc=$rc"; cat gpurun_out/isolation.log | grep scenario
exit $rc
