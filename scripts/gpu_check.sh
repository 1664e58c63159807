#!/bin/bash
# One GPU-box session: gpu tests, smoke, 1-GPU bench, rocprofv3 kernel stats.
# Stops at the first fault / abort / timeout (exit >= 2 and != test-failure).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --json-out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench1.log
ok $rc || exit $rc
if [ "${GSX_PROFILE_RUN:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
fi
exit 0
