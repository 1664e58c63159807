#!/bin/bash
# Round-2 GPU session: gpu tests, smoke, then the driver's bench command REPS times (run-to-run spread).
# Stops at the first fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02}
mkdir -p $OUT
ok() { rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
  echo "gpu tests rc=$rc"; tail -3 $OUT/gpu_tests.log
  ok $rc || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
  ok $rc || exit $rc
fi
for i in $(seq 1 ${REPS:-3}); do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} --json-out $OUT/bench$i.json > $OUT/bench$i.log 2>&1; rc=$?
  echo "bench $i rc=$rc"; tail -c 400 $OUT/bench$i.log; echo
  [ $rc -eq 0 ] || exit $rc
done
exit 0
