#!/bin/bash
# GPU session: kernel micro-benchmarks, GEMM rocprof, CU-partition isolation bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_kernels.py gpurun_out/kernels.json > gpurun_out/kernels.log 2>&1; rc=$?
echo "kernels rc=$rc"; tail -3 gpurun_out/kernels.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m gsxtools.isolation --seconds 8 --json-out gpurun_out/isolation.json > gpurun_out/isolation.log 2>&1; rc=$?
echo "isolation rc=$rc"; tail -6 gpurun_out/isolation.log
exit $rc
