#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "gemm" > gpurun_out/gemm_tests.log 2>&1; rc=$?
echo "gemm tests rc=$rc"; tail -5 gpurun_out/gemm_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/bench_kernels.py gpurun_out/kernels.json > gpurun_out/kernels.log 2>&1; rc=$?
echo "kernels rc=$rc"; tail -2 gpurun_out/kernels.log
exit $rc
