#!/bin/bash
# phased GEMM first (short limit), then the full gpu suite, kernel bench and the scale rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 180 python -m pytest tests/test_gpu_kernels.py -m gpu -q -k "phased or cfg" > gpurun_out/gemm_tests.log 2>&1; rc=$?
echo "gemm tests rc=$rc"; tail -5 gpurun_out/gemm_tests.log
ok $rc || exit $rc
timeout -k 10 300 python scripts/bench_kernels.py gpurun_out/kernels.json > gpurun_out/kernels.log 2>&1; rc=$?
echo "kernels rc=$rc"; tail -c 3000 gpurun_out/kernels.log
ok $rc || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
ok $rc || exit $rc
bash scripts/gpu_scale_rehearsal.sh
