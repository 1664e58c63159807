#!/bin/bash
# gpu tests, scale rehearsal, rocprofv3 kernel stats (bench + GEMM), then PMC counters for the GEMM tiles
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
ok $rc || exit $rc
bash scripts/gpu_scale_rehearsal.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench -- python3 bench.py --inproc --steps 30 --warmup 3 > gpurun_out/prof_bench.log 2>&1; rc=$?
echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gemm -o gemm -- python3 scripts/gemm_once.py 8192 3,5 > gpurun_out/prof_gemm.log 2>&1; rc=$?
echo "rocprof gemm rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1; echo "list-avail rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc_gemm1 -o pmc -- python3 scripts/gemm_once.py 8192 3,5 > gpurun_out/pmc_gemm1.log 2>&1; echo "pmc1 rc=$?"
