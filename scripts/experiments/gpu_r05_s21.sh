#!/bin/bash
# Round-5 session 21: the phased GEMM on the 32x32x16 MFMA (cfg 10): numerics (pytest), then an interleaved A/B
# against cfg 5 and hipBLASLt.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s21}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gemm" > $OUT/pytest_gemm.log 2>&1
rc=$?; tail -3 $OUT/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/experiments/gemm_ab.py > $OUT/gemm_ab.json 2> $OUT/gemm_ab.err || { tail -20 $OUT/gemm_ab.err; exit 1; }
cat $OUT/gemm_ab.json
