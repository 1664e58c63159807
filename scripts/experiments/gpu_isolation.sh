#!/bin/bash
# CU-partition isolation benchmark (BASELINE config 5) with the current GEMM kernel.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m gsxtools.isolation --seconds 6 \
  --json-out gpurun_out/isolation.json > gpurun_out/isolation.log 2>&1; rc=$?
cat gpurun_out/isolation.log | tail -12
exit $rc
