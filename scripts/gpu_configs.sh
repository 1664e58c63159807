#!/bin/bash
# BASELINE.json configurations 1-5 on the MI355X box (real device size, HBM arena, CU probe).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m gsxtools.configs --gpu --json-out gpurun_out/configs_gpu.json \
  > gpurun_out/configs_gpu.log 2>&1; rc=$?
cat gpurun_out/configs_gpu.log
exit $rc
