#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 240 python -m pytest tests/test_gpu_kernels.py -m gpu -q -k "gemm" > gpurun_out/gemm_tests.log 2>&1; rc=$?
echo "gemm tests rc=$rc"; tail -5 gpurun_out/gemm_tests.log
ok $rc || exit $rc
timeout -k 10 300 python scripts/bench_kernels.py gpurun_out/kernels.json > gpurun_out/kernels.log 2>&1; rc=$?
echo "kernels rc=$rc"
ok $rc || exit $rc
python - <<'PY'
import json
d = json.load(open("gpurun_out/kernels.json"))
for r in d["gemm_bf16_nt"]:
    print(r["m"], r["n"], r["k"], "torch", r["torch_tflops"], {k.split("_")[0]: v for k, v in r.items() if k.endswith("tflops") and k.startswith("cfg")})
PY
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES --kernel-trace -d gpurun_out/pmc_gemm3 -o pmc -- python3 scripts/gemm_once.py 8192 5,9 > gpurun_out/pmc_gemm3.log 2>&1; echo "pmc3 rc=$?"
