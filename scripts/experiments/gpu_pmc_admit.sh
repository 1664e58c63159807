#!/bin/bash
# PMC counters of the admission kernels at 1 MiB and 2 MiB stamp strides (scripts/experiments/pmc_admit.py).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export PYTHONPATH=$PWD
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
timeout -k 10 60 python3 scripts/experiments/pmc_admit.py 5 > $OUT/sanity.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 scripts/experiments/pmc_admit.py 20 > $OUT/kt.log 2>&1 || exit $?
echo "kernel trace ok"
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum SQ_WAVES \
  -d $OUT/p1 -o p1 -- python3 scripts/experiments/pmc_admit.py 20 > $OUT/p1.log 2>&1 || exit $?
echo "pmc ok"
