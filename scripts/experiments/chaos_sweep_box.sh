#!/bin/bash
# The kubelet-restart chaos row (native-plugin-batch + faithful batch rows of tests/test_chaos.py) over a seed range
# on a GPU box's CPUs (the rows use no GPU): SEEDS=first-last, WORKERS parallel pytest workers.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-chaos_sweep}
mkdir -p $OUT
GSX_CHAOS_BATCH_SEEDS=${SEEDS:-2000-2399} timeout -k 10 ${LIMIT:-900} python -u -m pytest tests/test_chaos.py -q -rf \
  -p no:cacheprovider -n ${WORKERS:-12} -k "native-plugin-batch or (faithful and binding and not event and not 7-)" \
  > $OUT/pytest.log 2>&1
rc=$?
tail -15 $OUT/pytest.log
exit $rc
