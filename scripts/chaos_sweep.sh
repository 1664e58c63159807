#!/bin/bash
# Chaos rows of tests/test_chaos.py over seed ranges on a GPU box's CPUs (the rows use no GPU):
#   GRACE=first-last   graceful deletes on a full node (both kubelet stand-ins), GSX_CHAOS_GRACE_SEEDS
#   BATCH=first-last   kubelet-restart batches + deletes (native-plugin-batch and faithful rows), GSX_CHAOS_BATCH_SEEDS
#   WORKERS=n          parallel pytest workers (default 12; the box's share is 16 CPUs)
# Progress goes to gpurun_out/$TAG/*.log (pytest -q dots), the verdict line to stdout.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-chaos_sweep}
mkdir -p $OUT
rc=0
if [ -n "${GRACE:-}" ]; then
  GSX_CHAOS_GRACE_SEEDS=$GRACE timeout -k 10 ${LIMIT:-1000} python -u -m pytest tests/test_chaos.py -q -rf \
    -p no:cacheprovider -n ${WORKERS:-12} -k "graceful_deletes" > $OUT/grace.log 2>&1
  rc=$?; echo "grace $GRACE rc=$rc: $(tail -1 $OUT/grace.log)"
  [ $rc -le 1 ] || exit $rc
fi
if [ -n "${BATCH:-}" ]; then
  GSX_CHAOS_BATCH_SEEDS=$BATCH timeout -k 10 ${LIMIT:-1000} python -u -m pytest tests/test_chaos.py -q -rf \
    -p no:cacheprovider -n ${WORKERS:-12} -k "native-plugin-batch or (faithful and binding and not event and not 7-)" \
    > $OUT/batch.log 2>&1
  rc2=$?; echo "batch $BATCH rc=$rc2: $(tail -1 $OUT/batch.log)"
  [ $rc2 -le 1 ] || exit $rc2
  [ $rc -ne 0 ] || rc=$rc2
fi
exit $rc
