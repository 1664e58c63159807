#!/bin/bash
# How much HBM does the HSA runtime take for scratch (private memory) behind the allocation API, and does the
# isolation library's account see it?  gsx-memprobe --scratch runs a kernel whose lanes keep a 1/16/64 KiB
# private array; the JSON carries amdkfd's per-process VRAM count before and after.  Unconfined, then under an
# 8 GiB share.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04_scratch}
mkdir -p $OUT
P=gpushare_scheduler_extender_amd/_native/gsx-memprobe
LIB=$PWD/gpushare_scheduler_extender_amd/_native/libgsx_isolate.so
ls /sys/class/kfd/kfd/proc/ > $OUT/kfd_proc.txt 2>&1 || true
for kib in 1 16 64; do
  timeout -k 10 60 $P --scratch $kib --blocks 16384 > $OUT/free.$kib.json 2> $OUT/free.$kib.err || { echo "free $kib rc=$?"; cat $OUT/free.$kib.err; exit 1; }
  cat $OUT/free.$kib.json
done
CONF=$OUT/iso.conf
printf 'hbm_limit_bytes=%d\nledger=%s\n' $((8 << 30)) $PWD/$OUT/hbm.ledger > $CONF
for kib in 1 16 64; do
  GSX_ISOLATION_CONFIG=$PWD/$CONF HSA_TOOLS_LIB=$LIB timeout -k 10 60 $P --alloc $((6 << 30)) --touch --scratch $kib --blocks 16384 \
    > $OUT/iso.$kib.json 2> $OUT/iso.$kib.err || { echo "iso $kib rc=$?"; cat $OUT/iso.$kib.err; exit 1; }
  cat $OUT/iso.$kib.json
done
for lim in $((1 << 30)); do
  HSA_SCRATCH_SINGLE_LIMIT=$lim timeout -k 10 60 $P --scratch 16 --blocks 16384 > $OUT/single.$lim.json 2> $OUT/single.$lim.err || { echo "single rc=$?"; cat $OUT/single.$lim.err; exit 1; }
  cat $OUT/single.$lim.json
done
# the async scratch threshold (hsa_amd_agent_set_async_scratch_limit) and the runtime's own knobs
timeout -k 10 60 $P --scratch 16 --blocks 16384 --scratch-limit $((256 << 20)) > $OUT/thresh.json 2> $OUT/thresh.err || { echo "thresh rc=$?"; cat $OUT/thresh.err; exit 1; }
cat $OUT/thresh.json
for mem in $((1 << 30)) 4096; do
  HSA_SCRATCH_MEM=$mem timeout -k 10 60 $P --scratch 16 --blocks 16384 > $OUT/mem.$mem.json 2> $OUT/mem.$mem.err || { echo "mem $mem rc=$?"; cat $OUT/mem.$mem.err; exit 1; }
  cat $OUT/mem.$mem.json
done
