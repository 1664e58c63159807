set -x
mkdir -p gpurun_out/isodbg
cd gpurun_out/isodbg
printf 'cu_mask=0x000000ff,0x000000ff,0x000000ff,0x000000ff,0x000000ff,0x000000ff,0x000000ff,0x000000ff\nhbm_limit_bytes=8589934592\nledger=%s/hbm.ledger\n' "$PWD" > iso.conf
cd ../..
N=gpushare_scheduler_extender_amd/_native
GSX_ISOLATION_VERBOSE=1 HSA_TOOLS_LIB=$PWD/$N/libgsx_isolate.so timeout -k 5 60 $N/gsx-cuprobe > gpurun_out/isodbg/a_noconf.txt 2>&1; echo "rc=$?" >> gpurun_out/isodbg/a_noconf.txt
GSX_ISOLATION_CONFIG=$PWD/gpurun_out/isodbg/iso.conf GSX_ISOLATION_VERBOSE=1 HSA_TOOLS_LIB=$PWD/$N/libgsx_isolate.so timeout -k 5 60 $N/gsx-cuprobe > gpurun_out/isodbg/b_conf.txt 2>&1; echo "rc=$?" >> gpurun_out/isodbg/b_conf.txt
GSX_ISOLATION_CONFIG=$PWD/gpurun_out/isodbg/iso.conf GSX_ISOLATION_VERBOSE=1 HSA_TOOLS_LIB=$PWD/$N/libgsx_isolate.so timeout -k 5 60 $N/gsx-memprobe --alloc 1073741824 > gpurun_out/isodbg/c_mem.txt 2>&1; echo "rc=$?" >> gpurun_out/isodbg/c_mem.txt
true
