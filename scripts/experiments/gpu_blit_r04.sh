#!/bin/bash
# Which engine runs a confined pod's copies ("check whether ROCr's internal blit queues honour
# the mask")?  A PyTorch process under libgsx_isolate.so (64-CU partition, 16 GiB share) copies H2D, D2D and D2H;
# rocprofv3's kernel trace lists every kernel dispatch with its queue, the memory-copy trace every SDMA copy.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04_blit}
mkdir -p $OUT
LIB=$PWD/gpushare_scheduler_extender_amd/_native/libgsx_isolate.so
python - > $OUT/env.sh <<PY
from gpushare_scheduler_extender_amd.deviceplugin.allocator import CUPartitioner
from gpushare_scheduler_extender_amd.deviceplugin.isolation import IsolationManager
iso = IsolationManager("$PWD/$OUT/iso")
_, env = iso.prepare("blit", CUPartitioner(256, 8).allocate("blit", 64), 256, 16 << 30, host_process=True)
for k, v in env.items():
    print(f"export {k}='{v}'")
PY
. $OUT/env.sh
cat > $OUT/copies.py <<'PY'
import ctypes, json, os
import torch
x = torch.randn(64 << 20, device="cpu").pin_memory()
a = x.to("cuda", non_blocking=True)        # H2D
b = a.clone()                               # D2D (same device)
c = torch.empty_like(a); c.copy_(b)         # D2D copy_
y = c.to("cpu")                             # D2H
torch.cuda.synchronize()
lib = ctypes.CDLL(os.environ["GSX_LIB"])
st = (ctypes.c_uint64 * 5)()
lib.gsx_isolate_stats(st)
print(json.dumps({"queues": st[0], "masked": st[1], "ok": bool(torch.equal(x, y))}))
PY
GSX_LIB=$HSA_TOOLS_LIB timeout -k 10 120 python $OUT/copies.py > $OUT/copies.json 2> $OUT/copies.err && cat $OUT/copies.json && \
GSX_LIB=$HSA_TOOLS_LIB timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $OUT/copies.py > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
find $OUT/prof -name "*.csv" | head -20
