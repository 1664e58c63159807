"""PMC probe of the pod-admission kernels: 4 x 64 GiB slices resident in a 256 GiB arena, a new slice stamped and
all four verified, at a 1 MiB and a 2 MiB stamp stride (one launch pair per admission, as PodRuntime does).
Run under rocprofv3 --pmc; the kernel names and the dispatch order tell the strides apart (1 MiB first)."""
import sys

from gpushare_scheduler_extender_amd.ops import hip

GiB, MiB = 1 << 30, 1 << 20
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
s = hip.Stream(0)
buf = hip.DeviceBuffer(0, 256 * GiB)
try:
    slices = [(buf.addr(i * 64 * GiB), 64 * GiB, 0x1000 + 2 * i + 1) for i in range(4)]
    for stride in (1 * MiB, 2 * MiB):
        hip.hbm_admit_n(s, slices, 4, stride)  # stamp all four once
        for _ in range(n):
            bad = hip.hbm_admit_n(s, slices[3:] + slices[:3], 1, stride)
            assert bad == 0, bad
    print("ok", n)
finally:
    s.sync()
    s.destroy()
    buf.free()
