"""GPU check of the opt-in one-launch admission (GSX_ADMIT_ONE_LAUNCH=1, read once per process):
   GSX_ADMIT_ONE_LAUNCH=1 PYTHONPATH=. python scripts/experiments/one_launch_check.py
Disjoint extents take the single launch (stamp rows + verify rows), an overlap the two-launch path; the bad-stamp
counts must match the default path's (tests/test_gpu_kernels.py::test_hbm_admit_n_multi_extent_pods)."""
import os

from gpushare_scheduler_extender_amd.ops import hip

assert os.environ.get("GSX_ADMIT_ONE_LAUNCH") == "1", "set GSX_ADMIT_ONE_LAUNCH=1"
s = hip.Stream(0)
buf = hip.DeviceBuffer(0, 64 << 20)
mib8, st = 8 << 20, 1 << 16
a, b = (buf.addr(0), mib8, 11), (buf.addr(2 * mib8), mib8, 22)
assert hip.hbm_admit_n(s, [a, b], 2, st) == 0                      # one launch: two new, nothing resident
c = [(buf.addr(mib8), mib8, 33), (buf.addr(3 * mib8), 2 * mib8, 33)]
assert hip.hbm_admit_n(s, c + [a, b], 2, st) == 0                  # one launch: stamp rows + verify rows
hip.hbm_fill(s, buf.addr(0), 1 << 20, 0)                           # damage a
s.sync()
assert hip.hbm_admit_n(s, c + [a, b], 0, st) == (1 << 20) // st    # verify-only table, one launch
d = [(buf.addr(mib8 + mib8 // 2), mib8, 44)]                       # overlaps c[0] and b: the two-launch path
assert hip.hbm_admit_n(s, d + c + [a, b], 1, st) == 2 * (mib8 // 2) // st + (1 << 20) // st
buf.free()
s.destroy()
print("one-launch ok")
