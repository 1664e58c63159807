#!/usr/bin/env python3
"""Run the bf16 GEMM tile configs a few times at one shape (for rocprofv3 kernel traces / PMC counters)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gpushare_scheduler_extender_amd.ops import hip  # noqa: E402

m = n = k = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
cfgs = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [3, 5]
a = torch.rand(m, k, device="cuda", dtype=torch.bfloat16) * 2 - 1
b = torch.rand(n, k, device="cuda", dtype=torch.bfloat16) * 2 - 1
c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
s = hip.Stream(0)
torch.cuda.synchronize()
for cfg in cfgs:
    for _ in range(5):
        hip.gemm_bf16_nt_cfg(s, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, cfg)
    s.sync()
for _ in range(5):
    torch.matmul(a, b.t())
torch.cuda.synchronize()
s.destroy()
print("ok", m, n, k, cfgs)
