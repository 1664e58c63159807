#!/usr/bin/env python3
"""Which shapes and tiles does the phased GEMM get wrong?  Every launch follows a device-wide synchronize (the
operands and the reference are produced on torch's stream, the GEMM runs on our own), on uniform [-1, 1) data;
per launch the 256x256 C tiles whose max abs error vs fp32 exceeds 1.0."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from gpushare_scheduler_extender_amd.ops import hip  # noqa: E402


def main():
    shapes = [(512, 256, 64), (256, 512, 64), (1024, 512, 128), (512, 1024, 128), (16384, 4096, 8192),
              (4096, 16384, 8192), (8192, 8192, 8192), (16384, 16384, 4096)]
    s = hip.Stream(0)
    for m, n, k in shapes:
        torch.manual_seed(0)
        a = torch.rand(m, k, device="cuda", dtype=torch.bfloat16) * 2 - 1
        b = torch.rand(n, k, device="cuda", dtype=torch.bfloat16) * 2 - 1
        ref = a.float() @ b.float().t()
        tb = torch.matmul(a, b.t()).float()
        torch.cuda.synchronize()
        row = {"shape": [m, n, k], "torch_bf16_err": round((tb - ref).abs().max().item(), 3)}
        for cfg in (0, 3, 5, 6, 10):
            runs = []
            for _ in range(2):
                c = torch.full((m, n), 7.0, device="cuda", dtype=torch.bfloat16)
                torch.cuda.synchronize()
                try:
                    hip.gemm_bf16_nt_cfg(s, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, cfg)
                except hip.HipError as e:
                    runs.append(f"refused: {e}")
                    break
                s.sync()
                err = (c.float() - ref).abs()
                tm, tn = max(1, m // 256), max(1, n // 256)
                t = err.view(tm, m // tm, tn, n // tn).amax(dim=(1, 3))
                bad = (t > 1.0).nonzero().tolist()
                runs.append({"max_err": round(err.max().item(), 3), "bad_tiles": len(bad), "first": bad[:4]})
            row[str(cfg)] = runs
        print(json.dumps(row), flush=True)
        del a, b, ref, tb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
