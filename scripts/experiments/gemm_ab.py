#!/usr/bin/env python3
"""Interleaved A/B of GEMM variants in one process (cdna guide rule 24): our phased 256x256 kernel on the 16x16x32
MFMA (cfg 5) and on the 32x32x16 MFMA (cfg 10) against torch.matmul (hipBLASLt), uniform [-1, 1) bf16 operands.
Prints one JSON line: per size, per variant, median / min TFLOP/s over the rounds and the max abs error vs fp32."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from gpushare_scheduler_extender_amd.ops import hip  # noqa: E402


def main():
    sizes = [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 16384, 8192)]
    rounds, iters = int(os.environ.get("ROUNDS", "7")), 20
    s = hip.Stream(0)
    ts = torch.cuda.ExternalStream(s.ptr)
    out = {}
    for m, n, k in sizes:
        a = torch.rand(m, k, device="cuda", dtype=torch.bfloat16) * 2 - 1
        b = torch.rand(n, k, device="cuda", dtype=torch.bfloat16) * 2 - 1
        c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        ref = a.float() @ b.float().t()
        torch.cuda.synchronize()  # operands and reference come from torch's stream; the GEMMs run on ours
        errs = {}
        for cfg in (5, 10):
            hip.gemm_bf16_nt_cfg(s, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, cfg)
            s.sync()
            errs[cfg] = (c.float() - ref).abs().max().item()
        errs["torch"] = (torch.matmul(a, b.t()).float() - ref).abs().max().item()
        del ref
        runs = {5: [], 10: [], "torch": []}

        def timed(fn):
            torch.cuda.synchronize()
            with torch.cuda.stream(ts):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(ts)
                for _ in range(iters):
                    fn()
                e1.record(ts)
            e1.synchronize()
            return 2 * m * n * k / (e0.elapsed_time(e1) / iters) / 1e9

        for _ in range(2):  # warm-up: clocks, code objects
            for cfg in (5, 10):
                timed(lambda cfg=cfg: hip.gemm_bf16_nt_cfg(s, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, cfg))
            timed(lambda: torch.matmul(a, b.t(), out=c))
        for _ in range(rounds):
            for cfg in (5, 10):
                runs[cfg].append(timed(
                    lambda cfg=cfg: hip.gemm_bf16_nt_cfg(s, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, cfg)))
            runs["torch"].append(timed(lambda: torch.matmul(a, b.t(), out=c)))
        out[f"{m}x{n}x{k}"] = {str(v): {"median_tflops": round(statistics.median(r), 1), "min_tflops": round(min(r), 1),
                                        "max_abs_err": round(errs[v], 4)} for v, r in runs.items()}
        del a, b, c
    print(json.dumps(out))


if __name__ == "__main__":
    main()
