#!/usr/bin/env python3
"""Micro-benchmarks of the HIP kernels on one MI355X: bf16 GEMM (ours vs torch/hipBLASLt), HBM fill, stamp/verify."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gpushare_scheduler_extender_amd.ops import hip  # noqa: E402


def gemm(size_list, iters=20):
    out = []
    s = hip.Stream(0)
    for m, n, k in size_list:
        a = torch.rand(m, k, device="cuda", dtype=torch.bfloat16) * 2 - 1
        b = torch.rand(n, k, device="cuda", dtype=torch.bfloat16) * 2 - 1
        c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        torch.cuda.synchronize()
        hip.time_gemm(s, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, 3)
        ms = hip.time_gemm(s, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, iters) / iters
        ours = 2 * m * n * k / ms / 1e9
        for _ in range(3):
            torch.matmul(a, b.t())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            torch.matmul(a, b.t())
        e1.record()
        torch.cuda.synchronize()
        tms = e0.elapsed_time(e1) / iters
        ref = 2 * m * n * k / tms / 1e9
        err = (c.float() - (a.float() @ b.float().t())).abs().max().item()
        row = {"m": m, "n": n, "k": k, "gsx_tflops": round(ours, 1), "torch_tflops": round(ref, 1),
               "gsx_ms": round(ms, 4), "max_abs_err": round(err, 4)}
        ts = torch.cuda.ExternalStream(s.ptr)
        for cfg, name in hip.GEMM_CFGS.items():
            try:
                hip.gemm_bf16_nt_cfg(s, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, cfg)
            except hip.HipError:
                continue
            s.sync()
            e = (c.float() - (a.float() @ b.float().t())).abs().max().item()
            torch.cuda.synchronize()
            with torch.cuda.stream(ts):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(ts)
                for _ in range(iters):
                    hip.gemm_bf16_nt_cfg(s, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, cfg)
                e1.record(ts)
            e1.synchronize()
            cms = e0.elapsed_time(e1) / iters
            row[f"cfg{cfg}_{name}_tflops"] = round(2 * m * n * k / cms / 1e9, 1)
            row[f"cfg{cfg}_err"] = round(e, 4)
        out.append(row)
        del a, b, c
    s.destroy()
    return out


def hbm(nbytes=16 << 30, reps=5):
    s = hip.Stream(0)
    buf = hip.DeviceBuffer(0, nbytes)
    hip.hbm_fill(s, buf.addr(), nbytes, 1)
    s.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        hip.hbm_fill(s, buf.addr(), nbytes, 2)
    s.sync()
    fill = reps * nbytes / (time.perf_counter() - t0) / 1e12
    gib64 = 64 << 30
    big = hip.DeviceBuffer(0, gib64)
    t0 = time.perf_counter()
    hip.hbm_stamp(s, big.addr(), gib64, 1 << 20, 42)
    s.sync()
    stamp_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    bad = hip.hbm_verify(s, big.addr(), gib64, 1 << 20, 42)
    verify_ms = (time.perf_counter() - t0) * 1e3
    buf.free()
    big.free()
    s.destroy()
    return {"fill_TBps": round(fill, 2), "stamp_64GiB_ms": round(stamp_ms, 3), "verify_64GiB_ms": round(verify_ms, 3),
            "bad": bad}


if __name__ == "__main__":
    sizes = [(4096, 4096, 4096), (8192, 8192, 8192), (2048, 8192, 4096), (16384, 16384, 8192)]
    res = {"gemm_bf16_nt": gemm(sizes), "hbm": hbm()}
    print(json.dumps(res))
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(res, f, indent=1)
