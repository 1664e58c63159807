"""The pod workload: a PyTorch-ROCm / HIP GEMM loop that stays inside its GPU share.

Counterpart of the reference's sample container (``samples/docker/main.py``:
TF1 with ``per_process_gpu_memory_fraction`` from ``SHARED_GPU_MEM_DEV`` /
``_CONTAINER``, a tiny matmul forever).  Here:

* the memory share becomes ``torch.cuda.set_per_process_memory_fraction``
  (allocated / device total), so the caching allocator refuses to grow past
  the pod's gpu-mem;
* a CU partition handed out by the device plugin (``GSX_CU_MASK`` words) is
  applied by running the work on a ``hipExtStreamCreateWithCUMask`` stream
  wrapped as a ``torch.cuda.ExternalStream``; ``HSA_CU_MASK`` (set by the plugin
  too) restricts every queue of the process, including torch's own;
* the compute is the bf16 MFMA GEMM of ``libgsx_kernels`` (``--kernel gsx``)
  or ``torch.matmul`` / hipBLASLt (``--kernel torch``), reported as TFLOP/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def parse_mask(s: str) -> list[int]:
    return [int(x, 16) for x in s.split(",") if x]


def run(total: float, allocated: float, *, kernel: str = "gsx", size: int = 8192, seconds: float = 0.0,
        iters: int = 0, report_every: float = 5.0, touch: bool = False, quiet: bool = False,
        probe_limit: bool = False) -> dict:
    import torch

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    frac = 1.0 if not total else max(0.0, min(1.0, allocated / total))
    torch.cuda.set_per_process_memory_fraction(frac, dev)
    stream = None
    hip_stream = None
    if os.environ.get("GSX_CU_MASK"):
        from gpushare_scheduler_extender_amd.ops import hip  # noqa: PLC0415

        hip_stream = hip.Stream(0, parse_mask(os.environ["GSX_CU_MASK"]))
        stream = torch.cuda.ExternalStream(hip_stream.ptr, device=dev)
    hold = None
    if touch:
        # claim (most of) the share so co-resident pods really contend for HBM
        hold = torch.empty(int(allocated * (1 << 30) * 0.9) // 2, dtype=torch.bfloat16, device=dev)
        hold.fill_(1)
    m = n = k = size
    a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
    c = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    if kernel == "gsx":
        from gpushare_scheduler_extender_amd.ops import hip  # noqa: PLC0415

        gs = hip_stream or hip.Stream(0)

        def step():
            hip.gemm_bf16_nt(gs, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k)

        def sync():
            gs.sync()
    else:
        def step():
            if stream is not None:
                with torch.cuda.stream(stream):
                    torch.matmul(a, b.t(), out=c)
            else:
                torch.matmul(a, b.t(), out=c)

        def sync():
            (stream or torch.cuda.current_stream()).synchronize()
    torch.cuda.synchronize()
    for _ in range(3):
        step()
    sync()
    start_at = float(os.environ.get("GSX_START_AT", "0") or 0)
    if start_at:  # co-resident pods start their timed loops together (isolation bench)
        time.sleep(max(0.0, start_at - time.time()))
    flops = 2.0 * m * n * k
    done = 0
    t0 = last = time.perf_counter()
    last_done = 0
    rates = []
    while True:
        for _ in range(10):
            step()
        done += 10
        sync()
        now = time.perf_counter()
        if now - last >= report_every:
            r = (done - last_done) * flops / (now - last) / 1e12
            rates.append(r)
            if not quiet:
                print(f"[workload] {r:.1f} TFLOP/s  share={allocated}/{total} GiB frac={frac:.3f}", flush=True)
            last, last_done = now, done
        if (seconds and now - t0 >= seconds) or (iters and done >= iters):
            break
    el = time.perf_counter() - t0
    out = {"tflops": done * flops / el / 1e12, "iters": done, "seconds": el, "fraction": frac,
           "cu_mask": os.environ.get("GSX_CU_MASK", ""), "kernel": kernel, "size": size,
           "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES", ""),
           "device_total_bytes": torch.cuda.get_device_properties(dev).total_memory}
    if probe_limit and allocated:
        # the share is a ceiling: one more share-sized tensor must be refused by the caching allocator
        try:
            extra = torch.empty(int(allocated * (1 << 30)) // 2, dtype=torch.bfloat16, device=dev)
            del extra
            out["limit_enforced"] = False
        except torch.cuda.OutOfMemoryError:
            out["limit_enforced"] = True
    del hold
    if hip_stream is not None:
        hip_stream.destroy()
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", type=float, default=float(os.environ.get("SHARED_GPU_MEM_DEV", "0") or 0))
    ap.add_argument("--allocated", type=float, default=float(os.environ.get("SHARED_GPU_MEM_CONTAINER", "0") or 0))
    ap.add_argument("--kernel", default="gsx", choices=["gsx", "torch"])
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--seconds", type=float, default=0.0, help="0 = run forever (like the reference sample)")
    ap.add_argument("--iters", type=int, default=0)
    ap.add_argument("--touch", action="store_true")
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--probe-limit", action="store_true", help="check that the memory share is enforced")
    a = ap.parse_args(argv)
    res = run(a.total, a.allocated, kernel=a.kernel, size=a.size, seconds=a.seconds, iters=a.iters, touch=a.touch,
              quiet=a.json, probe_limit=a.probe_limit)
    print(json.dumps(res) if a.json else res, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
