"""CU-partition isolation benchmark (BASELINE.json config 5: "4 pods co-resident on one MI355X with per-pod CU partitions").

The reference leaves isolation to the application (``docs/designs/designs.md:25-28``)
and lists "integrate Nvidia MPS" as a roadmap item (``README.md:77``).  Our
stand-in is a per-pod CU partition handed out by the device plugin.  This
harness runs the pod workload (:mod:`.workload`) as real processes with the
exact environment the device plugin's Allocate produces, in four scenarios:

* ``solo``          one pod alone on the GPU (reference throughput);
* ``shared``        4 pods co-resident, no partition (time-sliced, unisolated);
* ``partitioned``   4 pods co-resident, 64 CUs each via the stream CU mask;
* ``env``           4 pods co-resident, 64 CUs each via ``HSA_CU_MASK`` only
                    (process-wide; applies to torch's own queues too), hipBLASLt GEMM;
* ``env-gsx``       the same with the libgsx_kernels GEMM (stream mask vs process mask, same kernel);
* ``solo64``        one pod alone inside a 64-CU partition (what a partition is worth);
* ``noisy`` / ``noisy-partitioned``  pod 0 runs a small (latency-bound) GEMM
                    next to 3 pods running large GEMMs, without / with
                    partitions: pod 0's throughput relative to ``solo`` / ``solo64``
                    is the interference the partition removes.

Reported per scenario: per-pod TFLOP/s, aggregate, and fairness (min/max).
Run: ``python -m gsxtools.isolation --seconds 8``.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

from gpushare_scheduler_extender_amd.deviceplugin.allocator import CUPartitioner, build_response
from gpushare_scheduler_extender_amd.deviceplugin.devices import Device
from gpushare_scheduler_extender_amd.k8s.objects import make_pod
from gpushare_scheduler_extender_amd.models.profile import SHARED_GPU

ROOT = Path(__file__).resolve().parents[1]


def pod_envs(n_pods: int, cus_each: int, gpu_total_gib: int, pod_gib: int, with_mask: bool) -> list[dict]:
    dev = Device(index=0, total_bytes=gpu_total_gib << 30)
    part = CUPartitioner(dev.cu_count, dev.xcc_count)
    envs = []
    for i in range(n_pods):
        pod = make_pod(f"iso-{i}", pod_gib, annotations={SHARED_GPU.annotation_idx: "0",
                                                         SHARED_GPU.annotation_dev: str(gpu_total_gib)})
        cus = part.allocate(f"iso-{i}", cus_each) if with_mask else None
        envs.append(build_response(pod, dev, pod_gib, SHARED_GPU, mount_mode="all", cus=cus).envs)
    return envs


def run_pods(envs: list[dict], seconds: float, kernel: str, size, mask_mode: str) -> list[dict]:
    start_at = time.time() + 20.0  # time for every process to import torch and warm up
    procs = []
    sizes = size if isinstance(size, list) else [size] * len(envs)
    for e, sz in zip(envs, sizes):
        env = dict(os.environ)
        env.update({k: v for k, v in e.items() if k not in ("GSX_CU_MASK", "HSA_CU_MASK")})
        if mask_mode in ("stream", "both") and "GSX_CU_MASK" in e:
            env["GSX_CU_MASK"] = e["GSX_CU_MASK"]
        if mask_mode in ("env", "both") and "HSA_CU_MASK" in e:
            env["HSA_CU_MASK"] = e["HSA_CU_MASK"]
        env["HIP_VISIBLE_DEVICES"] = "0"
        env["ROCR_VISIBLE_DEVICES"] = "0"
        env["GSX_START_AT"] = str(start_at)
        env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
        cmd = [sys.executable, "-m", "gsxtools.workload", "--total",
               e["SHARED_GPU_MEM_DEV"], "--allocated", e["SHARED_GPU_MEM_CONTAINER"], "--kernel", kernel,
               "--size", str(sz), "--seconds", str(seconds), "--json"]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      cwd=str(ROOT)))
    out = []
    for p in procs:
        so, se = p.communicate(timeout=seconds + 180)
        if p.returncode != 0:
            raise RuntimeError(f"workload failed rc={p.returncode}: {se[-2000:]}")
        out.append(json.loads(so.strip().splitlines()[-1]))
    return out


def summarize(name: str, res: list[dict]) -> dict:
    t = [r["tflops"] for r in res]
    return {"scenario": name, "pods": len(t), "per_pod_tflops": [round(x, 1) for x in t],
            "aggregate_tflops": round(sum(t), 1), "fairness_min_over_max": round(min(t) / max(t), 3) if t else None}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=4)
    ap.add_argument("--cus", type=int, default=64)
    ap.add_argument("--pod-gib", type=int, default=64)
    ap.add_argument("--gpu-gib", type=int, default=287)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--kernel", default="gsx", choices=["gsx", "torch"])
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--small-size", type=int, default=2048)
    ap.add_argument("--scenarios",
                    default="solo,shared,partitioned,env,env-gsx,solo-small,solo64,noisy,noisy-partitioned")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)
    results = []
    for sc in a.scenarios.split(","):
        if sc == "solo":
            envs = pod_envs(1, a.cus, a.gpu_gib, a.pod_gib, False)
            res = run_pods(envs, a.seconds, a.kernel, a.size, "none")
        elif sc == "shared":
            envs = pod_envs(a.pods, a.cus, a.gpu_gib, a.pod_gib, False)
            res = run_pods(envs, a.seconds, a.kernel, a.size, "none")
        elif sc == "partitioned":
            envs = pod_envs(a.pods, a.cus, a.gpu_gib, a.pod_gib, True)
            res = run_pods(envs, a.seconds, a.kernel, a.size, "stream")
        elif sc == "solo64":
            envs = pod_envs(1, a.cus, a.gpu_gib, a.pod_gib, True)
            res = run_pods(envs, a.seconds, a.kernel, a.small_size, "stream")
        elif sc == "solo-small":
            envs = pod_envs(1, a.cus, a.gpu_gib, a.pod_gib, False)
            res = run_pods(envs, a.seconds, a.kernel, a.small_size, "none")
        elif sc in ("noisy", "noisy-partitioned"):
            masked = sc == "noisy-partitioned"
            envs = pod_envs(a.pods, a.cus, a.gpu_gib, a.pod_gib, masked)
            sizes = [a.small_size] + [a.size] * (a.pods - 1)
            res = run_pods(envs, a.seconds, a.kernel, sizes, "stream" if masked else "none")
        elif sc == "env":
            envs = pod_envs(a.pods, a.cus, a.gpu_gib, a.pod_gib, True)
            res = run_pods(envs, a.seconds, "torch" if a.kernel == "gsx" else a.kernel, a.size, "env")
        elif sc == "env-gsx":
            envs = pod_envs(a.pods, a.cus, a.gpu_gib, a.pod_gib, True)
            res = run_pods(envs, a.seconds, a.kernel, a.size, "env")
        else:
            raise SystemExit(f"unknown scenario {sc}")
        s = summarize(sc, res)
        print(json.dumps(s), flush=True)
        results.append(s)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(results, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
