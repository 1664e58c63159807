"""Enforced isolation on a real MI355X (VERDICT r2 "what's missing" #2): a plain HIP program that never sees
``HSA_CU_MASK`` still runs on exactly its 64-CU partition, and allocating past its HBM share fails.

Every pod environment here is produced by the device plugin's :class:`IsolationManager` for a host-process
launcher (``HSA_TOOLS_LIB`` + ``GSX_ISOLATION_CONFIG``; in a container the same files arrive as read-only
mounts and ``/etc/ld.so.preload``).  The programs are the compiled probes ``gsx-cuprobe`` (hardware CU id of
every workgroup) and ``gsx-memprobe`` (hipMalloc / hipMemGetInfo), and PyTorch itself.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

from gpushare_scheduler_extender_amd.deviceplugin.allocator import CUPartitioner
from gpushare_scheduler_extender_amd.deviceplugin.isolation import IsolationManager

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
NATIVE = ROOT / "gpushare_scheduler_extender_amd" / "_native"
GIB = 1 << 30


def _env(extra: dict) -> dict:
    env = {k: v for k, v in os.environ.items() if k not in ("HSA_CU_MASK", "GSX_CU_MASK", "HSA_TOOLS_LIB")}
    env.update(extra)
    return env


def _run(cmd, env, timeout=120) -> dict:
    r = subprocess.run([str(c) for c in cmd], env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (cmd, r.returncode, r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture
def iso(tmp_path):
    lib = NATIVE / "libgsx_isolate.so"
    if not lib.exists():
        pytest.fail("libgsx_isolate.so not built: python native/build.py isolate")
    return IsolationManager(str(tmp_path / "iso"))


def _cus(out: dict) -> set:
    return {tuple(c) for c in out["cus"]}


def test_cu_partition_is_enforced_without_hsa_cu_mask(iso):
    """Config 5 through the isolation library: four 64-CU pods, each probe process with HSA_CU_MASK unset."""
    probe = NATIVE / "gsx-cuprobe"
    full = _run([probe, "--list"], _env({}))
    assert full["distinct_cus"] == 256
    part = CUPartitioner(256, 8)
    sets = []
    for i in range(4):
        cus = part.allocate(f"pod-{i}", 64)
        _, env = iso.prepare(f"pod-{i}", cus, 256, 8 * GIB, host_process=True)
        out = _run([probe, "--list"], _env(env))
        assert out["hsa_cu_mask"] == ""
        assert out["distinct_cus"] == 64, out
        assert out["per_xcd"] == [8] * 8, out  # the partitioner's 8 CUs on each XCD
        sets.append(_cus(out))
    assert all(not (sets[i] & sets[j]) for i in range(4) for j in range(i + 1, 4))
    # a stream that asks for all 256 CUs (hipExtStreamCreateWithCUMask) stays inside the partition
    _, env0 = iso.prepare("pod-0", part.held()["pod-0"], 256, 8 * GIB, host_process=True)
    wide = _run([probe, "--mask", "0-255", "--list"], _env(env0))
    assert wide["distinct_cus"] == 64 and _cus(wide) == sets[0]
    # an HSA_CU_MASK the container sets for itself cannot widen it either
    env0b = dict(env0, HSA_CU_MASK="0:0-255")
    assert _run([probe, "--list"], _env(env0b))["distinct_cus"] == 64


def test_hbm_share_is_enforced_for_a_hip_program(iso):
    probe = NATIVE / "gsx-memprobe"
    share = 8 * GIB
    _, env = iso.prepare("mem-0", None, 256, share, host_process=True)
    out = _run([probe, "--alloc", f"{6 * GIB},{3 * GIB},{GIB}", "--touch"], _env(env))
    assert out["total"] == share, out  # hipMemGetInfo reports the share as the device size
    assert out["free"] <= share
    assert [a["ok"] for a in out["allocs"]] == [True, False, True], out
    assert out["allocs"][1]["err"] == "hipErrorOutOfMemory"
    over = _run([probe, "--alloc", str(share + GIB)], _env(env))
    assert over["allocs"][0]["ok"] is False
    free_ = _run([probe, "--alloc", str(share + GIB)], _env({}))  # unconfined control: the whole GPU
    assert free_["total"] > 200 * GIB and free_["allocs"][0]["ok"] is True


def test_hbm_share_is_per_pod_across_processes(iso):
    """Two processes of one pod share one account; a process that exits gives its bytes back."""
    probe = NATIVE / "gsx-memprobe"
    _, env = iso.prepare("mem-1", None, 256, 8 * GIB, host_process=True)
    holder = subprocess.Popen([str(probe), "--alloc", str(6 * GIB), "--touch", "--hold-ms", "20000"], env=_env(env),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        first = json.loads(holder.stdout.readline())  # printed once the 6 GiB are held
        assert first["allocs"][0]["ok"] is True
        other = _run([probe, "--alloc", f"{3 * GIB},{GIB}"], _env(env))
        assert [a["ok"] for a in other["allocs"]] == [False, True], other
        assert other["total"] == 8 * GIB and other["free"] <= 2 * GIB + (64 << 20)
    finally:
        holder.kill()
        holder.wait(30)
    after = _run([probe, "--alloc", str(6 * GIB)], _env(env))
    assert after["allocs"][0]["ok"] is True, after


def test_pytorch_sees_and_respects_the_share(iso):
    share = 16 * GIB
    _, env = iso.prepare("torch-0", None, 256, share, host_process=True)
    code = (
        "import json,torch\n"
        "free,total=torch.cuda.mem_get_info()\n"
        "props=torch.cuda.get_device_properties(0).total_memory\n"
        "x=torch.empty(8<<30,dtype=torch.uint8,device='cuda'); x.fill_(1); torch.cuda.synchronize()\n"
        "try:\n"
        "    y=torch.empty(12<<30,dtype=torch.uint8,device='cuda'); oom=False\n"
        "except torch.OutOfMemoryError:\n"
        "    oom=True\n"
        "print(json.dumps({'free':free,'total':total,'props':props,'oom':oom,'sum':int(x[:1024].sum())}))\n")
    out = _run([sys.executable, "-c", code], _env(env), timeout=300)
    assert out["total"] == share and out["props"] == share, out
    assert out["oom"] is True and out["sum"] == 1024


@pytest.mark.parametrize("api", ["async", "finegrained", "pitch", "vmem"])
def test_hbm_share_covers_every_device_allocation_api(iso, api):
    """Stream-ordered pools, fine-grained device memory, pitched allocations and the virtual-memory API
    (hipMemCreate: PyTorch's expandable segments) all take HBM, so all count against the pod's share."""
    probe = NATIVE / "gsx-memprobe"
    _, env = iso.prepare(f"api-{api}", None, 256, 8 * GIB, host_process=True)
    out = _run([probe, "--api", api, "--alloc", f"{6 * GIB},{6 * GIB}"], _env(env))
    assert [a["ok"] for a in out["allocs"]] == [True, False], out
    ctl = _run([probe, "--api", api, "--alloc", f"{6 * GIB},{6 * GIB}"], _env({}))  # unconfined: both fit
    assert [a["ok"] for a in ctl["allocs"]] == [True, True], ctl


def test_host_memory_is_not_the_share(iso):
    """Pinned host memory (hipHostMalloc) lives in system RAM: it must not count against the HBM share."""
    probe = NATIVE / "gsx-memprobe"
    _, env = iso.prepare("api-host", None, 256, 4 * GIB, host_process=True)
    out = _run([probe, "--api", "host", "--alloc", f"{3 * GIB},{3 * GIB}"], _env(env))
    assert [a["ok"] for a in out["allocs"]] == [True, True], out


def test_pytorch_expandable_segments_respect_the_share(iso):
    """PYTORCH_HIP_ALLOC_CONF=expandable_segments:True maps growing segments through the virtual-memory API."""
    share = 16 * GIB
    _, env = iso.prepare("torch-exp", None, 256, share, host_process=True)
    env = dict(env, PYTORCH_HIP_ALLOC_CONF="expandable_segments:True", PYTORCH_CUDA_ALLOC_CONF="expandable_segments:True")
    code = (
        "import json,torch\n"
        "xs=[]\n"
        "oom=False\n"
        "try:\n"
        "    for _ in range(24):\n"
        "        xs.append(torch.empty(1<<30,dtype=torch.uint8,device='cuda'))\n"
        "except torch.OutOfMemoryError:\n"
        "    oom=True\n"
        "print(json.dumps({'gib':len(xs),'oom':oom,'reserved':torch.cuda.memory_reserved()}))\n")
    out = _run([sys.executable, "-c", code], _env(env), timeout=300)
    assert out["oom"] is True and out["gib"] <= 16, out
    assert out["reserved"] <= share, out


def _preload_env(env: dict) -> dict:
    """The container route: the library arrives by preload only (LD_PRELOAD standing in for /etc/ld.so.preload),
    never through HSA_TOOLS_LIB in the environment the process starts with."""
    out = {k: v for k, v in env.items() if k != "HSA_TOOLS_LIB"}
    out = _env(out)
    out["LD_PRELOAD"] = ":".join(x for x in (os.environ.get("LD_PRELOAD", ""), env["HSA_TOOLS_LIB"]) if x)
    return out


def test_preloaded_library_confines_a_process_that_drops_hsa_tools_lib(iso):
    """VERDICT r3 missing 4: a process that unsets HSA_TOOLS_LIB before its first HIP call is still confined -- the
    library's own hsa_init puts it back right before ROCr reads it."""
    probe = NATIVE / "gsx-cuprobe"
    cus = CUPartitioner(256, 8).allocate("drop-0", 64)
    _, env = iso.prepare("drop-0", cus, 256, 8 * GIB, host_process=True)
    out = _run([probe, "--unsetenv", "HSA_TOOLS_LIB", "--list"], _preload_env(env))
    assert out["distinct_cus"] == 64 and out["per_xcd"] == [8] * 8, out


def test_preloaded_library_confines_pytorch_that_pops_hsa_tools_lib(iso):
    share = 16 * GIB
    _, env = iso.prepare("drop-torch", CUPartitioner(256, 8).allocate("drop-torch", 64), 256, share, host_process=True)
    code = (
        "import json,os\n"
        "os.environ.pop('HSA_TOOLS_LIB', None)\n"  # before import torch: before the first HIP call
        "import torch\n"
        "free,total=torch.cuda.mem_get_info()\n"
        "x=torch.empty(8<<30,dtype=torch.uint8,device='cuda'); x.fill_(1); torch.cuda.synchronize()\n"
        "try:\n"
        "    y=torch.empty(12<<30,dtype=torch.uint8,device='cuda'); oom=False\n"
        "except torch.OutOfMemoryError:\n"
        "    oom=True\n"
        "print(json.dumps({'total':total,'oom':oom,'tools':os.environ.get('HSA_TOOLS_LIB','')}))\n")
    out = _run([sys.executable, "-c", code], _preload_env(env), timeout=300)
    assert out["total"] == share and out["oom"] is True, out


def test_scratch_fits_in_the_share_or_the_kernel_is_refused(iso):
    """scratch (private memory) is allocated by the runtime behind every allocation API.  A code
    object whose kernel can need more scratch than the share has left is refused at load (cleanly: an error
    code, no fault); one that fits is charged against the share, and what the device really holds stays
    within it."""
    probe = NATIVE / "gsx-memprobe"
    share = 8 * GIB
    _, env = iso.prepare("scr-0", None, 256, share, host_process=True)
    # 16 KiB a lane: ~8.7 GB at full occupancy, more than the 8 GiB share
    big = _run([probe, "--scratch", "16", "--blocks", "16384"], _env(env))
    assert big["scratch"]["ok"] is False and big["scratch"]["stage"] == "load", big
    # 1 KiB a lane (1280-byte granules: ~0.67 GB): loads, runs, and the share's free memory shrinks by the charge
    small = _run([probe, "--scratch", "1", "--blocks", "16384"], _env(env))
    assert small["scratch"]["ok"] is True, small
    assert small["scratch"]["free_after"] <= share - 600 * (1 << 20), small
    # 6 GiB allocated first: a 4 KiB-a-lane kernel (~2.3 GB) no longer fits
    mid = _run([probe, "--alloc", str(6 * GIB), "--touch", "--scratch", "4", "--blocks", "16384"], _env(env))
    assert mid["allocs"][0]["ok"] is True and mid["scratch"]["ok"] is False, mid
    assert mid["scratch"]["stage"] == "load", mid
    # what the device holds for a pod process with 6 GiB allocated and a scratch kernel run (an unconfined observer
    # reads the device's free memory before and while it holds them): within the share, plus the HIP runtime's own
    # small allocations (queues, code objects), which no allocation API reports
    before = _run([probe], _env({}))["free"]
    holder = subprocess.Popen([str(probe), "--alloc", str(6 * GIB), "--touch", "--scratch", "1", "--blocks", "16384",
                               "--hold-ms", "20000"], env=_env(env), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True)
    try:
        first = json.loads(holder.stdout.readline())
        assert first["allocs"][0]["ok"] is True and first["scratch"]["ok"] is True, first
        during = _run([probe], _env({}))["free"]
    finally:
        holder.kill()
        holder.wait(30)
    assert before - during <= share + 512 * (1 << 20), (before, during)


def test_concurrent_scratch_is_charged_per_queue_or_refused(iso):
    """ROCr gives each hardware queue its own scratch, so four streams running the 1 KiB-a-lane
    kernel at the same instant hold four times one dispatch's.  The isolation library charges the worst kernel's
    scratch on every queue: under a share sized for one charge the work is refused cleanly (a queue or the code
    object, an error code, no fault) or runs fully charged; under a share with room for four it runs, and an
    unconfined observer sees the pod hold no more than the share (+ the runtime's own small allocations)."""
    probe = NATIVE / "gsx-memprobe"
    one = _run([probe, "--scratch", "1", "--blocks", "16384"],
               _env(iso.prepare("scr-one", None, 256, 8 * GIB, host_process=True)[1]))["scratch"]
    assert one["ok"] and one["iso"] and one["iso_worst"] > 0, one
    worst = one["iso_worst"]  # one queue's worst-case scratch for this kernel (~0.67 GB on MI355X)
    # a share for one charge, not four
    share = worst + 256 * (1 << 20)
    _, env = iso.prepare("scr-q1", None, 256, share, host_process=True)
    out = _run([probe, "--scratch", "1", "--blocks", "16384", "--streams", "4"], _env(env))["scratch"]
    assert out["iso"], out
    if out["ok"]:
        assert out["iso_worst"] * max(1, out["iso_queues"]) <= share, out  # every queue charged, inside the share
    else:
        assert out["stage"] in ("stream", "load", "launch"), out
        assert out["iso_queues_refused"] >= 1 or out["stage"] == "load", out
    # room for four: runs, every queue charged, and the device holds what the share allows
    share4 = 4 * worst + 512 * (1 << 20)
    _, env4 = iso.prepare("scr-q4", None, 256, share4, host_process=True)
    before = _run([probe], _env({}))["free"]
    holder = subprocess.Popen([str(probe), "--scratch", "1", "--blocks", "16384", "--streams", "4", "--hold-ms", "20000"],
                              env=_env(env4), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        first = json.loads(holder.stdout.readline())
        sc = first["scratch"]
        assert sc["ok"] is True and sc["iso_queues"] >= 1 and sc["iso_queues_refused"] == 0, first
        assert sc["iso_worst"] * max(1, sc["iso_queues"]) <= share4, first
        during = _run([probe], _env({}))["free"]
    finally:
        holder.kill()
        holder.wait(30)
    assert before - during <= share4 + 512 * (1 << 20), (before, during, share4)


def test_copies_of_a_confined_process_run_on_its_masked_queues(iso):
    """VERDICT r3 item 4 ("blit queues"): a confined PyTorch process's host<->device and device->device copies
    complete, and every queue the runtime created for it got the pod's CU mask (device->device copies are HIP blit
    kernels on those queues; host<->device copies use the SDMA engines: profiles/r04_blit/)."""
    _, env = iso.prepare("copies", CUPartitioner(256, 8).allocate("copies", 64), 256, 16 * GIB, host_process=True)
    code = (
        "import ctypes,json,os,torch\n"
        "x=torch.randn(16<<20).pin_memory(); a=x.to('cuda',non_blocking=True); b=a.clone(); c=torch.empty_like(a)\n"
        "c.copy_(b); y=c.to('cpu'); torch.cuda.synchronize()\n"
        "st=(ctypes.c_uint64*5)(); ctypes.CDLL(os.environ['HSA_TOOLS_LIB']).gsx_isolate_stats(st)\n"
        "print(json.dumps({'queues':st[0],'masked':st[1],'ok':bool(torch.equal(x,y))}))\n")
    out = _run([sys.executable, "-c", code], _env(env), timeout=300)
    assert out["ok"] and out["queues"] >= 1 and out["masked"] >= out["queues"], out
