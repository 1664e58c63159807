"""ctypes binding of ``libgsx_kernels.so`` (native/kernels/gsx_kernels.hip).

No silent fallback: on a host with a GPU every call goes to the HIP code,
and a missing library raises with the command that builds it.  Callers that
must also run on CPU-only hosts check :func:`gpu_available` first.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

_LIB = None
_LOCK = threading.Lock()
SO = Path(__file__).resolve().parents[1] / "_native" / "libgsx_kernels.so"


class HipError(RuntimeError):
    pass


class DevInfo(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 64), ("arch", ctypes.c_char * 32), ("pci_bus_id", ctypes.c_char * 32),
                ("total_mem", ctypes.c_uint64), ("cu_count", ctypes.c_int32), ("xcc_count", ctypes.c_int32),
                ("clock_khz", ctypes.c_int32), ("wave_size", ctypes.c_int32), ("lds_per_block", ctypes.c_uint64)]


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        if not SO.exists():
            if os.environ.get("GSX_AUTOBUILD", "1") == "1":
                from ..utils.build import build_native  # noqa: PLC0415

                build_native(["kernels"])
            if not SO.exists():
                raise ImportError(f"{SO} missing; run `python native/build.py kernels`")
        L = ctypes.CDLL(str(SO))
        vp, u32p, u64, i32 = ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint64, ctypes.c_int
        sig = {
            "gsx_last_error": ([], ctypes.c_char_p),
            "gsx_device_count": ([ctypes.POINTER(i32)], i32),
            "gsx_device_info": ([i32, ctypes.POINTER(DevInfo)], i32),
            "gsx_mem_info": ([i32, ctypes.POINTER(u64), ctypes.POINTER(u64)], i32),
            "gsx_synchronize": ([i32], i32),
            "gsx_stream_create": ([i32, u32p, i32, ctypes.POINTER(vp)], i32),
            "gsx_stream_get_mask": ([vp, u32p, i32], i32),
            "gsx_stream_destroy": ([vp], i32),
            "gsx_stream_sync": ([vp], i32),
            "gsx_malloc": ([i32, u64, ctypes.POINTER(vp)], i32),
            "gsx_free": ([vp], i32),
            "gsx_memcpy_d2h": ([vp, vp, u64], i32),
            "gsx_memcpy_h2d": ([vp, vp, u64], i32),
            "gsx_cuprobe": ([vp, i32, i32, u32p], i32),
            "gsx_hbm_stamp": ([vp, vp, u64, u64, u64], i32),
            "gsx_hbm_verify": ([vp, vp, u64, u64, u64, ctypes.POINTER(u64)], i32),
            "gsx_hbm_fill": ([vp, vp, u64, ctypes.c_uint32], i32),
            "gsx_gemm_bf16_nt": ([vp, vp, vp, vp, i32, i32, i32], i32),
            "gsx_event_time_gemm": ([vp, vp, vp, vp, i32, i32, i32, i32, ctypes.POINTER(ctypes.c_float)], i32),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _LIB = L
    return _LIB


def _ck(rc: int, what: str):
    if rc != 0:
        raise HipError(f"{what}: {lib().gsx_last_error().decode(errors='replace')}")


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().gsx_device_count(ctypes.byref(n))
    if rc != 0:
        return 0
    return n.value


def gpu_available() -> bool:
    try:
        return device_count() > 0
    except (OSError, ImportError):
        return False


def device_info(dev: int) -> dict:
    d = DevInfo()
    _ck(lib().gsx_device_info(dev, ctypes.byref(d)), "device_info")
    return {"name": d.name.decode(), "arch": d.arch.decode(), "pci_bus_id": d.pci_bus_id.decode(),
            "total_mem": d.total_mem, "cu_count": d.cu_count, "clock_khz": d.clock_khz,
            "wave_size": d.wave_size, "lds_per_block": d.lds_per_block}


def mem_info(dev: int) -> tuple[int, int]:
    f, t = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _ck(lib().gsx_mem_info(dev, ctypes.byref(f), ctypes.byref(t)), "mem_info")
    return f.value, t.value


def synchronize(dev: int):
    _ck(lib().gsx_synchronize(dev), "synchronize")


def mask_words(cus: list[int] | range, total_cus: int = 256) -> list[int]:
    words = [0] * ((total_cus + 31) // 32)
    for c in cus:
        if not 0 <= c < total_cus:
            raise ValueError(f"CU {c} out of range 0..{total_cus - 1}")
        words[c // 32] |= 1 << (c % 32)
    return words


class Stream:
    """A HIP stream, optionally restricted to a CU mask (hipExtStreamCreateWithCUMask)."""

    def __init__(self, dev: int = 0, cu_mask: list[int] | None = None):
        self.dev = dev
        self.handle = ctypes.c_void_p()
        if cu_mask:
            arr = (ctypes.c_uint32 * len(cu_mask))(*cu_mask)
            _ck(lib().gsx_stream_create(dev, arr, len(cu_mask), ctypes.byref(self.handle)), "stream_create(cu_mask)")
        else:
            _ck(lib().gsx_stream_create(dev, None, 0, ctypes.byref(self.handle)), "stream_create")

    def mask(self, words: int = 8) -> list[int]:
        arr = (ctypes.c_uint32 * words)()
        _ck(lib().gsx_stream_get_mask(self.handle, arr, words), "stream_get_mask")
        return list(arr)

    def sync(self):
        _ck(lib().gsx_stream_sync(self.handle), "stream_sync")

    def destroy(self):
        if self.handle:
            lib().gsx_stream_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    @property
    def ptr(self) -> int:
        return self.handle.value or 0


class DeviceBuffer:
    def __init__(self, dev: int, nbytes: int):
        self.dev = dev
        self.nbytes = int(nbytes)
        self.ptr = ctypes.c_void_p()
        _ck(lib().gsx_malloc(dev, self.nbytes, ctypes.byref(self.ptr)), f"malloc({self.nbytes})")

    def free(self):
        if self.ptr:
            lib().gsx_free(self.ptr)
            self.ptr = ctypes.c_void_p()

    def addr(self, offset: int = 0) -> int:
        return (self.ptr.value or 0) + offset

    def to_host(self, nbytes: int | None = None, offset: int = 0) -> bytes:
        n = self.nbytes - offset if nbytes is None else nbytes
        buf = ctypes.create_string_buffer(n)
        _ck(lib().gsx_memcpy_d2h(buf, ctypes.c_void_p(self.addr(offset)), n), "memcpy_d2h")
        return buf.raw

    def from_host(self, data: bytes, offset: int = 0):
        _ck(lib().gsx_memcpy_h2d(ctypes.c_void_p(self.addr(offset)), data, len(data)), "memcpy_h2d")


def cuprobe(stream: Stream, blocks: int = 4096, spin: int = 20000) -> list[tuple[int, int]]:
    out = (ctypes.c_uint32 * (2 * blocks))()
    _ck(lib().gsx_cuprobe(stream.handle, blocks, spin, out), "cuprobe")
    return [(out[2 * i], out[2 * i + 1] & 0x7FFFFFFF) for i in range(blocks)]


def decode_hw_id(hw: int, xcc: int) -> dict:
    """gfx9 HW_REG_HW_ID fields (WAVE, SIMD, PIPE, CU, SH, SE, TG, VM, QUEUE, STATE, ME)."""
    return {"wave": hw & 0xF, "simd": (hw >> 4) & 0x3, "pipe": (hw >> 6) & 0x3, "cu": (hw >> 8) & 0xF,
            "sh": (hw >> 12) & 0x1, "se": (hw >> 13) & 0x7, "tg": (hw >> 16) & 0xF, "vm": (hw >> 20) & 0xF,
            "queue": (hw >> 24) & 0x7, "xcc": xcc & 0xF}


def physical_cus(records: list[tuple[int, int]]) -> set[tuple[int, int, int, int]]:
    out = set()
    for hw, xcc in records:
        d = decode_hw_id(hw, xcc)
        out.add((d["xcc"], d["se"], d["sh"], d["cu"]))
    return out


def hbm_stamp(stream: Stream, addr: int, nbytes: int, stride: int, tag: int):
    _ck(lib().gsx_hbm_stamp(stream.handle, ctypes.c_void_p(addr), nbytes, stride, tag & 0xFFFFFFFFFFFFFFFF),
        "hbm_stamp")


def hbm_verify(stream: Stream, addr: int, nbytes: int, stride: int, tag: int) -> int:
    bad = ctypes.c_uint64(0)
    _ck(lib().gsx_hbm_verify(stream.handle, ctypes.c_void_p(addr), nbytes, stride, tag & 0xFFFFFFFFFFFFFFFF,
                             ctypes.byref(bad)), "hbm_verify")
    return bad.value


def hbm_fill(stream: Stream, addr: int, nbytes: int, pattern: int = 0):
    _ck(lib().gsx_hbm_fill(stream.handle, ctypes.c_void_p(addr), nbytes, pattern & 0xFFFFFFFF), "hbm_fill")


def gemm_bf16_nt(stream: Stream, a: int, b: int, c: int, m: int, n: int, k: int):
    _ck(lib().gsx_gemm_bf16_nt(stream.handle, ctypes.c_void_p(a), ctypes.c_void_p(b), ctypes.c_void_p(c), m, n, k),
        "gemm_bf16_nt")


def time_gemm(stream: Stream, a: int, b: int, c: int, m: int, n: int, k: int, iters: int) -> float:
    ms = ctypes.c_float(0)
    _ck(lib().gsx_event_time_gemm(stream.handle, ctypes.c_void_p(a), ctypes.c_void_p(b), ctypes.c_void_p(c),
                                  m, n, k, iters, ctypes.byref(ms)), "time_gemm")
    return ms.value


class Slice(ctypes.Structure):
    _fields_ = [("addr", ctypes.c_uint64), ("bytes", ctypes.c_uint64), ("tag", ctypes.c_uint64)]


def hbm_admit(stream: Stream, slices: list[tuple[int, int, int]], stamp_idx: int, stride: int) -> int:
    """Stamp slice ``stamp_idx`` (or none with -1) and verify all ``(addr, bytes, tag)`` slices in one launch."""
    L = lib()
    if not getattr(L, "_admit_sig", False):
        L.gsx_hbm_admit.argtypes = [ctypes.c_void_p, ctypes.POINTER(Slice), ctypes.c_int, ctypes.c_int,
                                    ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.gsx_hbm_admit.restype = ctypes.c_int
        L._admit_sig = True
    arr = (Slice * max(1, len(slices)))(*[Slice(a, b, t & 0xFFFFFFFFFFFFFFFF) for a, b, t in slices])
    bad = ctypes.c_uint64(0)
    _ck(L.gsx_hbm_admit(stream.handle, arr, len(slices), stamp_idx, stride, ctypes.byref(bad)), "hbm_admit")
    return bad.value


def hbm_admit_n(stream: Stream, slices: list[tuple[int, int, int]], n_stamp: int, stride: int,
                verify: bool = True) -> int:
    """Stamp the first ``n_stamp`` ``(addr, bytes, tag)`` extents, then verify all of them; one stream sync."""
    L = lib()
    if not getattr(L, "_admit_n_sig", False):
        L.gsx_hbm_admit_n.argtypes = [ctypes.c_void_p, ctypes.POINTER(Slice), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.gsx_hbm_admit_n.restype = ctypes.c_int
        L._admit_n_sig = True
    arr = (Slice * max(1, len(slices)))(*[Slice(a, b, t & 0xFFFFFFFFFFFFFFFF) for a, b, t in slices])
    bad = ctypes.c_uint64(0)
    _ck(L.gsx_hbm_admit_n(stream.handle, arr, len(slices), n_stamp, int(verify), stride, ctypes.byref(bad)),
        "hbm_admit_n")
    return bad.value


GEMM_CFGS = {0: "128x128/4w", 1: "256x128/8w", 2: "128x256/8w", 3: "256x256/8w", 4: "128x128/4w-nogroup",
             5: "256x256/8w-phased-g4", 6: "256x256/8w-phased-g8", 7: "256x256/4w-agpr-g4", 8: "256x256/4w-agpr-g8",
             9: "256x256/4w-asm-agpr-g4", 10: "256x256/8w-phased-g4-mfma32"}


def gemm_bf16_nt_cfg(stream: Stream, a: int, b: int, c: int, m: int, n: int, k: int, cfg: int):
    """Launch one tile configuration of the templated GEMM (native/kernels/gemm.hip)."""
    L = lib()
    if not getattr(L, "_cfg_sig", False):
        L.gsx_gemm_bf16_nt_launch_cfg.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 4
        L.gsx_gemm_bf16_nt_launch_cfg.restype = ctypes.c_int
        L.gsx_gemm_cfg_tile.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.gsx_gemm_cfg_tile.restype = ctypes.c_int
        L._cfg_sig = True
    bm, bn = ctypes.c_int(0), ctypes.c_int(0)
    if L.gsx_gemm_cfg_tile(cfg, ctypes.byref(bm), ctypes.byref(bn)) != 0:
        raise HipError(f"unknown GEMM config {cfg}")
    if m % bm.value or n % bn.value or k % 64:
        raise HipError(f"GEMM config {cfg} needs M%{bm.value}==0, N%{bn.value}==0, K%64==0")
    rc = L.gsx_gemm_bf16_nt_launch_cfg(stream.handle, ctypes.c_void_p(a), ctypes.c_void_p(b), ctypes.c_void_p(c),
                                       m, n, k, cfg)
    if rc != 0:
        raise HipError(f"gemm cfg {cfg}: hip error {rc}")
