"""Builds every native component of the framework in-tree.

Targets (outputs land in ``gpushare_scheduler_extender_amd/_native/``):

* ``engine``  – C++17 ledger/JSON engine, reflectors + controller, pybind11 module ``_engine``.
* ``schedsim`` – ``gsx-schedsim``, the compiled kube-scheduler stand-in used by the benchmark.
* ``nodeagent`` – ``gsx-nodeagent``, the compiled kubelet / device-plugin Allocate / runtime stand-in.
* ``fakeapi`` – ``gsx-fakeapi``, the compiled fake kube-apiserver.
* ``mxdev``   – C++17 amdsmi device library + pybind11 module ``_mxdev``
                (amdsmi is dlopen'ed with RTLD_DEEPBIND at run time so the
                module also loads on hosts without a GPU and never binds to the
                ROCm-SMI copy bundled inside the torch wheel).
* ``kernels`` – HIP/CDNA4 kernels for gfx950 (``libgsx_kernels.so``): CU probe,
                HBM touch/verify, bf16 MFMA GEMM workload, CU-masked streams.
* ``tools``   – standalone HIP executables (``gsx-cuprobe``, ``gsx-memprobe``).
* ``isolate`` – ``libgsx_isolate.so``, the HSA tools library that enforces a pod's CU partition and HBM share
                inside every HIP/HSA process of the pod, plus its host-only test driver (fake HSA runtime).
* ``asan``    – host-only sanitizer build of the engine unit test.

Usage: ``python native/build.py [targets...] [--force] [-v]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
NATIVE = ROOT / "native"
OUT = ROOT / "gpushare_scheduler_extender_amd" / "_native"
OBJ = ROOT / "build" / "obj"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("GSX_OFFLOAD_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter", "-fvisibility=hidden"]


def _pybind_includes() -> list[str]:
    import pybind11  # noqa: PLC0415

    return ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _newer(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _current(out: Path, srcs: list[Path], headers: list[Path], force: bool) -> bool:
    """``out`` is newer than every source and header it is built from: nothing to do, whatever ``build/obj`` holds
    (a tree copied without ``build/`` -- a gpurun snapshot -- must not recompile what it ships built)."""
    return not force and not _newer(out, [*srcs, *headers])


def _run(cmd: list[str], verbose: bool) -> None:
    # an artifact under _native/ is linked to a temporary name and renamed over the old one: a process that has the
    # old library mapped (a test run, a plugin) keeps its inode, instead of reading a file rewritten under it
    final = None
    if "-o" in cmd:
        i = cmd.index("-o") + 1
        if i < len(cmd) and Path(cmd[i]).parent == OUT:
            final = cmd[i]
            cmd = [*cmd[:i], f"{final}.tmp{os.getpid()}", *cmd[i + 1:]]
    if verbose:
        print("+", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        if final:
            Path(f"{final}.tmp{os.getpid()}").unlink(missing_ok=True)
        raise RuntimeError(f"native build failed: {' '.join(cmd[:3])} ... (exit {r.returncode})")
    if final:
        os.replace(f"{final}.tmp{os.getpid()}", final)


def _compile_objs(srcs: list[Path], compiler: str, flags: list[str], tag: str, force: bool, verbose: bool,
                  headers: list[Path]) -> list[Path]:
    OBJ.mkdir(parents=True, exist_ok=True)
    jobs = []
    objs = []
    for s in srcs:
        o = OBJ / f"{tag}_{s.stem}.o"
        objs.append(o)
        if force or _newer(o, [s, *headers]):
            jobs.append([compiler, *flags, "-c", str(s), "-o", str(o)])
    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs))
    return objs


def build_engine(force: bool = False, verbose: bool = False) -> Path:
    src = NATIVE / "engine"
    srcs = sorted(src.glob("*.cc"))
    srcs = [s for s in srcs if s.name not in ("engine_test.cc", "controller_test.cc")]
    headers = sorted(src.glob("*.h"))
    out = OUT / f"_engine{EXT}"
    if _current(out, srcs, headers, force):
        return out
    flags = [*CXXFLAGS, *_pybind_includes(), "-I" + str(src)]
    objs = _compile_objs(srcs, "g++", flags, "engine", force, verbose, headers)
    if force or _newer(out, objs):
        OUT.mkdir(parents=True, exist_ok=True)
        _run(["g++", "-shared", "-o", str(out), *map(str, objs), "-lssl", "-lcrypto", "-lpthread", "-ldl"], verbose)
    return out


def _build_native_tool(name: str, srcdir: str, force: bool, verbose: bool) -> Path:
    """A standalone executable from ``native/<srcdir>/*.cc`` linked with the engine's objects."""
    src = NATIVE / "engine"
    eng = [s for s in sorted(src.glob("*.cc")) if s.name not in ("bindings.cc", "engine_test.cc", "controller_test.cc")]
    headers = sorted(src.glob("*.h"))
    out = OUT / name
    if _current(out, [*eng, *sorted((NATIVE / srcdir).glob("*.cc"))], headers, force):
        return out
    flags = [*CXXFLAGS, "-I" + str(src)]
    objs = _compile_objs(eng, "g++", flags, "tool", force, verbose, headers)
    objs += _compile_objs(sorted((NATIVE / srcdir).glob("*.cc")), "g++", flags, srcdir, force, verbose, headers)
    if force or _newer(out, objs):
        OUT.mkdir(parents=True, exist_ok=True)
        _run(["g++", "-o", str(out), *map(str, objs), "-lssl", "-lcrypto", "-lpthread", "-ldl"], verbose)
    return out


def build_schedsim(force: bool = False, verbose: bool = False) -> Path:
    """``gsx-schedsim``: the compiled kube-scheduler stand-in (reflectors + serial cycle + bind pool)."""
    return _build_native_tool("gsx-schedsim", "schedsim", force, verbose)


def build_nodeagent(force: bool = False, verbose: bool = False) -> Path:
    """``gsx-nodeagent``: the compiled kubelet + device-plugin Allocate + runtime stand-in for one node."""
    return _build_native_tool("gsx-nodeagent", "nodeagent", force, verbose)


def build_fakeapi(force: bool = False, verbose: bool = False) -> Path:
    """``gsx-fakeapi``: the compiled fake kube-apiserver (its asyncio twin is the test fixture tests/fixtures/fakeapi.py)."""
    return _build_native_tool("gsx-fakeapi", "fakeapi", force, verbose)


def build_mxdev(force: bool = False, verbose: bool = False) -> Path:
    src = NATIVE / "mxdev"
    srcs = sorted(src.glob("*.cc"))
    srcs = [s for s in srcs if not s.name.endswith("_test.cc") and not s.name.startswith("fake_")]
    headers = sorted(src.glob("*.h"))
    out = OUT / f"_mxdev{EXT}"
    # the test-only stand-in for libamd_smi.so (a shuffled amdsmi/HIP topology, tests/test_device_topology.py)
    fake = ROOT / "build" / "libfake_amdsmi.so"
    if force or _newer(fake, [src / "fake_amdsmi.cc"]):
        fake.parent.mkdir(parents=True, exist_ok=True)
        _run(["g++", *CXXFLAGS, "-I" + str(ROCM / "include"), "-shared", str(src / "fake_amdsmi.cc"), "-o",
              str(fake)], verbose)
    if _current(out, srcs, [*headers, *sorted((NATIVE / "engine").glob("*.h"))], force):
        return out
    flags = [*CXXFLAGS, *_pybind_includes(), "-I" + str(src), "-I" + str(ROCM / "include"),
             "-I" + str(NATIVE / "engine")]
    objs = _compile_objs(srcs, "g++", flags, "mxdev", force, verbose, headers)
    if force or _newer(out, objs):
        OUT.mkdir(parents=True, exist_ok=True)
        _run(["g++", "-shared", "-o", str(out), *map(str, objs), "-ldl"], verbose)
    return out


def _hipcc() -> str:
    h = ROCM / "bin" / "hipcc"
    return str(h) if h.exists() else (shutil.which("hipcc") or "hipcc")


def build_kernels(force: bool = False, verbose: bool = False) -> Path:
    src = NATIVE / "kernels"
    srcs = sorted(src.glob("*.hip"))
    srcs = [s for s in srcs if not s.stem.startswith("tool_")]
    headers = sorted(src.glob("*.h"))
    out = OUT / "libgsx_kernels.so"
    if _current(out, srcs, headers, force):
        return out
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-I" + str(src),
             "-munsafe-fp-atomics"]
    objs = _compile_objs(srcs, _hipcc(), flags, "kern", force, verbose, headers)
    if force or _newer(out, objs):
        OUT.mkdir(parents=True, exist_ok=True)
        _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(out), *map(str, objs)], verbose)
    return out


def build_tools(force: bool = False, verbose: bool = False) -> list[Path]:
    src = NATIVE / "kernels"
    outs = []
    for s in sorted(src.glob("tool_*.hip")):
        out = OUT / ("gsx-" + s.stem[len("tool_"):])
        deps = [s, *sorted(src.glob("*.h")), *sorted(src.glob("*.hip"))]
        if force or _newer(out, deps):
            OUT.mkdir(parents=True, exist_ok=True)
            others = [str(x) for x in sorted(src.glob("*.hip")) if not x.stem.startswith("tool_")]
            _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-I" + str(src), str(s), *others,
                  "-L" + str(ROCM / "lib"), "-lhsa-runtime64", "-o", str(out)], verbose)
        outs.append(out)
    # the scratch probe's kernels, one code object per private-array size (gsx-memprobe --scratch KIB)
    probe = src / "probes" / "scratch.hip"
    for kib, ints in ((1, 256), (4, 1024), (16, 4096), (64, 16384)):
        out = OUT / f"gsx-scratch-{kib}.hsaco"
        if force or _newer(out, [probe]):
            OUT.mkdir(parents=True, exist_ok=True)
            _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "--genco", f"-DSCRATCH_INTS={ints}",
                  str(probe), "-o", str(out)], verbose)
        outs.append(out)
    return outs


HSA_FLAGS = ["-DAMD_INTERNAL_BUILD", "-I" + str(ROCM / "include"), "-I" + str(ROCM / "include" / "hsa")]


def build_isolate(force: bool = False, verbose: bool = False) -> list[Path]:
    """``libgsx_isolate.so`` (host C++ against the HSA API-table ABI; no HIP, no device code) and
    ``build/isolate_test`` (the library driven through a fake HSA runtime on the CPU)."""
    src = NATIVE / "isolate"
    lib = OUT / "libgsx_isolate.so"
    deps = [src / "gsx_isolate.cc"]
    if force or _newer(lib, deps):
        OUT.mkdir(parents=True, exist_ok=True)
        # loaded into arbitrary container userlands: libc only (no C++ runtime: compiled without exceptions /
        # RTTI / thread-safe statics and linked by the C driver)
        obj = ROOT / "build" / "gsx_isolate.o"
        obj.parent.mkdir(parents=True, exist_ok=True)
        _run(["g++", *CXXFLAGS, *HSA_FLAGS, "-fno-exceptions", "-fno-rtti", "-fno-threadsafe-statics", "-c",
              str(src / "gsx_isolate.cc"), "-o", str(obj)], verbose)
        _run(["gcc", "-shared", str(obj), "-o", str(lib), "-static-libgcc", "-Wl,--exclude-libs,ALL",
              "-Wl,-z,defs", "-lpthread"], verbose)
    test = ROOT / "build" / "isolate_test"
    if force or _newer(test, [src / "isolate_test.cc"]):
        test.parent.mkdir(parents=True, exist_ok=True)
        _run(["g++", "-O1", "-g", "-std=c++17", "-Wall", *HSA_FLAGS, str(src / "isolate_test.cc"), "-o", str(test),
              "-ldl"], verbose)
    return [lib, test]


TEST_MAINS = ("engine_test.cc", "controller_test.cc")


def _host_clang() -> str:
    """ROCm's clang++: its sanitizer runtimes intercept pthread_cond_clockwait, which std::condition_variable
    uses for steady-clock waits on this glibc; GCC 11's libtsan does not and reports false double locks."""
    c = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "lib" / "llvm" / "bin" / "clang++"
    return str(c) if c.exists() else "g++"


def _sanitized(test: str, tag: str, flags: list[str], force: bool, verbose: bool) -> Path:
    """Host-only sanitizer build of one test main against every engine source (not the Python bindings)."""
    src = NATIVE / "engine"
    out = ROOT / "build" / f"{test}_{tag}"
    lib = [s for s in sorted(src.glob("*.cc")) if s.name != "bindings.cc" and s.name not in TEST_MAINS]
    srcs = [*lib, src / f"{test}.cc"]
    if force or _newer(out, srcs + sorted(src.glob("*.h"))):
        out.parent.mkdir(parents=True, exist_ok=True)
        _run([_host_clang(), "-O1", "-g", "-std=c++17", *flags, "-fno-omit-frame-pointer", "-I" + str(src),
              *map(str, srcs), "-o", str(out), "-lssl", "-lcrypto", "-lpthread", "-ldl"], verbose)
    return out


def build_asan(force: bool = False, verbose: bool = False) -> list[Path]:
    """ASan + UBSan builds of the engine unit/stress test and the controller concurrency test."""
    return [_sanitized(t, "asan", ["-fsanitize=address,undefined"], force, verbose)
            for t in ("engine_test", "controller_test")]


def build_tsan(force: bool = False, verbose: bool = False) -> list[Path]:
    """ThreadSanitizer builds of the same tests (epoll loops, bind pool, reflectors, resync, GC, tracker)."""
    return [_sanitized(t, "tsan", ["-fsanitize=thread"], force, verbose) for t in ("engine_test", "controller_test")]


def build_tools_tsan(force: bool = False, verbose: bool = False) -> list[Path]:
    """ThreadSanitizer builds of the compiled stand-ins (``build/gsx-{fakeapi,schedsim,nodeagent}_tsan``);
    ``GSX_NATIVE_TOOLS_SUFFIX=_tsan`` makes gsxtools/cluster.py start these instead of the optimised ones."""
    src = NATIVE / "engine"
    lib = [s for s in sorted(src.glob("*.cc")) if s.name != "bindings.cc" and s.name not in TEST_MAINS]
    outs = []
    for tool in ("fakeapi", "schedsim", "nodeagent"):
        mains = sorted((NATIVE / tool).glob("*.cc"))
        out = ROOT / "build" / f"gsx-{tool}_tsan"
        if force or _newer(out, lib + mains + sorted(src.glob("*.h"))):
            out.parent.mkdir(parents=True, exist_ok=True)
            _run([_host_clang(), "-O1", "-g", "-std=c++17", "-fsanitize=thread", "-fno-omit-frame-pointer",
                  "-I" + str(src), *map(str, lib + mains), "-o", str(out), "-lssl", "-lcrypto", "-lpthread", "-ldl"],
                 verbose)
        outs.append(out)
    return outs


TARGETS = {
    "engine": build_engine,
    "schedsim": build_schedsim,
    "nodeagent": build_nodeagent,
    "fakeapi": build_fakeapi,
    "mxdev": build_mxdev,
    "kernels": build_kernels,
    "tools": build_tools,
    "isolate": build_isolate,
    "asan": build_asan,
    "tsan": build_tsan,
    "tools_tsan": build_tools_tsan,
}
DEFAULT = ["engine", "schedsim", "nodeagent", "fakeapi", "mxdev", "kernels", "tools", "isolate"]


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("targets", nargs="*", default=DEFAULT)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    for t in a.targets:
        r = TARGETS[t](force=a.force, verbose=a.verbose)
        print(f"[native] {t}: {r}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
