"""Packaging and deployment contracts: the image pins what the tests run with,
the plugin's runtime-built gRPC descriptors work under that protobuf, the manifests wire the device plugin to the
extender (and authenticate it), and the docs do not describe code that is gone."""
import os
import re
import subprocess
import sys
from importlib.metadata import version
from pathlib import Path

import yaml

ROOT = Path(__file__).resolve().parents[1]


def _pins() -> dict:
    text = (ROOT / "deploy" / "Dockerfile").read_text()
    line = next(ln for ln in text.splitlines() if ln.startswith("RUN pip3 install"))
    return dict(tok.split("==", 1) for tok in line.split()[3:])


def test_image_pins_are_the_versions_the_tests_run_with():
    pins = _pins()
    dist = {"aiohttp": "aiohttp", "pyyaml": "PyYAML", "grpcio": "grpcio", "protobuf": "protobuf",
            "prometheus_client": "prometheus_client", "pybind11": "pybind11"}
    assert set(pins) == set(dist), pins
    for pkg, d in dist.items():
        assert pins[pkg] == version(d), (pkg, pins[pkg], version(d))


def test_plugin_descriptors_build_and_round_trip_under_the_pinned_protobuf():
    import google.protobuf

    from gpushare_scheduler_extender_amd.deviceplugin import api

    assert google.protobuf.__version__ == _pins()["protobuf"]
    req = api.AllocateRequest()
    c = req.container_requests.add()
    c.devices_ids.extend(["fake-0001-_-3", "fake-0001-_-4"])
    back = api.AllocateRequest.FromString(req.SerializeToString())
    assert list(back.container_requests[0].devices_ids) == ["fake-0001-_-3", "fake-0001-_-4"]
    resp = api.AllocateResponse()
    cr = resp.container_responses.add()
    cr.envs["HIP_VISIBLE_DEVICES"] = "3"
    cr.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
    assert api.AllocateResponse.FromString(resp.SerializeToString()).container_responses[0].envs[
        "HIP_VISIBLE_DEVICES"] == "3"


def _docs(path: str) -> list:
    return [d for d in yaml.safe_load_all((ROOT / "deploy" / path).read_text()) if d]


def test_device_plugin_manifest_reaches_the_extender_and_the_extender_reviews_its_token():
    ds = next(d for d in _docs("device-plugin-ds.yaml") if d["kind"] == "DaemonSet")
    spec = ds["spec"]["template"]["spec"]
    env = {e["name"]: e.get("value") for e in spec["containers"][0]["env"]}
    assert env.get("GSX_PODRESOURCES_SOCKET") and env.get("GSX_EXTENDER_URL"), env
    assert spec.get("hostNetwork") and spec.get("dnsPolicy") == "ClusterFirstWithHostNet"
    ext = _docs("gpushare-schd-extender.yaml")
    svc = next(d for d in ext if d["kind"] == "Service")
    m = re.match(r"http://([^.]+)\.([^.]+)\.svc:(\d+)$", env["GSX_EXTENDER_URL"])
    assert m and m.group(1) == svc["metadata"]["name"] and m.group(2) == svc["metadata"]["namespace"]
    assert int(m.group(3)) in [p["port"] for p in svc["spec"]["ports"]]
    dep = next(d for d in ext if d["kind"] == "Deployment")
    eenv = {e["name"]: e.get("value") for e in dep["spec"]["template"]["spec"]["containers"][0]["env"]}
    sa = ds["spec"]["template"]["spec"]["serviceAccountName"]
    assert eenv.get("GSX_PLUGIN_AUTH") == "tokenreview"
    assert f"system:serviceaccount:{ds['metadata']['namespace']}:{sa}" in eenv.get("GSX_PLUGIN_USERS", "").split(",")
    role = next(d for d in ext if d["kind"] == "ClusterRole")
    assert any("tokenreviews" in r.get("resources", []) and "create" in r.get("verbs", []) for r in role["rules"])
    # the DaemonSet's CPU request: one core is what the plugin needs (gsxtools/plugincpu.py)
    assert spec["containers"][0]["resources"]["requests"]["cpu"] in ("1", 1)


def test_plugin_refuses_to_reconcile_without_an_extender():
    env = {k: v for k, v in os.environ.items() if k not in ("GSX_EXTENDER_URL", "GSX_NO_EXTENDER")}
    env["PYTHONPATH"] = str(ROOT)
    r = subprocess.run([sys.executable, "-m", "gpushare_scheduler_extender_amd.deviceplugin", "--node", "n1",
                        "--backend", "fake", "--podresources-socket", "/tmp/nonexistent-podresources.sock"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "GSX_EXTENDER_URL" in r.stderr, (r.returncode, r.stderr[-500:])


STALE = ("ExtenderServer.bind", "asyncio fallback", "aiohttp front end", "parallel/workqueue")


def test_docs_do_not_describe_removed_code():
    files = [ROOT / "README.md", *sorted((ROOT / "docs").glob("*.md"))]
    hits = [(f.name, s) for f in files if not f.name.startswith("ROUND") for s in STALE if s in f.read_text()]
    assert not hits, hits
    assert not (ROOT / "gpushare_scheduler_extender_amd" / "parallel").exists()


# phrases code comments must not carry any more: a file that moved, figures re-measured since, behaviour changed
CODE_STALE = ("deviceplugin/agent.py", "idle 0.3 %", "one pod a second 0.7 %", "/opt/gpushare",
              "the extender frees on deletion", "finalise graceful deletes on their own timer")


def test_code_comments_do_not_describe_removed_code():
    """the doc-drift check covers code comments and manifests too."""
    exts = {".py", ".cc", ".h", ".hip", ".yaml", ".sh", ".md"}
    roots = [ROOT / d for d in ("native", "gpushare_scheduler_extender_amd", "gsxtools", "deploy", "samples", "docs")]
    files = [f for r in roots for f in r.rglob("*") if f.suffix in exts and f.is_file()] + [ROOT / "bench.py"]
    hits = [(str(f.relative_to(ROOT)), s) for f in files for s in CODE_STALE if s in f.read_text(errors="replace")]
    assert not hits, hits


def _dockerfile_copies(dockerfile: Path) -> tuple[list[tuple[list[str], str]], list[str]]:
    """(COPY sources -> destination) and RUN commands of a Dockerfile, in order (continuation lines joined)."""
    lines, cur = [], ""
    for raw in dockerfile.read_text().splitlines():
        s = raw.strip()
        if not s or s.startswith("#"):
            continue
        cur = f"{cur} {s[:-1]}" if s.endswith("\\") else f"{cur} {s}"
        if not s.endswith("\\"):
            lines.append(cur.strip())
            cur = ""
    copies, runs = [], []
    for ln in lines:
        op, _, rest = ln.partition(" ")
        if op == "COPY":
            *src, dst = rest.split()
            copies.append((src, dst))
        elif op == "RUN":
            runs.append(rest)
    return copies, runs


def test_sample_workload_image_is_self_contained(tmp_path):
    """the sample image's file set, assembled exactly as its Dockerfile does (its COPY lines, and its
    hipcc RUN line cross-compiling the MFMA GEMM for gfx950), runs ``main.py --help`` from there with nothing of the
    repository on the path; ``run.sh`` is the entry and passes its arguments on."""
    df = ROOT / "samples" / "workload" / "Dockerfile"
    copies, runs = _dockerfile_copies(df)
    text = df.read_text()
    assert "ARG BASE=rocm/pytorch:rocm" in text and ":latest" not in text  # a pinned base
    assert 'ENTRYPOINT ["/app/run.sh"]' in text

    def here(p: str) -> Path:  # an image path under the temp root
        return tmp_path / p.lstrip("/")
    for srcs, dst in copies:
        for s in srcs:
            target = here(dst) / Path(s).name if dst.endswith("/") else here(dst)
            target.parent.mkdir(parents=True, exist_ok=True)
            target.write_bytes((ROOT / s).read_bytes())
            target.chmod((ROOT / s).stat().st_mode)
    (hip,) = [r for r in runs if r.startswith("hipcc")]
    cmd = hip.split("&&")[0].replace("${GPU_ARCH}", "gfx950").replace("/build", str(here("build"))).replace(
        "/app", str(here("app")))
    r = subprocess.run(cmd, shell=True, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (here("app") / "libgsx_kernels.so").stat().st_size > 0
    env = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH", "GSX_KERNELS_LIB")}
    app = here("app")
    assert sorted(p.name for p in app.iterdir()) == ["libgsx_kernels.so", "main.py", "run.sh"]
    out = subprocess.run(["bash", str(app / "run.sh"), "--help"], capture_output=True, text=True, cwd=str(tmp_path),
                         env={**env, "GSX_APP_DIR": str(app)}, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "GEMM loop inside the pod's GPU share" in out.stdout and "--probe-limit" in out.stdout
    # the library the image built is the one main.py finds
    probe = ("import sys; sys.argv = ['x']; import runpy; m = runpy.run_path(sys.argv[0] if False else "
             f"'{app / 'main.py'}', run_name='probe'); print(m['kernels_lib_path']())")
    got = subprocess.run([sys.executable, "-c", probe], capture_output=True, text=True, cwd=str(tmp_path), env=env,
                         timeout=120)
    assert got.stdout.strip() == str(app / "libgsx_kernels.so"), got.stderr[-1000:]
