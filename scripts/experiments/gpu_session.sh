#!/bin/bash
# One GPU-box session: GPU tests, smoke, the default 1-GPU bench, a rocprofv3 kernel-stats pass over the
# bench (in-process control plane, no child processes under the profiler), then the N=1..8 rehearsal with
# fake devices on the box's CPUs.  Every GPU step has its own time limit; the script stops at the first
# failure.  Usage: scripts/experiments/gpu_session.sh [tag]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-s}
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/gpu_tests.log" 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 "$out/gpu_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 "$out/smoke.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --json-out "$out/bench_n1.json" > "$out/bench_n1.log" 2>&1; rc=$?
echo "bench N=1 rc=$rc"; tail -1 "$out/bench_n1.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o bench -- python3 bench.py --steps 20 --warmup 5 \
  > "$out/prof.log" 2>&1; rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
db=$(find "$out/prof" -name '*.db' | head -n 1)
[ -n "$db" ] && python scripts/rocpd_summary.py "$db" > "$out/kernels.md"
for n in 1 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 50 --warmup 10 --devices fake \
    --json-out "$out/fake_$n.json" > "$out/fake_$n.log" 2>&1; rc=$?
  echo "fake N=$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python - "$out" <<'PY'
import json, sys
o = sys.argv[1]
for f in ["bench_n1"] + [f"fake_{n}" for n in (1, 2, 4, 8)]:
    d = json.load(open(f"{o}/{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["wave_ms"], d["p50_bind_latency_ms"], d.get("cpu_s"))
PY
