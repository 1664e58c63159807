#!/bin/bash
# Fake-device rehearsal on the GPU box's CPUs (no GPU use): N in $NS (default "1 8"), printing the
# per-route busy time of the fake apiserver and the CPU seconds of every control-plane process.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-fp}
out=gpurun_out/$tag
mkdir -p "$out"
if [ "${REAL:-0}" = 1 ]; then
  timeout -k 10 300 python bench.py --json-out "$out/real_1.json" > "$out/real_1.log" 2>&1; rc=$?
  echo "real GPU N=1 rc=$rc"; tail -1 "$out/real_1.log" | cut -c1-600; [ $rc -eq 0 ] || exit $rc
fi
for n in ${NS:-1 8}; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 400)) bench.py --gpus $n --steps 50 --warmup 10 --devices fake \
    --json-out "$out/fake_$n.json" > "$out/fake_$n.log" 2>&1; rc=$?
  echo "fake N=$n rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/fake_$n.log"; exit $rc; }
  python - "$out/fake_$n.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["value"], d["ms_per_step"], d["wave_ms"], "p50 bind", d["p50_bind_latency_ms"], d["cpu_s"])
a = d.get("apiserver") or {}
print("apiserver busy ms", a.get("busy_ms"), "max_iter", a.get("max_iter_ms"))
for k, v in sorted((a.get("route_ms") or {}).items(), key=lambda x: -x[1][1])[:8]:
    print("  ", k, v, round(1000 * v[1] / max(v[0], 1), 1), "us/op")
print("node agent", d.get("node_agent"))
PY
done
