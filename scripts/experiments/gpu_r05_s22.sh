#!/bin/bash
# Round-5 session 22: the phased GEMM's wrong tiles at 16384x16384x8192 (session 21) -- which shapes, which tiles,
# every launch or some.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_s22}
mkdir -p $OUT
timeout -k 10 500 python scripts/experiments/gemm_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; cat $OUT/probe.jsonl; exit 1; }
cat $OUT/probe.jsonl
