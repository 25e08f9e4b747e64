#!/bin/bash
# round-5 session M: barrier probe (fixed ping-pong), compact vs list per-iteration times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/barrier_probe > gpurun_out/barrier_probe_v2.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/barrier_probe_v2.txt; exit 1; }
echo "probe ok"
for s in 3 5; do
SWMM5_SPARSE=$s timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/cmp_$s.log 2>&1 || { echo "s$s failed"; exit 1; }
echo "sparse $s ok"
done
