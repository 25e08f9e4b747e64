#!/bin/bash
# round-5 session I: RCCL one-rank leg against the plain run, same (list) graph
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/rccl_plain.log 2>&1 || { echo "plain failed"; exit 1; }
echo "plain ok"
timeout -k 10 400 python -u bench.py --rccl-1rank --no-cpu --no-stream --kernel-reps 0 > gpurun_out/rccl_1rank.log 2>&1 || { echo "rccl failed"; exit 1; }
echo "rccl ok"
timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/rccl_plain2.log 2>&1
echo "plain2 exit $?"
