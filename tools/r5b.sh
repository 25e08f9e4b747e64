#!/bin/bash
# round-5 session B: compact graph (two-round kernels) bitwise + bench A/B; envelope case
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vs_oracle.py -x -v -s -p no:cacheprovider --timeout 500 --timeout-method thread -k "frozen_junctions_bitwise or sparse_tail_bitwise_1m" > gpurun_out/t_compact.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 > gpurun_out/b_compact.log 2>&1 || exit $?
SWMM5_COMPACT=0 timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --no-stream > gpurun_out/b_list.log 2>&1 || exit $?
SWMM5_PROBE=1 timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --steps 50 --no-stream > gpurun_out/b_cprobe.log 2>&1 || exit $?
true
echo "env exit $?"
