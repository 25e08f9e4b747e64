#!/bin/bash
# round-5 session A: compact graph bitwise tests, bench A/B, envelope parity
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_vs_oracle.py -x -v -s -p no:cacheprovider --timeout 500 --timeout-method thread -k "frozen_junctions_bitwise or sparse_tail_bitwise_1m" > gpurun_out/t_compact.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 > gpurun_out/b_compact.log 2>&1 || exit $?
SWMM5_COMPACT=0 timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 > gpurun_out/b_list.log 2>&1 || exit $?
SWMM5_PROBE=1 timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --steps 50 > gpurun_out/b_cprobe.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_report.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "shapes or irregular or culverts or streets or branches or dummy" > gpurun_out/t_env.log 2>&1
echo "env tests exit $?"
timeout -k 10 600 python -u -m pytest tests/test_multigpu.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "write_error or write_one_gpu" > gpurun_out/t_mgpu.log 2>&1
echo "mgpu tests exit $?"
