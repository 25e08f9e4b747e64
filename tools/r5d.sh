#!/bin/bash
# round-5 session D: same-box A/B of the round-4 library against the current one; envelope case
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  SWMM5_LIB=$PWD/ab/libswmm5_r4.so timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --no-stream > gpurun_out/ab_r4_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --no-stream > gpurun_out/ab_r5_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "example_shapes_var" > gpurun_out/t_env.log 2>&1
echo "env exit $?"
