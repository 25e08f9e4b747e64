#!/bin/bash
# round-5 session C: SKIP_STEADY_STATE fixtures, envelope window rule, bench sanity
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stats.py tests/test_gpu_report.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "steady or example_shapes_var or example_var or grid10_surcharge" > gpurun_out/t_steady.log 2>&1
echo "steady tests exit $?"
timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --no-stream > gpurun_out/b_default.log 2>&1
echo "bench exit $?"
