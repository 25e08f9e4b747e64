#!/bin/bash
# round-5 session E: list graph under partition (host transport), envelope case, weak-scaling regimes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_multigpu.py -v -s -p no:cacheprovider --timeout 600 --timeout-method thread -m gpu -k "list_graph or match_one_gpu_bitwise" > gpurun_out/t_mlist.log 2>&1
echo "mgpu list exit $?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "example_shapes_var" > gpurun_out/t_env.log 2>&1
echo "env exit $?"
for r in 1414 2828 5656; do
  ROWS=$r TRAJ_FROM=500 TRAJ_STEPS=1200 TRAJ_EVERY=50 timeout -k 10 600 python tools/regime_traj.py 0.12 > gpurun_out/traj_rows$r.log 2>&1 || exit $?
done
