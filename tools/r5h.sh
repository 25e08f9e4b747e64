#!/bin/bash
# round-5 session H: list graph for networks with pumps / regulators
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vs_oracle.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "regulators" > gpurun_out/t_listreg.log 2>&1 || { echo "listreg failed"; exit 1; }
echo "listreg ok"
timeout -k 10 900 python -u -m pytest tests/test_multigpu.py -v -s -p no:cacheprovider --timeout 600 --timeout-method thread -m gpu -k "regulators or list_graph" > gpurun_out/t_mreg.log 2>&1 || { echo "mreg failed"; exit 1; }
echo "mreg ok"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stats.py tests/test_gpu_report.py -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "regulators" > gpurun_out/t_regpar.log 2>&1
echo "regpar exit $?"
