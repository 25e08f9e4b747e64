#!/bin/bash
# round-5 final: the full GPU suite on the final source
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05_pytest_gpu.log 2>&1
st=$?
tail -3 gpurun_out/r05_pytest_gpu.log
grep -E "FAILED|ERROR" gpurun_out/r05_pytest_gpu.log | head -20
exit $st
