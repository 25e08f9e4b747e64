#!/bin/bash
# round-5 final evidence in one call: the profile session (tools/r5q.sh), then the full GPU suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r5q.sh || exit $?
timeout -k 10 840 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05_pytest_gpu.log 2>&1
st=$?
tail -3 gpurun_out/r05_pytest_gpu.log
grep -E "FAILED|ERROR" gpurun_out/r05_pytest_gpu.log | head -20
exit $st
