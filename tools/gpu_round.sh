#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> bench -> rocprof summary.
# Each GPU step has its own time limit; a fault/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
run() { # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local st=$?
  echo "=== $name exit $st"
  tail -n 30 "gpurun_out/$name.log"
  if fatal $st; then echo "FATAL status $st in $name -- stopping"; exit $st; fi
  return 0
}
STEPS="${STEPS:-smoke pytest bench prof}"
for s in $STEPS; do
  case $s in
    build)  run build 600 python -c "import __graft_entry__ as g; g.build()" ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 1200 python -m pytest tests -x -q -m gpu ;;
    bench)  run bench 600 python bench.py ;;
    bench100k) run bench100k 600 python bench.py --grid 224 --steps 400 --no-cpu ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --no-cpu ;;
  esac
done
