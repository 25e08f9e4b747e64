#!/bin/bash
# round-5 session FF: kernel trace of the driver's invocation, this build and the previous one
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abff
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_after -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-stream > $O/after.log 2>&1 || { echo "after failed"; tail -5 $O/after.log; exit 1; }
export SWMM5_LIB=$PWD/ab/lib_prev.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_before -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-stream > $O/before.log 2>&1 || { echo "before failed"; tail -5 $O/before.log; exit 1; }
echo done
