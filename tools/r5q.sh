#!/bin/bash
# round-5 final: smoke, rocprofv3 kernel trace + PMC passes of the driver's own
# bench invocation (--steps 20 --warmup 5), the calibration kernel, 100k trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5f
mkdir -p $O
export TMPDIR=/tmp
step() { # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local st=$?
  echo "$name exit $st"
  [ $st -eq 0 ] || { tail -5 "$O/$name.log"; exit $st; }
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu
step calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib_fetch -o run -- ./tools/pmc_calib
step calib_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/calib_write -o run -- ./tools/pmc_calib
step prof100k 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof100k -o run -- python3 bench.py --config 100k --steps 20 --warmup 5 --no-cpu
