#!/bin/bash
# round-5 final bench lines: the driver's invocation, then the other presets
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5u
mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo "driver bench failed"; tail -5 $O/bench_driver.log; exit 1; }
echo "driver bench ok"
for c in 100k 1m_fixed 1m_quality 4m; do
  timeout -k 10 600 python3 bench.py --config $c --no-cpu > $O/bench_$c.log 2>&1 || { echo "$c failed"; tail -5 $O/bench_$c.log; exit 1; }
  echo "$c ok"
done
