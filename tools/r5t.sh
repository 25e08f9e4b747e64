#!/bin/bash
# round-5 session T: k_tail grid at 100k (its launch exits at once when steps converge at iteration 1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for g in 0 16 64 0 16 64; do
  if [ $g -eq 0 ]; then unset SWMM5_TAIL_GRID; else export SWMM5_TAIL_GRID=$g; fi
  timeout -k 10 300 python -u bench.py --config 100k --no-cpu --no-stream --kernel-reps 0 --steps 400 > gpurun_out/tg_$g.log 2>&1 || { echo "g$g failed"; exit 1; }
  python3 -c "
import json; l=[x for x in open('gpurun_out/tg_$g.log') if x.startswith('{')][-1]; d=json.loads(l); print('tailgrid $g', d['ms_per_step'], d['value']/1e9, d['config']['step_graphs'])"
done
