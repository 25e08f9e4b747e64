#!/bin/bash
# round-5 session GG: node kernels (k_node, k_node_list) at three waves per SIMD -- bitwise A/B + timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abgg
mkdir -p $O
timeout -k 10 300 python -u tools/ab_grid.py ab/lib_prev.so stormwater-management-model_amd/libswmm5_mi355x.so > $O/grid.log 2>&1 || { echo "grid A/B failed"; tail -5 $O/grid.log; exit 1; }
tail -2 $O/grid.log
for r in after before after before; do
  if [ $r = before ]; then export SWMM5_LIB=$PWD/ab/lib_prev.so; else unset SWMM5_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-stream --kernel-reps 0 ${BENCH_ARGS} > $O/b_$r.log 2>&1 || { echo "bench $r failed"; exit 1; }
  python3 -c "
import json; l=[x for x in open('$O/b_$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$r', d['ms_per_step'], [x['k_node_us'] for x in r['per_iteration']], r['other_kernels']['k_step_end+k_finalize']['avg_launch_us'])"
done
