#!/bin/bash
# round-5 session EE: frozen junctions' final depths in the step end / k_finalize
# (no k_unfreeze launch) -- bitwise A/B, focused GPU tests, timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abee
mkdir -p $O
timeout -k 10 300 python -u tools/ab_grid.py ab/lib_prev.so stormwater-management-model_amd/libswmm5_mi355x.so > $O/grid.log 2>&1 || { echo "grid A/B failed"; tail -5 $O/grid.log; exit 1; }
tail -2 $O/grid.log
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_vs_oracle.py -k "unfreeze or frozen_junctions or list_graph or sparse_tail or window_707" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -3 $O/pytest.log
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_multigpu.py tests/test_gpu_stats.py > $O/pytest2.log 2>&1 || { echo "pytest2 failed"; tail -30 $O/pytest2.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -3 $O/pytest2.log
for r in after before after before; do
  if [ $r = before ]; then export SWMM5_LIB=$PWD/ab/lib_prev.so; else unset SWMM5_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > $O/b_$r.log 2>&1 || { echo "bench $r failed"; exit 1; }
  python3 -c "
import json; l=[x for x in open('$O/b_$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$r', d['ms_per_step'], r['other_kernels']['k_step_end+k_finalize']['avg_launch_us'])"
done
