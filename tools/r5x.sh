#!/bin/bash
# round-5 session X: shared circular index parts in the conduit update -- A/B against the previous build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abx
timeout -k 10 300 python -u tools/ab_grid.py ab/lib_before.so stormwater-management-model_amd/libswmm5_mi355x.so > gpurun_out/abx/grid.log 2>&1 || { echo "grid A/B failed"; tail -5 gpurun_out/abx/grid.log; exit 1; }
cat gpurun_out/abx/grid.log | tail -2
for L in before after; do
  lib=ab/lib_before.so; [ $L = after ] && lib=stormwater-management-model_amd/libswmm5_mi355x.so
  timeout -k 10 200 python -u tools/ab_bitwise.py $lib gpurun_out/abx/$L grid12 grid12_var_qual grid10_surcharge > gpurun_out/abx/golden_$L.log 2>&1 || { echo "golden $L failed"; exit 1; }
done
for c in grid12 grid12_var_qual grid10_surcharge; do cmp gpurun_out/abx/before/$c.out gpurun_out/abx/after/$c.out && echo "$c .out identical"; done
for r in after before after before; do
  if [ $r = before ]; then export SWMM5_LIB=$PWD/ab/lib_before.so; else unset SWMM5_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/abx/b_$r.log 2>&1 || { echo "bench $r failed"; tail -3 gpurun_out/abx/b_$r.log; exit 1; }
  python3 -c "
import json; l=[x for x in open('gpurun_out/abx/b_$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$r', d['ms_per_step'], r['per_iteration'][0]['k_link_us'], r['per_iteration'][1]['k_link_us'], [x['k_link_us'] for x in r['per_iteration'][2:4]])"
done
