#!/bin/bash
# round-5 session Y: list walks without the shared index parts -- bitwise + A/B against sharing everywhere
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/aby
timeout -k 10 300 python -u tools/ab_grid.py ab/lib_before.so stormwater-management-model_amd/libswmm5_mi355x.so > gpurun_out/aby/grid.log 2>&1 || { echo "grid A/B failed"; tail -5 gpurun_out/aby/grid.log; exit 1; }
tail -2 gpurun_out/aby/grid.log
for r in walknoshare shareall walknoshare shareall; do
  if [ $r = shareall ]; then export SWMM5_LIB=$PWD/ab/lib_share_all.so; else unset SWMM5_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/aby/b_$r.log 2>&1 || { echo "bench $r failed"; tail -3 gpurun_out/aby/b_$r.log; exit 1; }
  python3 -c "
import json; l=[x for x in open('gpurun_out/aby/b_$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$r', d['ms_per_step'], r['per_iteration'][0]['k_link_us'], r['per_iteration'][1]['k_link_us'], [x['k_link_us'] for x in r['per_iteration'][2:]])"
done
