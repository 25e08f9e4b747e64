#!/bin/bash
# round-5 session J: k_link occupancy hint 3 vs 4 (fast variant, 1m_surcharge)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in 3 4 3 4; do
SWMM5_LINK_WAVES=$w timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 20 > gpurun_out/lw_$w.log 2>&1 || { echo "w$w failed"; exit 1; }
python3 -c "
import json; l=[x for x in open('gpurun_out/lw_$w.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('waves $w', d['ms_per_step'], r['per_iteration'][0]['k_link_us'], r['per_iteration'][1]['k_link_us'], {k:v for k,v in r['other_kernels'].items() if 'k_link' in k})"
done
