#!/bin/bash
# round-5 session K: k_step_end order (SWMM5_END_REV) A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/endrev_check.py > gpurun_out/endrev_check.log 2>&1 || { echo "check failed"; tail -5 gpurun_out/endrev_check.log; exit 1; }
tail -1 gpurun_out/endrev_check.log
for r in 0 1 0 1; do
SWMM5_END_REV=$r timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/er_$r.log 2>&1 || { echo "r$r failed"; exit 1; }
python3 -c "
import json; l=[x for x in open('gpurun_out/er_$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; o=r['other_kernels']
print('rev $r', d['ms_per_step'], r['per_iteration'][0]['k_link_us'], r['per_iteration'][0]['k_node_us'], o['k_step_end+k_finalize'])"
done
