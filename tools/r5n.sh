#!/bin/bash
# round-5 session N: k_node_list with preloaded node inputs (SWMM5_NODE_PRE) -- bitwise + A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ab_env_bitwise.py SWMM5_NODE_PRE 0 1 SWMM5_SPARSE=3 > gpurun_out/npre_check.log 2>&1 || { echo "check failed"; tail -5 gpurun_out/npre_check.log; exit 1; }
tail -1 gpurun_out/npre_check.log
for r in 0 1 0 1; do
SWMM5_NODE_PRE=$r timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/np_$r.log 2>&1 || { echo "r$r failed"; exit 1; }
python3 -c "
import json; l=[x for x in open('gpurun_out/np_$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('pre $r', d['ms_per_step'], [x['k_node_us'] for x in r['per_iteration'][2:]])"
done
