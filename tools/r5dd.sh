#!/bin/bash
# round-5 session DD: k_node_list claim exchange issued with the flag load -- bitwise A/B + timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abdd
mkdir -p $O
timeout -k 10 300 python -u tools/ab_grid.py ab/lib_prev.so stormwater-management-model_amd/libswmm5_mi355x.so > $O/grid.log 2>&1 || { echo "grid A/B failed"; tail -5 $O/grid.log; exit 1; }
tail -2 $O/grid.log
CASES="grid12 grid12_var_qual grid10_surcharge example example_var example_storage_var example_regulators example_shapes example_shapes_var example_culverts_var example_irregular_var example_branches_var example_dummy_var example_exfil_var example_slot_pond example_options example_tidal_var"
for L in before after; do
  lib=ab/lib_prev.so; [ $L = after ] && lib=stormwater-management-model_amd/libswmm5_mi355x.so
  timeout -k 10 300 python -u tools/ab_bitwise.py $lib $O/$L $CASES > $O/golden_$L.log 2>&1 || { echo "golden $L failed"; tail -3 $O/golden_$L.log; exit 1; }
done
n=0; for c in $CASES; do cmp -s $O/before/$c.out $O/after/$c.out && n=$((n+1)) || echo "$c .out DIFFERS"; done; echo "$n identical .out files"
for r in after before after before; do
  if [ $r = before ]; then export SWMM5_LIB=$PWD/ab/lib_prev.so; else unset SWMM5_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > $O/b_$r.log 2>&1 || { echo "bench $r failed"; exit 1; }
  python3 -c "
import json; l=[x for x in open('$O/b_$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$r', d['ms_per_step'], r['per_iteration'][0]['k_link_us'], r['per_iteration'][1]['k_link_us'], [x['k_link_us'] for x in r['per_iteration'][2:4]], [x['k_node_us'] for x in r['per_iteration'][2:8]])"
done
