#!/bin/bash
# Round-5 GPU-box sessions, one named function each (formerly tools/r5<x>.sh).
# They produced the round-5 records under profiles/ and the measurements in
# DESIGN.md sections 4-6; kept so that each record names the command behind it.
#   usage: bash tools/round5_sessions.sh <session> [<session> ...]
#   (bash tools/round5_sessions.sh list  prints the names)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"

# ---- compact-graph-tests (was tools/r5a.sh)
s_compact_graph_tests() {
# round-5 session A: compact graph bitwise tests, bench A/B, envelope parity
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_vs_oracle.py -x -v -s -p no:cacheprovider --timeout 500 --timeout-method thread -k "frozen_junctions_bitwise or sparse_tail_bitwise_1m" > gpurun_out/t_compact.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 > gpurun_out/b_compact.log 2>&1 || exit $?
SWMM5_COMPACT=0 timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 > gpurun_out/b_list.log 2>&1 || exit $?
SWMM5_PROBE=1 timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --steps 50 > gpurun_out/b_cprobe.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_report.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "shapes or irregular or culverts or streets or branches or dummy" > gpurun_out/t_env.log 2>&1
echo "env tests exit $?"
timeout -k 10 600 python -u -m pytest tests/test_multigpu.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "write_error or write_one_gpu" > gpurun_out/t_mgpu.log 2>&1
echo "mgpu tests exit $?"
}

# ---- compact-two-round-ab (was tools/r5b.sh)
s_compact_two_round_ab() {
# round-5 session B: compact graph (two-round kernels) bitwise + bench A/B; envelope case
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vs_oracle.py -x -v -s -p no:cacheprovider --timeout 500 --timeout-method thread -k "frozen_junctions_bitwise or sparse_tail_bitwise_1m" > gpurun_out/t_compact.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 > gpurun_out/b_compact.log 2>&1 || exit $?
SWMM5_COMPACT=0 timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --no-stream > gpurun_out/b_list.log 2>&1 || exit $?
SWMM5_PROBE=1 timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --steps 50 --no-stream > gpurun_out/b_cprobe.log 2>&1 || exit $?
true
echo "env exit $?"
}

# ---- steady-fixtures (was tools/r5c.sh)
s_steady_fixtures() {
# round-5 session C: SKIP_STEADY_STATE fixtures, envelope window rule, bench sanity
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stats.py tests/test_gpu_report.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "steady or example_shapes_var or example_var or grid10_surcharge" > gpurun_out/t_steady.log 2>&1
echo "steady tests exit $?"
timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --no-stream > gpurun_out/b_default.log 2>&1
echo "bench exit $?"
}

# ---- r4-vs-r5-ab (was tools/r5d.sh)
s_r4_vs_r5_ab() {
# round-5 session D: same-box A/B of the round-4 library against the current one; envelope case
mkdir -p gpurun_out
for i in 1 2; do
  SWMM5_LIB=$PWD/ab/libswmm5_r4.so timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --no-stream > gpurun_out/ab_r4_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 --no-stream > gpurun_out/ab_r5_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "example_shapes_var" > gpurun_out/t_env.log 2>&1
echo "env exit $?"
}

# ---- list-graph-partition (was tools/r5e.sh)
s_list_graph_partition() {
# round-5 session E: list graph under partition (host transport), envelope case, weak-scaling regimes
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_multigpu.py -v -s -p no:cacheprovider --timeout 600 --timeout-method thread -m gpu -k "list_graph or match_one_gpu_bitwise" > gpurun_out/t_mlist.log 2>&1
echo "mgpu list exit $?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "example_shapes_var" > gpurun_out/t_env.log 2>&1
echo "env exit $?"
for r in 1414 2828 5656; do
  ROWS=$r TRAJ_FROM=500 TRAJ_STEPS=1200 TRAJ_EVERY=50 timeout -k 10 600 python tools/regime_traj.py 0.12 > gpurun_out/traj_rows$r.log 2>&1 || exit $?
done
}

# ---- suite-and-4m-rehearsal (was tools/r5f.sh)
s_suite_and_4m_rehearsal() {
# round-5 session F: full GPU suite; 2-rank 4M host rehearsal (per-rank sparse work)
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
echo "suite exit $?"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config 4m --steps 10 --warmup 2 --timing-steps 3 --exchange host --no-cpu --no-stream --kernel-reps 0 > gpurun_out/mrehearse4m.log 2>&1
echo "rehearse exit $?"
}

# ---- interleaved-partition (was tools/r5g.sh)
s_interleaved_partition() {
# round-5 session G: interleaved partition (bitwise + 4M two-rank balance); branches envelope
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_multigpu.py -v -s -p no:cacheprovider --timeout 600 --timeout-method thread -m gpu -k "list_graph" > gpurun_out/t_mlist2.log 2>&1
echo "mgpu list exit $?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "example_branches or example_shapes" > gpurun_out/t_env2.log 2>&1
echo "env exit $?"
for b in 22624 5656; do
SWMM5_PART_BLOCK=$b timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config 4m --steps 10 --warmup 2 --timing-steps 3 --exchange host --no-cpu --no-stream --kernel-reps 0 > gpurun_out/mrehearse4m_b$b.log 2>&1
echo "rehearse $b exit $?"
done
}

# ---- list-graph-regulators (was tools/r5h.sh)
s_list_graph_regulators() {
# round-5 session H: list graph for networks with pumps / regulators
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vs_oracle.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "regulators" > gpurun_out/t_listreg.log 2>&1 || { echo "listreg failed"; exit 1; }
echo "listreg ok"
timeout -k 10 900 python -u -m pytest tests/test_multigpu.py -v -s -p no:cacheprovider --timeout 600 --timeout-method thread -m gpu -k "regulators or list_graph" > gpurun_out/t_mreg.log 2>&1 || { echo "mreg failed"; exit 1; }
echo "mreg ok"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stats.py tests/test_gpu_report.py -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "regulators" > gpurun_out/t_regpar.log 2>&1
echo "regpar exit $?"
}

# ---- rccl-one-rank (was tools/r5i.sh)
s_rccl_one_rank() {
# round-5 session I: RCCL one-rank leg against the plain run, same (list) graph
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/rccl_plain.log 2>&1 || { echo "plain failed"; exit 1; }
echo "plain ok"
timeout -k 10 400 python -u bench.py --rccl-1rank --no-cpu --no-stream --kernel-reps 0 > gpurun_out/rccl_1rank.log 2>&1 || { echo "rccl failed"; exit 1; }
echo "rccl ok"
timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/rccl_plain2.log 2>&1
echo "plain2 exit $?"
}

# ---- link-waves-ab (was tools/r5j.sh)
s_link_waves_ab() {
# round-5 session J: k_link occupancy hint 3 vs 4 (fast variant, 1m_surcharge)
mkdir -p gpurun_out
for w in 3 4 3 4; do
SWMM5_LINK_WAVES=$w timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 20 > gpurun_out/lw_$w.log 2>&1 || { echo "w$w failed"; exit 1; }
python3 -c "
import json; l=[x for x in open('gpurun_out/lw_$w.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('waves $w', d['ms_per_step'], r['per_iteration'][0]['k_link_us'], r['per_iteration'][1]['k_link_us'], {k:v for k,v in r['other_kernels'].items() if 'k_link' in k})"
done
}

# ---- stepend-order-ab (was tools/r5k.sh)
s_stepend_order_ab() {
# round-5 session K: k_step_end order (SWMM5_END_REV) A/B
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/endrev_check.py > gpurun_out/endrev_check.log 2>&1 || { echo "check failed"; tail -5 gpurun_out/endrev_check.log; exit 1; }
tail -1 gpurun_out/endrev_check.log
for r in 0 1 0 1; do
SWMM5_END_REV=$r timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/er_$r.log 2>&1 || { echo "r$r failed"; exit 1; }
python3 -c "
import json; l=[x for x in open('gpurun_out/er_$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; o=r['other_kernels']
print('rev $r', d['ms_per_step'], r['per_iteration'][0]['k_link_us'], r['per_iteration'][0]['k_node_us'], o['k_step_end+k_finalize'])"
done
}

# ---- barrier-probe (was tools/r5m.sh)
s_barrier_probe() {
# round-5 session M: barrier probe (fixed ping-pong), compact vs list per-iteration times
mkdir -p gpurun_out
timeout -k 10 120 ./tools/barrier_probe > gpurun_out/barrier_probe_v2.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/barrier_probe_v2.txt; exit 1; }
echo "probe ok"
for s in 3 5; do
SWMM5_SPARSE=$s timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/cmp_$s.log 2>&1 || { echo "s$s failed"; exit 1; }
echo "sparse $s ok"
done
}

# ---- node-list-preload-ab (was tools/r5n.sh)
s_node_list_preload_ab() {
# round-5 session N: k_node_list with preloaded node inputs (SWMM5_NODE_PRE) -- bitwise + A/B
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ab_env_bitwise.py SWMM5_NODE_PRE 0 1 SWMM5_SPARSE=3 > gpurun_out/npre_check.log 2>&1 || { echo "check failed"; tail -5 gpurun_out/npre_check.log; exit 1; }
tail -1 gpurun_out/npre_check.log
for r in 0 1 0 1; do
SWMM5_NODE_PRE=$r timeout -k 10 400 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > gpurun_out/np_$r.log 2>&1 || { echo "r$r failed"; exit 1; }
python3 -c "
import json; l=[x for x in open('gpurun_out/np_$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('pre $r', d['ms_per_step'], [x['k_node_us'] for x in r['per_iteration'][2:]])"
done
}

# ---- full-suite (was tools/r5p.sh)
s_full_suite() {
# round-5 final: the full GPU suite on the final source
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05_pytest_gpu.log 2>&1
st=$?
tail -3 gpurun_out/r05_pytest_gpu.log
grep -E "FAILED|ERROR" gpurun_out/r05_pytest_gpu.log | head -20
exit $st
}

# ---- final-profile (was tools/r5q.sh)
s_final_profile() {
# round-5 final: smoke, rocprofv3 kernel trace + PMC passes of the driver's own
# bench invocation (--steps 20 --warmup 5), the calibration kernel, 100k trace
O=gpurun_out/r5f
mkdir -p $O
export TMPDIR=/tmp
step() { # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local st=$?
  echo "$name exit $st"
  [ $st -eq 0 ] || { tail -5 "$O/$name.log"; exit $st; }
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu
step calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib_fetch -o run -- ./tools/pmc_calib
step calib_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/calib_write -o run -- ./tools/pmc_calib
step prof100k 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof100k -o run -- python3 bench.py --config 100k --steps 20 --warmup 5 --no-cpu
}

# ---- list-graph-networks (was tools/r5r.sh)
s_list_graph_networks() {
# round-5 session R: list graph over more networks (+ quality unfreeze fold); 1m_quality A/B vs previous timing
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_vs_oracle.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "list_graph_bitwise or fused_quality or config3" > gpurun_out/t_lgnet.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/t_lgnet.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/t_lgnet.log | tail -2
for c in 1m_quality 1m_surcharge; do
timeout -k 10 400 python -u bench.py --config $c --no-cpu --no-stream --kernel-reps 0 > gpurun_out/q_$c.log 2>&1 || { echo "$c failed"; exit 1; }
python3 -c "
import json; l=[x for x in open('gpurun_out/q_$c.log') if x.startswith('{')][-1]; d=json.loads(l); print('$c', d['ms_per_step'], d['config']['step_graphs'])"
done
}

# ---- final-profile-and-suite (was tools/r5s.sh)
s_final_profile_and_suite() {
# round-5 final evidence in one call: the profile session (tools/r5q.sh), then the full GPU suite
( s_final_profile ) || exit $?
timeout -k 10 840 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05_pytest_gpu.log 2>&1
st=$?
tail -3 gpurun_out/r05_pytest_gpu.log
grep -E "FAILED|ERROR" gpurun_out/r05_pytest_gpu.log | head -20
exit $st
}

# ---- tail-grid-100k (was tools/r5t.sh)
s_tail_grid_100k() {
# round-5 session T: k_tail grid at 100k (its launch exits at once when steps converge at iteration 1)
mkdir -p gpurun_out
for g in 0 16 64 0 16 64; do
  if [ $g -eq 0 ]; then unset SWMM5_TAIL_GRID; else export SWMM5_TAIL_GRID=$g; fi
  timeout -k 10 300 python -u bench.py --config 100k --no-cpu --no-stream --kernel-reps 0 --steps 400 > gpurun_out/tg_$g.log 2>&1 || { echo "g$g failed"; exit 1; }
  python3 -c "
import json; l=[x for x in open('gpurun_out/tg_$g.log') if x.startswith('{')][-1]; d=json.loads(l); print('tailgrid $g', d['ms_per_step'], d['value']/1e9, d['config']['step_graphs'])"
done
}

# ---- final-bench-lines (was tools/r5u.sh)
s_final_bench_lines() {
# round-5 final bench lines: the driver's invocation, then the other presets
O=gpurun_out/r5u
mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { echo "driver bench failed"; tail -5 $O/bench_driver.log; exit 1; }
echo "driver bench ok"
for c in 100k 1m_fixed 1m_quality 4m; do
  timeout -k 10 600 python3 bench.py --config $c --no-cpu > $O/bench_$c.log 2>&1 || { echo "$c failed"; tail -5 $O/bench_$c.log; exit 1; }
  echo "$c ok"
done
}

# ---- quality-pmc (was tools/r5v.sh)
s_quality_pmc() {
# round-5 session V: PMC bytes of the 1m_quality step (k_qual_node)
O=gpurun_out/r5v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --config 1m_quality --steps 20 --warmup 5 --no-cpu > $O/pmc_fetch.log 2>&1 || { echo "fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --config 1m_quality --steps 20 --warmup 5 --no-cpu > $O/pmc_write.log 2>&1 || { echo "write failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config 1m_quality --steps 20 --warmup 5 --no-cpu > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo ok
}

# ---- rehearsal-4-ranks (was tools/r5w.sh)
s_rehearsal_4_ranks() {
# round-5 session W: bench.py's multi-rank path with 4 ranks (host transport, one GPU), small grid,
# and the default-preset weak-scaling spin-up logic with 2 ranks
mkdir -p gpurun_out
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 10 --warmup 2 --grid 120 --spinup 50 --exchange host --no-cpu --no-stream --kernel-reps 0 > gpurun_out/mrehearse4.log 2>&1 || { echo "4-rank failed"; tail -20 gpurun_out/mrehearse4.log; exit 1; }
grep '^{' gpurun_out/mrehearse4.log | tail -1 | cut -c1-900
}

# ---- shared-index-ab (was tools/r5x.sh)
s_shared_index_ab() {
# round-5 session X: shared circular index parts in the conduit update -- A/B against the previous build
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
}

# ---- walks-unshared-ab (was tools/r5y.sh)
s_walks_unshared_ab() {
# round-5 session Y: list walks without the shared index parts -- bitwise + A/B against sharing everywhere
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
}

# ---- final-quality-and-bench (was tools/r5z.sh)
s_final_quality_and_bench() {
# round-5 final (after the shared circular index change): 1m_quality profile + PMC, then the bench lines
( s_quality_pmc ) || exit $?
( s_final_bench_lines ) || exit $?
}

# ---- recip-pairs-ab (was tools/r5aa.sh)
s_recip_pairs_ab() {
# round-5 session AA: shared reciprocal pairs for the momentum divisions -- bitwise A/B + timing
O=gpurun_out/abaa
mkdir -p $O
timeout -k 10 300 python -u tools/ab_grid.py ab/lib_shared.so stormwater-management-model_amd/libswmm5_mi355x.so > $O/grid.log 2>&1 || { echo "grid A/B failed"; tail -5 $O/grid.log; exit 1; }
tail -2 $O/grid.log
CASES="grid12 grid12_var_qual grid10_surcharge example example_var example_storage_var example_regulators example_shapes example_shapes_var example_culverts_var example_irregular_var example_branches_var example_dummy_var example_exfil_var example_slot_pond example_options example_tidal_var"
for L in before after; do
  lib=ab/lib_shared.so; [ $L = after ] && lib=stormwater-management-model_amd/libswmm5_mi355x.so
  timeout -k 10 300 python -u tools/ab_bitwise.py $lib $O/$L $CASES > $O/golden_$L.log 2>&1 || { echo "golden $L failed"; tail -3 $O/golden_$L.log; exit 1; }
done
n=0; for c in $CASES; do cmp -s $O/before/$c.out $O/after/$c.out && n=$((n+1)) || echo "$c .out DIFFERS"; done; echo "$n identical .out files"
for r in after before after before; do
  if [ $r = before ]; then export SWMM5_LIB=$PWD/ab/lib_shared.so; else unset SWMM5_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-stream --kernel-reps 0 > $O/b_$r.log 2>&1 || { echo "bench $r failed"; exit 1; }
  python3 -c "
import json; l=[x for x in open('$O/b_$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$r', d['ms_per_step'], r['per_iteration'][0]['k_link_us'], r['per_iteration'][1]['k_link_us'], [x['k_link_us'] for x in r['per_iteration'][2:4]])"
done
}

# ---- finalize-partials-ab (was tools/r5bb.sh)
s_finalize_partials_ab() {
# round-5 session BB: finalize partial loads in one round -- bitwise A/B + timing
O=gpurun_out/abbb
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
print('$r', d['ms_per_step'], r['other_kernels']['k_step_end+k_finalize'])"
done
}

# ---- rare-link-ab (was tools/r5cc.sh)
s_rare_link_ab() {
# round-5 session CC: rare link arrays behind one pointer -- bitwise A/B + timing
O=gpurun_out/abcc
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
print('$r', d['ms_per_step'], r['per_iteration'][0]['k_link_us'], r['per_iteration'][1]['k_link_us'], [x['k_link_us'] for x in r['per_iteration'][2:4]])"
done
}

# ---- claim-with-flag-ab (was tools/r5dd.sh)
s_claim_with_flag_ab() {
# round-5 session DD: k_node_list claim exchange issued with the flag load -- bitwise A/B + timing
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
}

# ---- unfreeze-in-stepend-ab (was tools/r5ee.sh)
s_unfreeze_in_stepend_ab() {
# round-5 session EE: frozen junctions' final depths in the step end / k_finalize
# (no k_unfreeze launch) -- bitwise A/B, focused GPU tests, timing
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
}

# ---- driver-window-trace (was tools/r5ff.sh)
s_driver_window_trace() {
# round-5 session FF: kernel trace of the driver's invocation, this build and the previous one
O=gpurun_out/abff
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_after -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-stream > $O/after.log 2>&1 || { echo "after failed"; tail -5 $O/after.log; exit 1; }
export SWMM5_LIB=$PWD/ab/lib_prev.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_before -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-stream > $O/before.log 2>&1 || { echo "before failed"; tail -5 $O/before.log; exit 1; }
echo done
}

# ---- node-three-waves-ab (was tools/r5gg.sh)
s_node_three_waves_ab() {
# round-5 session GG: node kernels (k_node, k_node_list) at three waves per SIMD -- bitwise A/B + timing
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
}

# ---- rehearsal-8-ranks (was tools/r5hh.sh)
s_rehearsal_8_ranks() {
# round-5 session HH: eight-rank rehearsal of the partitioned path on the one GPU
# of a test box (host transport: RCCL refuses several ranks on one device),
# weak scaling (1m_surcharge strips) and strong scaling (4m)
O=gpurun_out/r5hh
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while sleep 20; do date >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 8 --exchange host --spinup 200 --steps 5 --warmup 2 --no-cpu --no-stream --kernel-reps 0 > $O/weak8.log 2>&1 || { echo "weak8 failed"; tail -20 $O/weak8.log; exit 1; }
grep '^{' $O/weak8.log | tail -1 | cut -c1-900
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 8 --config 4m --exchange host --spinup 200 --steps 5 --warmup 2 --no-cpu --no-stream --kernel-reps 0 > $O/strong8.log 2>&1 || { echo "strong8 failed"; tail -20 $O/strong8.log; exit 1; }
grep '^{' $O/strong8.log | tail -1 | cut -c1-900
}

# ---- final-evidence (was tools/r5final.sh)
s_final_evidence() {
# round-5 final evidence, one call: profile + PMC + suite (r5s), then quality profile + bench lines (r5z)
( s_final_profile_and_suite ) || exit $?
( s_final_quality_and_bench ) || exit $?
}

if [ "$1" = list ] || [ $# -eq 0 ]; then
  echo "compact-graph-tests compact-two-round-ab steady-fixtures r4-vs-r5-ab list-graph-partition suite-and-4m-rehearsal interleaved-partition list-graph-regulators rccl-one-rank link-waves-ab stepend-order-ab barrier-probe node-list-preload-ab full-suite final-profile list-graph-networks final-profile-and-suite tail-grid-100k final-bench-lines quality-pmc rehearsal-4-ranks shared-index-ab walks-unshared-ab final-quality-and-bench recip-pairs-ab finalize-partials-ab rare-link-ab claim-with-flag-ab unfreeze-in-stepend-ab driver-window-trace node-three-waves-ab rehearsal-8-ranks final-evidence"
  exit 0
fi
for s in "$@"; do
  f="s_${s//-/_}"
  declare -F "$f" > /dev/null || { echo "unknown session $s"; exit 2; }
  ( "$f" ) || exit $?
done
