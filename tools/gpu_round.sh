#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> bench -> rocprof summary.
# Each GPU step has its own time limit; a fault/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
run() { # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local st=$?
  echo "=== $name exit $st"
  tail -n 30 "gpurun_out/$name.log"
  if fatal $st; then echo "FATAL status $st in $name -- stopping"; exit $st; fi
  return 0
}
STEPS="${STEPS:-smoke pytest bench prof}"
for s in $STEPS; do
  case $s in
    build)  run build 600 python -c "import __graft_entry__ as g; g.build()" ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 900 python -u -m pytest tests -v -m gpu --maxfail=5 -p no:cacheprovider --timeout 600 --timeout-method thread ;;
    bench)  run bench 600 python bench.py ;;
    benchdrv) for i in 1 2; do run benchdrv_$i 600 python bench.py --steps 20 --warmup 5; done ;;
    benchq)  run benchq 600 python bench.py --steps 200 --no-cpu ;;
    tailab) for t in 0 1; do SWMM5_TAIL=$t run bench_tail$t 600 python bench.py --steps 200 --no-cpu; SWMM5_TAIL=$t run bench100k_tail$t 600 python bench.py --config 100k --steps 400 --no-cpu; done ;;
    bench100k) run bench100k 600 python bench.py --config 100k --steps 400 --no-cpu ;;
    benchall) for c in 100k 1m_fixed 1m_quality; do run bench_$c 600 python bench.py --config $c --no-cpu; done ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu ${BARGS:-} ;;
    benchqual) run benchqual 600 python bench.py --config 1m_quality --steps 200 --no-cpu ;;
    bench4m) run bench4m 900 python bench.py --config 4m --steps 100 ;;
    mrehearse4m) run mrehearse4m 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config 4m --steps 10 --warmup 2 --spinup 20 --exchange host --no-cpu ;;
    prof100k) run prof100k 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof100k -o run -- python3 bench.py --config 100k --steps 200 --no-cpu ;;
    probe)  run probe 120 ./tools/outfall_latency ;;
    mrehearse) run mrehearse 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --grid 120 --spinup 50 --exchange host --no-cpu ;;
    tsparse) run tsparse 900 python -u -m pytest tests/test_gpu_vs_oracle.py -x -v -p no:cacheprovider --timeout 400 --timeout-method thread -k "${TK:-frozen or sparse or regime_window_707}" ;;
    tipc) run tipc 900 python -u -m pytest tests/test_multigpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "${TKM:-ipc}" ;;
    ipc2) for x in ${XS:-ipc host}; do run ipc2_$x 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-2} --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py --gpus ${NP:-2} --config ${CFG:-1m_surcharge} --steps ${BSTEPS:-20} --warmup 5 --spinup ${SPIN:-200} --exchange $x --no-cpu --no-stream --kernel-reps 0; done ;;
    sig) # per-iteration exchange cost: a tiny launch-bound grid on one rank, then on two ranks of this GPU
         SWMM5_SPARSE=3 run sig_1 300 python bench.py --grid ${SGRID:-24} --spinup 0 --steps 400 --warmup 20 --no-cpu --no-stream --kernel-reps 0
         for x in ${XS:-ipc host}; do
           run sig_2_$x 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29400 + RANDOM % 100)) bench.py --gpus 2 --grid ${SGRID:-24} --spinup 0 --steps 400 --warmup 20 --exchange $x --no-cpu --no-stream --kernel-reps 0
         done ;;
    trace2) # kernel traces of both ranks of a small 2-rank IPC run (tools/mrank_launch.py: one rocprofv3 per rank)
           rm -rf gpurun_out/trace2 && run trace2 300 python tools/mrank_launch.py --np 2 --prof gpurun_out/trace2 -- bench.py --gpus 2 --grid ${SGRID:-24} --spinup 0 --steps 100 --warmup 10 --exchange ${XCH:-ipc} --no-cpu --no-stream --kernel-reps 0 --timing-steps 2 ;;
    sigq) # the 2-rank IPC run on this one GPU with fewer hardware queues per process
           for q in ${HWQ:-1 2}; do
             GPU_MAX_HW_QUEUES=$q run sigq_$q 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29400 + RANDOM % 100)) bench.py --gpus 2 --grid ${SGRID:-24} --spinup 0 --steps 400 --warmup 20 --exchange ${XCH:-ipc} --no-cpu --no-stream --kernel-reps 0
           done ;;
    sigx) # fused (k_ipc_xchg) against split (k_ipc_pack + k_ipc_unpack) exchanges, 2 ranks on this GPU
           for f in 1 0; do
             SWMM5_XCHG_FUSED=$f GPU_MAX_HW_QUEUES=${HWQ:-2} run sigx_$f 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29400 + RANDOM % 100)) bench.py --gpus 2 --grid ${SGRID:-24} --spinup 0 --steps 400 --warmup 20 --exchange ipc --no-cpu --no-stream --kernel-reps 0
           done ;;
    ablib) # the same bench against older builds of the engine (ab/*.so via SWMM5_LIB), interleaved
           for rep in 1 2; do for l in ${ABLIBS:-r05 head}; do
             SWMM5_LIB=$PWD/ab/libswmm5_$l.so run ablib_${l}_$rep 300 python bench.py --no-cpu --kernel-reps 0 ${BARGS:---steps 20 --warmup 5}
           done; done ;;
    sigprobe) # the IPC signalling alone (tools/ipc_signal_probe.hip): two ranks on two streams of one
           # process, then two processes on this one device
           for g in ${SGRAN:-22624}; do run sigprobe_thread_$g 60 ./tools/ipc_signal_probe thread $g || break; done \
           && rm -rf gpurun_out/sigp && mkdir -p gpurun_out/sigp \
           && run sigprobe_proc 120 bash -c './tools/ipc_signal_probe proc 0 gpurun_out/sigp > gpurun_out/sigprobe_p0.txt 2>&1 & ./tools/ipc_signal_probe proc 1 gpurun_out/sigp > gpurun_out/sigprobe_p1.txt 2>&1; s1=$?; wait $!; s0=$?; cat gpurun_out/sigprobe_p0.txt gpurun_out/sigprobe_p1.txt; exit $((s0 | s1))' ;;
    rcclprobe) # the captured RCCL call pattern on one rank (tools/rccl_capture_probe.cpp), phase by phase,
           # bootstrap on the loopback interface and, for comparison, on RCCL's own interface choice
           # (graphs destroyed before the communicator); TEARDOWN=comm: the round-5 order
           for n in ${PREPS:-2 8 16}; do
             NCCL_SOCKET_IFNAME=lo NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,BOOTSTRAP run rcclprobe_lo_$n 90 ./tools/rccl_capture_probe $n ${TEARDOWN:-graphs}
             NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,BOOTSTRAP run rcclprobe_auto_$n 90 ./tools/rccl_capture_probe $n ${TEARDOWN:-graphs}
           done ;;
    rcclteardown) # the round-5 teardown order alone, bounded (expected to hang in ncclCommDestroy)
           NCCL_SOCKET_IFNAME=lo NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT run rcclprobe_commfirst 60 ./tools/rccl_capture_probe 2 comm ;;
    calib) # partition weights from one GPU (tools/calibrate_partition.py) -> profiles/partition_weights.json
           for spec in ${CALS:-4m:2 1m_surcharge:2 1m_surcharge:4 1m_surcharge:8}; do
             run calib_${spec/:/_} 600 python tools/calibrate_partition.py --config ${spec%%:*} --gpus ${spec##*:}
           done
           cp profiles/partition_weights.json gpurun_out/ ;;
    balance) # the 2-rank 4M rehearsal on this GPU: equal strips against weighted blocks (per_rank_sparse_work)
           for bal in ${BALS:-off auto}; do
             run balance_$bal 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-2} --master-addr 127.0.0.1 --master-port $((29700 + RANDOM % 200)) bench.py --gpus ${NP:-2} --config ${CFG:-4m} --steps 10 --warmup 2 --timing-steps 4 --exchange ${XCH:-ipc} --balance $bal --no-cpu --no-stream --kernel-reps 0
           done ;;
    blocks) # the 2-rank 4M rehearsal with node blocks dealt in turn (shared nodes freeze since round 6)
           for b in ${PBLOCKS:-22624 90496}; do
             SWMM5_PART_BLOCK=$b run balance_block_$b 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29700 + RANDOM % 200)) bench.py --gpus 2 --config ${CFG:-4m} --steps 10 --warmup 2 --timing-steps 4 --exchange ${XCH:-ipc} --balance off --no-cpu --no-stream --kernel-reps 0
           done ;;
    tmulti) run tmulti 900 python -u -m pytest tests/test_multigpu.py -x -v -p no:cacheprovider --timeout 600 --timeout-method thread -m gpu -k "${TKM:-write_one_gpu or rccl}" ;;
    rccl1) for c in ${RCFGS:-1m_surcharge 4m}; do run rccl1_$c 600 python bench.py --config $c --rccl-1rank --no-cpu --kernel-reps 0 --steps 100 && run plain1_$c 600 python bench.py --config $c --no-cpu --kernel-reps 0 --steps 100; done ;;
    tk) run tk 900 python -u -m pytest tests -x -v -p no:cacheprovider -m gpu --timeout 400 --timeout-method thread -k "${TK:-exfil}" ;;
    traj) run traj 900 python tools/regime_traj.py ${QS:-0.15 0.2 0.25} ;;
    trajrows) for r in ${TROWS:-1414 2828}; do ROWS=$r TRAJ_FROM=${TFROM:-600} TRAJ_STEPS=${T4_STEPS:-1100} TRAJ_EVERY=50 run trajrows_$r 900 python tools/regime_traj.py ${QS4:-0.12}; done ;;
    traj4m) GRID=1414 TRAJ_FROM=0 TRAJ_STEPS=${T4_STEPS:-1500} TRAJ_EVERY=100 run traj4m 900 python tools/regime_traj.py ${QS4:-0.12} ;;
    lgrid) for g in ${LGRIDS:-0.25 0.5 1 2}; do SWMM5_SPARSE=3 SWMM5_NODE_LIST_GRID=$g run lgrid_$g 300 python bench.py --config ${CFG:-1m_surcharge} --no-cpu --kernel-reps 0 --steps 100 ${BARGS:-}; done ;;
    lprobe) SWMM5_SPARSE=3 SWMM5_PROBE=1 run lprobe 300 python bench.py --config ${CFG:-1m_surcharge} --no-cpu --kernel-reps 0 --steps 50 ;;
    envab) # ENVS="A=1,B=2 C=3": one bench per comma-joined env set
           i=0; for e in ${ENVS}; do i=$((i+1)); run envab_$i 300 env ${e//,/ } python bench.py --config ${CFG:-1m_surcharge} --no-cpu --kernel-reps 0 ${BARGS:-}; done ;;
    matrix) # MATRIX="cfg:A=1,B=2 cfg2: ...": one bench per entry (config, comma-joined env set)
           i=0; for m in ${MATRIX}; do i=$((i+1)); c=${m%%:*}; e=${m#*:}; run matrix_${i}_$c 300 env ${e//,/ } X_=1 python bench.py --config $c --no-cpu --kernel-reps 0 ${BARGS:-}; done ;;
    sparseab)for s in ${SPARSES:-2 0}; do SWMM5_SPARSE=$s run bench_sparse$s 400 python bench.py --config ${CFG:-1m_surcharge} --no-cpu --kernel-reps 0 ${BARGS:-}; done ;;
    regime)for q in ${QS:-0.1 0.2 0.3 0.5 1.0}; do for su in ${SPINUPS:-400}; do run regime_q${q}_s${su} 300 python bench.py --q $q --spinup $su --steps 50 --warmup 5 --timing-steps 5 --kernel-reps 0 --no-cpu; done; done ;;
    gsweep)for g in ${GFACTORS:-0.34 0.67 2}; do SWMM5_GRID_FACTOR=$g run gsweep_$g 300 python bench.py --no-cpu; done ;;
    nsweep) for g in ${NFACTORS:-1 2 3}; do SWMM5_NODE_GRID_FACTOR=$g run nsweep_$g 300 python bench.py --no-cpu; done ;;
    sweep)  for w in 1 3 4 5; do SWMM5_LINK_WAVES=$w run sweep_w$w 300 python bench.py --steps 200 --no-cpu; done ;;
    pmc)    run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --no-cpu ${BARGS:-} \
              && run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --no-cpu ${BARGS:-} ;;
    mrank) # the driver's multi-GPU invocation rehearsed on this one GPU (default config, weak scaling)
           for n in ${NPS:-2 4}; do
             GPU_MAX_HW_QUEUES=${HWQ:-2} run mrank_$n 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29800 + RANDOM % 100)) bench.py --gpus $n ${BARGS:---steps 20 --warmup 5} --no-cpu
           done ;;
    pmcskip) # k_step_end byte attribution: FETCH/WRITE passes per SWMM5_STEPEND_SKIP mask
           for m in ${SKIPS:-0 1 2 4 8 16 32 64}; do
             SWMM5_STEPEND_SKIP=$m run pmcskip_f_$m 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcskip_f_$m -o run -- python3 bench.py --no-cpu --steps 30 --warmup 5 --timing-steps 2 --kernel-reps 0 \
             && SWMM5_STEPEND_SKIP=$m run pmcskip_w_$m 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcskip_w_$m -o run -- python3 bench.py --no-cpu --steps 30 --warmup 5 --timing-steps 2 --kernel-reps 0; done ;;
    pmccal) run calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_fetch -o run -- ./tools/pmc_calib \
              && run calib_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib_write -o run -- ./tools/pmc_calib ;;
    sq)     run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu ;;
  esac
done
