#!/bin/bash
# round-5 session HH: eight-rank rehearsal of the partitioned path on the one GPU
# of a test box (host transport: RCCL refuses several ranks on one device),
# weak scaling (1m_surcharge strips) and strong scaling (4m)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
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
