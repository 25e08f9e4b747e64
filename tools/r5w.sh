#!/bin/bash
# round-5 session W: bench.py's multi-rank path with 4 ranks (host transport, one GPU), small grid,
# and the default-preset weak-scaling spin-up logic with 2 ranks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 10 --warmup 2 --grid 120 --spinup 50 --exchange host --no-cpu --no-stream --kernel-reps 0 > gpurun_out/mrehearse4.log 2>&1 || { echo "4-rank failed"; tail -20 gpurun_out/mrehearse4.log; exit 1; }
grep '^{' gpurun_out/mrehearse4.log | tail -1 | cut -c1-900
