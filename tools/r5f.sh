#!/bin/bash
# round-5 session F: full GPU suite; 2-rank 4M host rehearsal (per-rank sparse work)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
echo "suite exit $?"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config 4m --steps 10 --warmup 2 --timing-steps 3 --exchange host --no-cpu --no-stream --kernel-reps 0 > gpurun_out/mrehearse4m.log 2>&1
echo "rehearse exit $?"
