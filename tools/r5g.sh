#!/bin/bash
# round-5 session G: interleaved partition (bitwise + 4M two-rank balance); branches envelope
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_multigpu.py -v -s -p no:cacheprovider --timeout 600 --timeout-method thread -m gpu -k "list_graph" > gpurun_out/t_mlist2.log 2>&1
echo "mgpu list exit $?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "example_branches or example_shapes" > gpurun_out/t_env2.log 2>&1
echo "env exit $?"
for b in 22624 5656; do
SWMM5_PART_BLOCK=$b timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config 4m --steps 10 --warmup 2 --timing-steps 3 --exchange host --no-cpu --no-stream --kernel-reps 0 > gpurun_out/mrehearse4m_b$b.log 2>&1
echo "rehearse $b exit $?"
done
