#!/bin/bash
# round-5 session R: list graph over more networks (+ quality unfreeze fold); 1m_quality A/B vs previous timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_vs_oracle.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "list_graph_bitwise or fused_quality or config3" > gpurun_out/t_lgnet.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/t_lgnet.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/t_lgnet.log | tail -2
for c in 1m_quality 1m_surcharge; do
timeout -k 10 400 python -u bench.py --config $c --no-cpu --no-stream --kernel-reps 0 > gpurun_out/q_$c.log 2>&1 || { echo "$c failed"; exit 1; }
python3 -c "
import json; l=[x for x in open('gpurun_out/q_$c.log') if x.startswith('{')][-1]; d=json.loads(l); print('$c', d['ms_per_step'], d['config']['step_graphs'])"
done
