#!/bin/bash
# round-5 session V: PMC bytes of the 1m_quality step (k_qual_node)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --config 1m_quality --steps 20 --warmup 5 --no-cpu > $O/pmc_fetch.log 2>&1 || { echo "fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --config 1m_quality --steps 20 --warmup 5 --no-cpu > $O/pmc_write.log 2>&1 || { echo "write failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config 1m_quality --steps 20 --warmup 5 --no-cpu > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo ok
