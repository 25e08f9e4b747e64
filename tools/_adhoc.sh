cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/latency_probe > gpurun_out/latency.log 2>&1; echo "latency exit $?"; cat gpurun_out/latency.log
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 500 --timeout-method thread -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?"
tail -3 gpurun_out/pytest_gpu.log
b() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 $BARGS > gpurun_out/b_$tag.log 2>&1 || { echo "FAIL $tag"; exit 1; }
  tail -1 gpurun_out/b_$tag.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); o=b['roofline']['other_kernels']; print('$tag', b['value'], b['ms_per_step'], [(x['k_link_us'],x['k_node_us']) for x in b['roofline']['per_iteration']], o['k_step_end+k_finalize'], o.get('k_qual_node+k_qual_link'))"
}
b scan SWMM5_TAIL=0
b ng1 SWMM5_TAIL=0 SWMM5_NODE_GRID_FACTOR=1
BARGS="--config 1m_quality"
b qual X=1
BARGS="--config 100k --steps 400"
b k100 X=1
