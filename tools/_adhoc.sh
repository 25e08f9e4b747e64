cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "dummy" > gpurun_out/pt_dummy.log 2>&1; echo "pytest exit $?"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_dummy.log | tail -8
b() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 $BARGS > gpurun_out/b_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/b_$tag.log; exit 1; }
  tail -1 gpurun_out/b_$tag.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('$tag', b['value'], b['ms_per_step'], [(x['k_link_us'],x['k_node_us']) for x in b['roofline']['per_iteration']])"
}
b w3 X=1
b w4 SWMM5_LINK_WAVES=4
b w1 SWMM5_LINK_WAVES=1
