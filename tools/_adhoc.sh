cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
b() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 $BARGS > gpurun_out/b_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/b_$tag.log; exit 1; }
  grep "probe k=" gpurun_out/b_$tag.log
  tail -1 gpurun_out/b_$tag.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('$tag', b['value'], b['ms_per_step'], [(x['k_link_us'],x['k_node_us']) for x in b['roofline']['per_iteration']])"
}
H=stormwater-management-model_amd/libswmm5_head.so
b head1 SWMM5_LIB=$H
b new1 X=1
b head2 SWMM5_LIB=$H
b new2 X=1
b newp SWMM5_PROBE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_vs_oracle.py tests/test_multigpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1; echo "pytest exit $?"; tail -3 gpurun_out/pt.log
