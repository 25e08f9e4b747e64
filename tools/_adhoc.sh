cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
b() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 $BARGS > gpurun_out/b_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/b_$tag.log; exit 1; }
  tail -1 gpurun_out/b_$tag.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); o=b['roofline']['other_kernels']; print('$tag', b['value'], b['ms_per_step'], o['k_node<first>']['avg_launch_us'], o['k_node iteration 1']['avg_launch_us'], o['k_node iterations>=2']['avg_launch_us'])"
}
H=stormwater-management-model_amd/libswmm5_head.so
b head1 SWMM5_LIB=$H
b new1 X=1
b head2 SWMM5_LIB=$H
b new2 X=1
BARGS="--config 100k --steps 400"
b head100k SWMM5_LIB=$H
b new100k X=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vs_oracle.py tests/test_multigpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "grid or example_qual or regulators or bitwise or surcharge or frozen" > gpurun_out/pt.log 2>&1; echo "pytest exit $?"; tail -3 gpurun_out/pt.log
