cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
b() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 $BARGS > gpurun_out/b_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/b_$tag.log; exit 1; }
  tail -1 gpurun_out/b_$tag.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); o=b['roofline']['other_kernels']; print('$tag', b['value'], b['ms_per_step'], o['k_node<first>']['avg_launch_us'], o['k_node iteration 1']['avg_launch_us'], o['k_node iterations>=2']['avg_launch_us'])"
}
H=stormwater-management-model_amd/libswmm5_head.so
for r in 1 2; do b head$r SWMM5_LIB=$H; b new8_$r X=1; b new4_$r SWMM5_NODE_SPARSE_GRID_FACTOR=4; b new2_$r SWMM5_NODE_SPARSE_GRID_FACTOR=2; done
