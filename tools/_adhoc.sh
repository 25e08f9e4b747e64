cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
b() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 $BARGS > gpurun_out/b_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/b_$tag.log; exit 1; }
  tail -1 gpurun_out/b_$tag.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); o=b['roofline']['other_kernels']; print('$tag', b['value'], b['ms_per_step'], o['k_step_end+k_finalize']['avg_launch_us'], o.get('k_qual_node+k_qual_link',{}).get('avg_launch_us'))"
}
H=stormwater-management-model_amd/libswmm5_head.so
b head1 SWMM5_LIB=$H
b new1 X=1
b head2 SWMM5_LIB=$H
b new2 X=1
BARGS="--config 1m_quality"
b headq SWMM5_LIB=$H
b newq X=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_stats.py tests/test_gpu_parity.py tests/test_multigpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "grid or example_qual or regulators or bitwise" > gpurun_out/pt.log 2>&1; echo "pytest exit $?"; tail -3 gpurun_out/pt.log
