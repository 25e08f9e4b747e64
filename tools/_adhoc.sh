cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
b() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 $BARGS > gpurun_out/b_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/b_$tag.log; exit 1; }
  tail -1 gpurun_out/b_$tag.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); o=b['roofline']['other_kernels']; print('$tag', b['value'], b['ms_per_step'], o.get('k_qual_node+k_qual_link',{}).get('avg_launch_us'))"
}
H=stormwater-management-model_amd/libswmm5_head.so
N=stormwater-management-model_amd/libswmm5_mi355x.so
C="example_qual grid12_var_qual example_regulators_var_qual example_storage_qual example_dividers example_avg"
timeout -k 10 300 python tools/ab_bitwise.py $H gpurun_out/abA $C > gpurun_out/abA.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_bitwise.py $N gpurun_out/abB $C > gpurun_out/abB.log 2>&1 || exit 1
for c in $C; do cmp gpurun_out/abA/$c.out gpurun_out/abB/$c.out && echo "same $c"; done
BARGS="--config 1m_quality"
for r in 1 2; do b headq$r SWMM5_LIB=$H; b newq$r X=1; done
