cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
b() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu --kernel-reps 0 $BARGS > gpurun_out/b_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/b_$tag.log; exit 1; }
  tail -1 gpurun_out/b_$tag.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); o=b['roofline']['other_kernels']; print('$tag', b['value'], b['ms_per_step'], o['k_step_end+k_finalize']['avg_launch_us'])"
}
H=stormwater-management-model_amd/libswmm5_head.so
N=stormwater-management-model_amd/libswmm5_mi355x.so
C="example_var grid12_var_qual example_regulators_var_qual example_stride example_avg example_tidal_var"
timeout -k 10 300 python tools/ab_bitwise.py $H gpurun_out/abA $C > gpurun_out/abA.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_bitwise.py $N gpurun_out/abB $C > gpurun_out/abB.log 2>&1 || exit 1
for c in $C; do cmp gpurun_out/abA/$c.out gpurun_out/abB/$c.out && cmp gpurun_out/abA/$c.rpt gpurun_out/abB/$c.rpt && echo "same $c"; done
for r in 1 2; do b head$r SWMM5_LIB=$H; b new$r X=1; done
BARGS="--config 100k --steps 400"
for r in 1 2; do b head100k$r SWMM5_LIB=$H; b new100k$r X=1; done
