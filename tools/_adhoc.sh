cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 200 python -u tools/dev_case.py example_shapes_var
