cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k "extfile" > gpurun_out/pytest_shapes.log 2>&1; echo "pytest $?"; grep -E "^E |passed|failed" gpurun_out/pytest_shapes.log | head -30
