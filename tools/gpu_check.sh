R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_full_gpu.py tests/test_parity_2b_gpu.py tests/test_full_2b_gpu.py > gpurun_out/t_check.log 2>&1; rc=$?; tail -2 gpurun_out/t_check.log; exit $rc
