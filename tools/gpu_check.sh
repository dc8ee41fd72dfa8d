R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_parity_2b_gpu.py tests/test_model_gpu.py > gpurun_out/t_check.log 2>&1; rc=$?; tail -4 gpurun_out/t_check.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 0 1; do echo "== ROWS=$v"; LTX_LORA_ROWS=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>>gpurun_out/b_check.err | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' || exit 1; done; done
