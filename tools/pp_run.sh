R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "ping_pong" > gpurun_out/t_pp.log 2>&1; tail -3 gpurun_out/t_pp.log
for i in 1 2; do for v in 0 4; do echo "== PP=$v"; LTX_ATTN_PP=$v timeout -k 10 120 python -u tools/attn_bench.py --which self --iters 30 2>&1 | grep -v amdgpu.ids || exit 1; done; done
