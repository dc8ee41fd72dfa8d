# persistent backward kernels on the GPU box: bitwise against the per-block kernels, A/B timing,
# phase stamps (diag library)
set -e
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "w1p" > gpurun_out/w1p_tests.txt 2>&1
timeout -k 10 200 python -u tools/attn_bench.py --which self --env-ab LTX_ATTN_DKDV_W1 --env-vals 1,2 > gpurun_out/w1p_ab.txt 2>&1
timeout -k 10 200 python -u tools/attn_bench.py --which self --env-ab LTX_ATTN_DQ_W1 --env-vals 1,2 > gpurun_out/w1p_ab_dq.txt 2>&1
bash tools/w1_stamps.sh 22 22
