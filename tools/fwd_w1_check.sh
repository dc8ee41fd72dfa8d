# one-wave forward on the GPU box: bitwise against the pipelined kernel, then A/B timing
set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fwd_w1" > gpurun_out/fwd_w1_tests.txt 2>&1
timeout -k 10 200 python -u tools/attn_bench.py --which self --env-ab LTX_ATTN_FWD_W1 --env-vals 0,1 > gpurun_out/fwd_w1_ab.txt 2>&1
