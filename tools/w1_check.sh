# the one-wave backward kernels on the GPU box: bitwise tests against the pipelined kernels, phase
# stamps of both loops (diag library), per-kernel times of the self-attention shapes
set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "w1" > gpurun_out/w1_tests.txt 2>&1
export LTX_HIP_LIB=$R/video-generation-for-human-avatars_amd/ltx_amd/libltxhip_diag.so
timeout -k 10 120 python -u tools/dkdv_stamps.py 12 > gpurun_out/w1_dkdv_st.txt 2>&1
timeout -k 10 120 python -u tools/dq_stamps.py 12 > gpurun_out/w1_dq_st.txt 2>&1
unset LTX_HIP_LIB
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ap -o run -- python3 $R/tools/attn_bench.py --iters 5 --which self > /tmp/ap.log 2>&1
cp /tmp/ap/run_kernel_stats.csv $R/gpurun_out/w1_attn_stats.csv
