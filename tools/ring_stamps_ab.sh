# ring GEMM phase stamps (tools/ring_stamps.py) for each LTX_GEMM_EPI_BATCH mode given, after the
# ring GEMM bitwise tests; run on the GPU box: bash tools/ring_stamps_ab.sh 1 2
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_ring_gpu.py > gpurun_out/ring_tests.txt 2>&1
export LTX_HIP_LIB=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd/libltxhip_stamps.so
for b in "$@"; do
  LTX_GEMM_EPI_BATCH=$b timeout -k 10 200 python -u tools/ring_stamps.py > gpurun_out/rs_b$b.txt 2>&1
done
