#!/bin/bash
# round 4, GPU call 6: single-asm ring kernel (main loop + fused K extension) bitwise tests, step A/B
# (t-kernel vs ring), per-phase stamps of the ring kernel on the step's shapes
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_ring_gpu.py > gpurun_out/r04_ring_tests6.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
for i in 1 2; do
  for R in 0 1; do
    LTX_GEMM_RING=$R $T 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench6_r${R}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
LTX_HIP_LIB=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd/libltxhip_stamps.so $T 200 python -u tools/ring_stamps.py 20 > gpurun_out/r04_ring_stamps6.txt 2>&1 || exit $?
LTX_HIP_LIB=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd/libltxhip_stamps.so $T 200 python -u tools/ring_stamps.py 0 > gpurun_out/r04_ring_stamps6_t.txt 2>&1 || true
