#!/bin/bash
# round 4, GPU call 13: main library (body3 layout restored for LTX_RING_X3=0) -- ring bitwise
# tests on both builds, then interleaved step A/B main vs X3 (libltxhip_x3.so)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_ring_gpu.py > gpurun_out/r04_ring_tests13.txt 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for lib in libltxhip.so libltxhip_x3.so; do
    LTX_HIP_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench13_${lib%.so}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
