#!/bin/bash
# round 4, GPU call 16: ring GEMM K loop touching the epilogue's aux0 rows (LTX_RING_TOUCH=1,
# libltxhip.so) against the loop without (libltxhip_notouch.so): bitwise GEMM tests, stamps of both,
# step A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_ring_gpu.py > gpurun_out/r04_ring_tests16.txt 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
LTX_HIP_LIB=$L/libltxhip_stamps.so timeout -k 10 200 python -u tools/ring_stamps.py 20 > gpurun_out/r04_ring_stamps16_touch.txt 2>&1 || exit $?
LTX_HIP_LIB=$L/libltxhip_stamps_notouch.so timeout -k 10 200 python -u tools/ring_stamps.py 20 > gpurun_out/r04_ring_stamps16_notouch.txt 2>&1 || exit $?
for i in 1 2; do
  for lib in libltxhip.so libltxhip_notouch.so; do
    LTX_HIP_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench16_${lib%.so}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
