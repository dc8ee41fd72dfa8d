#!/bin/bash
# round 4, GPU call 12: ring GEMM with three X stages (gen_gemm_ring.py body4, libltxhip_x3.so)
# against the two-stage body (libltxhip.so): bitwise GEMM tests on the X3 build, GEMM microbench,
# step A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd
LTX_HIP_LIB=$L/libltxhip_x3.so timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_ring_gpu.py > gpurun_out/r04_ring_tests12.txt 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
LTX_HIP_LIB=$L/libltxhip_stamps.so timeout -k 10 200 python -u tools/ring_stamps.py 20 > gpurun_out/r04_ring_stamps12_x2.txt 2>&1 || exit $?
LTX_HIP_LIB=$L/libltxhip_stamps_x3.so timeout -k 10 200 python -u tools/ring_stamps.py 20 > gpurun_out/r04_ring_stamps12_x3.txt 2>&1 || exit $?
for i in 1 2; do
  for lib in libltxhip.so libltxhip_x3.so; do
    LTX_HIP_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench12_${lib%.so}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
