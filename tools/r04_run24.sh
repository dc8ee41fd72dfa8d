#!/bin/bash
# round 4, GPU call 24: ring GEMM output rows as non-temporal stores (libltxhip_nt.so,
# LTX_RING_NT_STORE=1) against plain stores (libltxhip.so): ring tests, step A/B x3
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd
LTX_HIP_LIB=$L/libltxhip_nt.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_ring_gpu.py > gpurun_out/r04_nt_tests24.txt 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for lib in libltxhip.so libltxhip_nt.so; do
    LTX_HIP_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench24_${lib%.so}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
