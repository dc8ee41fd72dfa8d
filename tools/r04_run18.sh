#!/bin/bash
# round 4, GPU call 18: q/k norm + RoPE kernels with the batch-fastest per-XCD item order
# (libltxhip_qkx.so) against HEAD's order (libltxhip.so): kernel times + bitwise outputs, the
# norm/RoPE GPU tests on the new build, step A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd
LTX_HIP_LIB=$L/libltxhip.so timeout -k 10 120 python -u tools/qk_norm_bench.py /tmp/qk_ref.pt > gpurun_out/r04_qk18.txt 2>&1 || exit $?
LTX_HIP_LIB=$L/libltxhip_qkx.so timeout -k 10 120 python -u tools/qk_norm_bench.py /tmp/qk_new.pt /tmp/qk_ref.pt >> gpurun_out/r04_qk18.txt 2>&1 || exit $?
LTX_HIP_LIB=$L/libltxhip.so timeout -k 10 120 python -u tools/qk_norm_bench.py /tmp/qk_ref2.pt /tmp/qk_new.pt >> gpurun_out/r04_qk18.txt 2>&1 || exit $?
LTX_HIP_LIB=$L/libltxhip_qkx.so timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/r04_qk_tests18.txt 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lib in libltxhip.so libltxhip_qkx.so; do
    LTX_HIP_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench18_${lib%.so}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
