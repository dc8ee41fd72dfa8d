#!/bin/bash
# round 4, GPU call 10: dK/dV kernel's first transposed fragments read an iteration ahead + the
# forward's f32 row sums per k-step: bitwise A/B (F32SUM off) and timing A/B against the r04c
# library, attention GPU tests, step A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd
LTX_ATTN_FWD_F32SUM=0 timeout -k 10 120 python -u tools/attn_ab_bitwise.py $L/libltxhip_r04c.so $L/libltxhip.so > gpurun_out/r04_attn_ab10.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
ATTN_ONLY=1 timeout -k 10 400 bash tools/ab_libs.sh $L/libltxhip_r04c.so $L/libltxhip.so 3 > gpurun_out/r04_attn_libs10.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_large_logits_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r04_attn_tests10.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
for i in 1 2; do
  for lib in libltxhip_r04c.so libltxhip.so; do
    LTX_HIP_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench10_${lib%.so}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
