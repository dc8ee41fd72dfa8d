#!/bin/bash
# round 4, GPU call 11: 4-buffer LDS-DMA rings in the dQ and dK/dV kernels (DMA two tiles ahead),
# lora_wgrad at 512 blocks: bitwise A/B vs r04c (F32SUM off), env A/B of the buffer counts,
# attention GPU tests, step A/B vs r04c
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd
LTX_ATTN_FWD_F32SUM=0 timeout -k 10 120 python -u tools/attn_ab_bitwise.py $L/libltxhip_r04c.so $L/libltxhip.so > gpurun_out/r04_attn_ab11.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -u tools/attn_bench.py --which self --iters 20 --rounds 3 --env-ab LTX_ATTN_DQ_NBUF > gpurun_out/r04_attn_nbuf11.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/attn_bench.py --which self --iters 20 --rounds 3 --env-ab LTX_ATTN_DKDV_NBUF >> gpurun_out/r04_attn_nbuf11.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_large_logits_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r04_attn_tests11.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
for i in 1 2; do
  for lib in libltxhip_r04c.so libltxhip.so; do
    LTX_HIP_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench11_${lib%.so}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
