#!/bin/bash
# round 4, GPU call 8: attention bitwise A/B vs the previous library, whole GPU suite on the working
# tree (ring default + batched ring epilogue + vector pack2 + dQ tk prefetch), step A/B against the previous library (libltxhip_prev.so = HEAD 98a3ab8), smoke
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd
LTX_ATTN_FWD_F32SUM=0 timeout -k 10 120 python -u tools/attn_ab_bitwise.py $L/libltxhip_prev.so $L/libltxhip.so > gpurun_out/r04_attn_ab8.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread > gpurun_out/r04_gpu_tests8.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r04_gpu_tests8.txt
[ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -u tools/attn_bench.py --which self --iters 20 --rounds 3 --env-ab LTX_ATTN_FWD_F32SUM > gpurun_out/r04_attn_f32sum8.txt 2>&1 || exit $?
for i in 1 2; do
  LTX_HIP_LIB=$L/libltxhip_prev.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench8_prev_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench8_new_$i.json 2>> gpurun_out/r04_bench.err || exit $?
done
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke8.txt 2>&1 || exit $?
LTX_HIP_LIB=$L/libltxhip_stamps.so timeout -k 10 200 python -u tools/ring_stamps.py 20 > gpurun_out/r04_ring_stamps8.txt 2>&1
exit $rc
