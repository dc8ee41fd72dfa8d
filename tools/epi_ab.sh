#!/bin/bash
# attention tests, the dK/dV item stamps (diag library, tools/build_diag.sh), then an interleaved A/B
# of a baseline library against the tree's libltxhip.so. The baseline is built by hand beforehand:
#   git stash; make -C video-generation-for-human-avatars_amd/csrc ARCH=gfx950;
#   cp video-generation-for-human-avatars_amd/ltx_amd/libltxhip{,_base}.so; git stash pop; make ... again
# env ATTN_ONLY=1 (attention microbench only), ROUNDS (default 2)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
L=$R/video-generation-for-human-avatars_amd/ltx_amd
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_large_logits_gpu.py -m gpu -x -q \
    -k "attention" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_tests.log; [ $rc -ne 0 ] && exit $rc
LTX_HIP_LIB=$L/libltxhip_diag.so timeout -k 10 150 python -u tools/dkdv_item_stamps.py > gpurun_out/item_stamps2.txt 2>&1
rc=$?; cat gpurun_out/item_stamps2.txt; [ $rc -ne 0 ] && exit $rc
ATTN_ONLY=${ATTN_ONLY:-} bash tools/ab_libs.sh $L/libltxhip_base.so $L/libltxhip.so ${ROUNDS:-2} > gpurun_out/epi_ab.txt 2>&1
rc=$?; cat gpurun_out/epi_ab.txt; exit $rc
