#!/bin/bash
# A/B of the attention kernels: base library (build_exp/libltxhip_base.so) vs the in-tree build,
# interleaved in one call (tools/attn_bench.py, HIP events).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for i in 1 2; do
  for lib in build_exp/libltxhip_base.so video-generation-for-human-avatars_amd/ltx_amd/libltxhip.so; do
    echo "== $lib"
    LTX_HIP_LIB=$R/$lib timeout -k 10 120 python -u tools/attn_bench.py --iters 30 || exit $?
  done
done
