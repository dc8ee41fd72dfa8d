#!/bin/bash
# Fast diag library: only attention_pipe.o rebuilt with the timing-only loop variants
# (tools/gen_attn_bwd.py --diag), linked with the default build's other objects.
set -e
cd "$(dirname "$0")/../video-generation-for-human-avatars_amd/csrc"
mkdir -p build_diag
python3 ../../tools/gen_attn_bwd.py --diag build_diag/attn_bwd_body_diag.h
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
    -I../../include -I. -Ibuild_diag -DLTX_DKDV_DIAG -fno-slp-vectorize -c attention_pipe.hip -o build_diag/attention_pipe.o
objs=$(for f in *.hip; do o=build/${f%.hip}.o; [ "$o" != build/attention_pipe.o ] && echo $o; done)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../ltx_amd/libltxhip_diag.so $objs build_diag/attention_pipe.o
echo built ../ltx_amd/libltxhip_diag.so
