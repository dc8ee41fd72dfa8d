#!/bin/bash
# debug aid: a library whose one-wave forward body comes from tools/gen_attn_fwd.py with VARIANT flags
# ($1, comma separated), built next to the default one as ltx_amd/libltxhip_fv.so (only
# attention_pipe.o differs; it is compiled with -DLTX_FWD_W1, as `make fwdw1` does)
set -e
cd "$(dirname "$0")/../video-generation-for-human-avatars_amd/csrc"
mkdir -p build_fv
GEN_FWD_VARIANT="$1" python3 ../../tools/gen_attn_fwd.py build_fv/attn_fwd_body.h > /dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
    -I../../include -I. -Ibuild_fv -DLTX_FWD_W1 -fno-slp-vectorize -c attention_pipe.hip -o build_fv/attention_pipe.o
objs=$(for f in *.hip; do o=build/${f%.hip}.o; [ "$o" != build/attention_pipe.o ] && echo $o; done)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../ltx_amd/libltxhip_fv.so $objs build_fv/attention_pipe.o
echo built ../ltx_amd/libltxhip_fv.so "($1)"
