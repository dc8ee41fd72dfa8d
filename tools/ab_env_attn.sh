#!/bin/bash
# Attention microbenchmark A/B of one environment switch in the in-tree library, interleaved:
#   tools/ab_env_attn.sh VAR VALUE_A VALUE_B [rounds] [which]
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
V=$1; A=$2; B=$3; N=${4:-2}; W=${5:-self}
for i in $(seq 1 $N); do
  for x in "$A" "$B"; do
    echo "== $V=$x"
    env $V=$x timeout -k 10 120 python -u tools/attn_bench.py --iters 30 --which $W 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
