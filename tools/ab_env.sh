#!/bin/bash
# Interleaved A/B of an env switch in one GPU call: tools/ab_env.sh VAR valA valB [rounds] [script args]
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
VAR=$1; A=$2; B=$3; N=${4:-2}; shift 4
for i in $(seq 1 $N); do for v in "$A" "$B"; do
  echo "== $VAR=$v"; env $VAR=$v timeout -k 10 120 python -u "$@" || exit $?
done; done
