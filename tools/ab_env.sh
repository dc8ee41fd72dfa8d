#!/bin/bash
# Interleaved A/B of bench.py under two environment settings in one GPU call:
#   tools/ab_env.sh "LTX_TEXT_BATCH=0" "LTX_TEXT_BATCH=1" [rounds]
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
A="$1"; B="$2"; N=${3:-2}
for i in $(seq 1 $N); do
  for e in "$A" "$B"; do
    echo "== $e"
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} 2>>gpurun_out/ab_env.err \
      | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' || exit $?
  done
done
