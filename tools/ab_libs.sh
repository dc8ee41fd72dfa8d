#!/bin/bash
# Interleaved A/B of two library builds in one GPU call (LTX_HIP_LIB):
#   tools/ab_libs.sh <libA.so> <libB.so> [rounds]   -- attention microbench, then bench.py
# env ATTN_ONLY=1 skips bench.py; BENCH_ARGS passes extra bench.py flags.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
A="$1"; B="$2"; N=${3:-2}
for i in $(seq 1 $N); do
  for L in "$A" "$B"; do
    echo "== attn $L"
    LTX_HIP_LIB=$L timeout -k 10 120 python -u tools/attn_bench.py --iters 30 || exit $?
  done
done
[ -n "$ATTN_ONLY" ] && exit 0
for i in $(seq 1 $N); do
  for L in "$A" "$B"; do
    echo "== bench $L"
    LTX_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} 2>>gpurun_out/ab_libs.err \
      | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], [(k["kernel"][:60], k["ms_per_step"]) for k in d["kernels"][:4]])' || exit $?
  done
done
