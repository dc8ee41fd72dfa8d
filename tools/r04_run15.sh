#!/bin/bash
# round 4, GPU call 15: dQ and dK/dV kernels concurrently on two streams (LTX_ATTN_BWD_CONC,
# off by default): attention microbench A/B, step A/B, attention GPU tests with it on
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 200 python -u tools/attn_bench.py --which self --iters 20 --rounds 3 --env-ab LTX_ATTN_BWD_CONC > gpurun_out/r04_attn_conc15.txt 2>&1 || exit $?
LTX_ATTN_BWD_CONC=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_large_logits_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r04_attn_tests15.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
for i in 1 2; do
  for c in 0 1; do
    LTX_ATTN_BWD_CONC=$c timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench15_conc${c}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
