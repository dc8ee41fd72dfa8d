#!/bin/bash
# round 4, GPU call 20: the batched text side's attn2 k_norm as one grouped launch per pass
# (LTX_TEXT_KNORM_GROUPED, default 1): kernel / model-level tests, step A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "qk_norm" tests/test_parity_2b_gpu.py -k "qk_norm or text_stack" > gpurun_out/r04_knorm_tests20.txt 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for c in 0 1; do
    LTX_TEXT_KNORM_GROUPED=$c timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench20_g${c}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
