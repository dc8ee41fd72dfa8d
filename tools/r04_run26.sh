#!/bin/bash
# round 4, GPU call 26: the text-key batch sums of every block in one launch (LTX_TEXT_BSUM_GROUPED,
# with the grouped k_norm): text-stack / k_norm / attention tests, step A/B x3, kernel-trace stats
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/k26
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parity_2b_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -k "qk_norm or text_stack or frozen_caption or attention_bwd_one_pass or lora" > gpurun_out/r04_bsum_tests26.txt 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for c in 0 1; do
    LTX_TEXT_BSUM_GROUPED=$c timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench26_b${c}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
for c in 0 1; do
  LTX_TEXT_BSUM_GROUPED=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k26_$c -o run -- \
      python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline > $R/gpurun_out/k26/bench_$c.jsonl 2> $R/gpurun_out/k26/err_$c.txt || exit $?
  cp /tmp/k26_$c/run_kernel_stats.csv $R/gpurun_out/k26/kernel_stats_$c.csv
done
