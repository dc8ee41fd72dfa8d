#!/bin/bash
# round 4, GPU call 2: ring GEMM bitwise tests, attention tests (large logits, noise criterion,
# query-split cross backward), GEMM microbenchmark, step A/B ring vs default
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_ring_gpu.py > gpurun_out/r04_ring_tests.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
$T 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_attention_large_logits_gpu.py "tests/test_kernels_gpu.py" -k "attention" > gpurun_out/r04_attn_tests.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
GEMM_VARIANTS=0,20 $T 300 python -u tools/bench_gemm.py > gpurun_out/r04_gemm_ring.txt 2>&1 || exit $?
for i in 1 2; do
  $T 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench_t$i.json 2>> gpurun_out/r04_bench.err || exit $?
  LTX_GEMM_RING=1 $T 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench_ring$i.json 2>> gpurun_out/r04_bench.err || exit $?
done
