#!/bin/bash
# round 4, GPU call 4: ring2 / ring3 bitwise tests, GEMM microbench, step A/B (t-kernel, ring2, ring3)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_ring_gpu.py > gpurun_out/r04_ring_tests4.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
GEMM_VARIANTS=0,21,22 $T 300 python -u tools/bench_gemm.py > gpurun_out/r04_gemm_ring4.txt 2>&1 || exit $?
for i in 1 2; do
  for R in 0 2 3; do
    LTX_GEMM_RING=$R $T 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench4_r${R}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
