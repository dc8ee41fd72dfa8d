#!/bin/bash
# round 4, GPU call 3: ring2 bitwise tests, GEMM microbench (t-kernel / ring / ring2 / hipBLASLt),
# PMC passes (SQ + TA/TCP) on one shape, step with LTX_GEMM_RING=2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_ring_gpu.py > gpurun_out/r04_ring_tests3.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
GEMM_VARIANTS=0,20,21 $T 300 python -u tools/bench_gemm.py > gpurun_out/r04_gemm_ring3.txt 2>&1 || exit $?
PASSES="P1 P3" $T 400 bash tools/gemm_pmc_cmp.sh r04ring n2048_k8192 "0 20 21" torch > gpurun_out/r04_pmc.log 2>&1 || exit $?
$T 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench3_t.json 2>> gpurun_out/r04_bench.err || exit $?
LTX_GEMM_RING=2 $T 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench3_ring2.json 2>> gpurun_out/r04_bench.err || exit $?
