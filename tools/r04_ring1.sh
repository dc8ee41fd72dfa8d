#!/bin/bash
# round 4: first GPU run of the ring GEMM: bitwise tests vs gemm_nt_kernel_t, then the GEMM
# microbenchmark (variants 0 = gemm_nt_kernel_t, 20 = ring) and the step with / without the ring
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_ring_gpu.py > gpurun_out/r04_ring_tests.txt 2>&1 || exit $?
GEMM_VARIANTS=0,20 timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/r04_gemm_ring.txt 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench_t$i.json 2>> gpurun_out/r04_bench.err || exit $?
  LTX_GEMM_RING=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench_ring$i.json 2>> gpurun_out/r04_bench.err || exit $?
done
