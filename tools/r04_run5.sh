#!/bin/bash
# round 4, GPU call 5: ring3 + K extension bitwise tests, step A/B (t-kernel vs ring3), rocprof
# kernel stats of the ring3 step
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_ring_gpu.py > gpurun_out/r04_ring_tests5.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
for i in 1 2; do
  for R in 0 3; do
    LTX_GEMM_RING=$R $T 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04_bench5_r${R}_$i.json 2>> gpurun_out/r04_bench.err || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
LTX_GEMM_RING=3 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 16 --warmup 2 --no-cpu-baseline > /tmp/r5prof.log 2>&1 || exit $?
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py stats /tmp/r5prof/run_kernel_stats.csv $GRAFT_REPO_ROOT/gpurun_out/r04_ring3_kernel_stats.md > /dev/null
cp /tmp/r5prof/run_kernel_stats.csv $GRAFT_REPO_ROOT/gpurun_out/r04_ring3_kernel_stats.csv
