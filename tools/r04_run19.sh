#!/bin/bash
# round 4, GPU call 19: the final tree -- whole GPU suite, smoke, default bench line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread > gpurun_out/r04_gpu_tests19.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r04_gpu_tests19.txt
[ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke19.txt 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > gpurun_out/r04_bench19.jsonl 2> gpurun_out/r04_bench19.err
