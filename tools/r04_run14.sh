#!/bin/bash
# round 4, GPU call 14: round-end evidence on HEAD: whole GPU suite, smoke, tools/final_profile.sh
# (default bench line, kernel-trace stats, FETCH/WRITE and SQ counter passes), config X at B = 8
# and B = 1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread > gpurun_out/r04_gpu_tests14.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r04_gpu_tests14.txt
[ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke14.txt 2>&1 || exit $?
timeout -k 10 900 bash tools/final_profile.sh > gpurun_out/r04_final_profile14.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --config x --no-cpu-baseline > gpurun_out/final/bench_config_x.jsonl 2> gpurun_out/final/bench_config_x.err || exit $?
timeout -k 10 300 python3 -u bench.py --config x --batch 1 --no-cpu-baseline > gpurun_out/final/bench_config_x_b1.jsonl 2> gpurun_out/final/bench_config_x_b1.err
