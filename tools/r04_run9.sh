#!/bin/bash
# round 4, GPU call 9: round-end evidence on the working tree: tools/final_profile.sh (default bench
# line, kernel-trace stats, FETCH/WRITE and SQ counter passes) + config X bench line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1100 bash tools/final_profile.sh > gpurun_out/r04_final_profile.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --config x --no-cpu-baseline > gpurun_out/final/bench_config_x.jsonl 2> gpurun_out/final/bench_config_x.err
