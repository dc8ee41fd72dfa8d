#!/bin/bash
# One GPU call: the -m gpu suite, then the default bench line, then (optionally) the round-end
# profile. A step that times out, aborts or faults (124/134/137/139) ends the call there; a plain
# test failure (exit 1) does not stop the bench.
#   usage: tools/gpu_run.sh [tests-args] ; env PROFILE=1 to run tools/final_profile.sh as well
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ $1 -gt 128 ] && return 0; return 1; }
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${1:-} \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log
if fatal $rc; then echo "tests ended with $rc: stopping"; exit $rc; fi
if [ -n "$NO_BENCH" ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.jsonl 2> gpurun_out/bench.err
rc2=$?; tail -c 3000 gpurun_out/bench.jsonl
if fatal $rc2; then echo "bench ended with $rc2: stopping"; exit $rc2; fi
if [ -n "$PROFILE" ]; then
  timeout -k 10 600 bash tools/final_profile.sh > gpurun_out/final_profile.log 2>&1
  rc3=$?; tail -3 gpurun_out/final_profile.log; exit $rc3
fi
exit $rc
