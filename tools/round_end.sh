#!/bin/bash
# Full GPU test suite, then the round-end profile (tools/final_profile.sh).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/final_profile.sh > gpurun_out/final_profile.log 2>&1; rc=$?
tail -3 gpurun_out/final_profile.log
exit $rc
