#!/bin/bash
# round 4, GPU call 22: the final tree -- whole GPU suite, smoke, tools/final_profile.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread > gpurun_out/r04_gpu_tests22.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r04_gpu_tests22.txt
[ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke22.txt 2>&1 || exit $?
timeout -k 10 900 bash tools/final_profile.sh > gpurun_out/r04_final_profile22.log 2>&1
