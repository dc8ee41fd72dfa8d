#!/bin/bash
# round 4, GPU call 7: the whole GPU suite on HEAD (ring GEMM default) incl. the 28-layer 50-step
# loss curve, then smoke()
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread > gpurun_out/r04_gpu_tests7.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r04_gpu_tests7.txt
[ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke7.txt 2>&1
exit $rc
