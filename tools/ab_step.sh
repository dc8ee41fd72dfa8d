#!/bin/bash
# Interleaved step A/B on one box: the in-tree library against build_ab/libltxhip_base.so (the
# previous build), bench.py twice each; then the GPU tests named by $TESTS (pytest -k expression).
#   usage: TAG=r06e TESTS="rowdot or gemm_ring" bash tools/ab_step.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -q -k "$TESTS" --timeout 300 --timeout-method thread -x > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_new$i.json 2>$O/bench_new$i.err || exit 6
  LTX_HIP_LIB=$PWD/build_ab/libltxhip_base.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_base$i.json 2>$O/bench_base$i.err || exit 7
done
python - <<PY
import json
for t in ('new1','base1','new2','base2'):
    d=json.loads(open('$O/bench_'+t+'.json').read().strip().splitlines()[-1])
    ks={k['kernel'].split('(')[0].replace('ltx::',''): k['ms_per_step'] for k in d['kernels']}
    print(t, d['value'], d['ms_per_step'], {k: v for k, v in ks.items() if '8, 0, 7' in k})
PY
