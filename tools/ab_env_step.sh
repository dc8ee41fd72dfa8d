#!/bin/bash
# Interleaved step A/B of one environment switch on one box: bench.py twice with $VAR=$A and twice
# with $VAR=$B (same library), then the GPU tests named by $TESTS (pytest -k expression) first.
#   usage: TAG=r06o VAR=LTX_LORA_DY_DA A=1 B=0 TESTS="lora_dy" bash tools/ab_env_step.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-abenv}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -q -k "$TESTS" --timeout 300 --timeout-method thread -x > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  env $VAR=$A timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_a$i.json 2>$O/bench_a$i.err || exit 6
  env $VAR=$B timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_b$i.json 2>$O/bench_b$i.err || exit 7
done
python - <<PY
import json
for t in ('a1','b1','a2','b2'):
    d=json.loads(open('$O/bench_'+t+'.json').read().strip().splitlines()[-1])
    print(t, '$VAR=' + ('$A' if t[0]=='a' else '$B'), d['value'], d['ms_per_step'])
PY
