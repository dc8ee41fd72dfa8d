#!/bin/bash
# Kernel traces of bench.py under two environment settings (same call): per-kernel totals and
# device idle gaps of each.   tools/prof_ab.sh "LTX_TEXT_BATCH=0" "LTX_TEXT_BATCH=1"
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/prof_ab; RAW=/tmp/ltx_prof_ab
mkdir -p $OUT $RAW; cd /tmp; export TMPDIR=/tmp
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $RAW/t$i -o run -- \
      python3 $R/bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline > $OUT/bench_$i.jsonl 2> $RAW/t$i.err || exit $?
  echo "== $e" > $OUT/summary_$i.txt
  python3 $R/tools/step_gaps.py $RAW/t$i/run_results.db 500 20 ${SKIP_MS:-1200} >> $OUT/summary_$i.txt
  python3 $R/tools/rocpd_summary.py $RAW/t$i/run_results.db 1 70 >> $OUT/summary_$i.txt
  head -30 $OUT/summary_$i.txt
done
