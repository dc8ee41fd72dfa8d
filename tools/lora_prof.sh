# Per-kernel durations of tools/lora_bench.py (or $SCRIPT) under rocprofv3 for an LTX_* switch:
#   lora_prof.sh VAR v1 v2 ...
set -e
R=$GRAFT_REPO_ROOT
VAR=$1; shift
cd /tmp; export TMPDIR=/tmp
for v in "$@"; do
  export "$VAR=$v"
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lp_$v -o run -- python3 $R/${SCRIPT:-tools/lora_bench.py} >> $R/gpurun_out/lora_prof.log 2>&1
  python3 -c "
import csv
for r in csv.DictReader(open('/tmp/lp_$v/run_kernel_stats.csv')):
    if 'lora' in r['Name']: print('$VAR=$v', r['Name'][:40], r['Calls'], r['AverageNs'])" >> $R/gpurun_out/lora_prof_sum.log
done
