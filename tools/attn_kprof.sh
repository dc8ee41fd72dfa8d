# Per-kernel durations of tools/attn_bench.py (--which $WHICH) under rocprofv3 for an LTX_* switch:
#   attn_kprof.sh VAR v1 v2 ...   (WHICH=cross|self, default cross)
set -e
R=$GRAFT_REPO_ROOT
VAR=$1; shift
cd /tmp; export TMPDIR=/tmp
for v in "$@"; do
  export "$VAR=$v"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ak_$v -o run -- python3 $R/tools/attn_bench.py --which ${WHICH:-cross} > /dev/null 2>&1
  python3 -c "
import csv
for r in csv.DictReader(open('/tmp/ak_$v/run_kernel_stats.csv')):
    if 'attn' in r['Name']: print('$VAR=$v', r['Name'][:48], r['Calls'], r['AverageNs'])"
done
