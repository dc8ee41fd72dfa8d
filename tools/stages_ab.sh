# A/B of the 128x128 GEMM's LDS stages (LTX_GEMM_SMALL_STAGES: 0 = auto, 2..4 forced), GPU box
set -e
R=$GRAFT_REPO_ROOT
cd /tmp; export TMPDIR=/tmp
for v in 2 3 4 2 3 4; do
  LTX_GEMM_SMALL_STAGES=$v timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/st_$v -o run -- python3 $R/tools/text_gemm_bench.py >> $R/gpurun_out/stages.log 2>&1
  python3 -c "
import csv
for r in csv.DictReader(open('/tmp/st_$v/run_kernel_stats.csv')):
    if 'gemm_nt_kernel' in r['Name'] or 'splitk' in r['Name']: print('stages $v', r['Name'][:48], r['Calls'], r['AverageNs'])" >> $R/gpurun_out/stages_sum.log
done
