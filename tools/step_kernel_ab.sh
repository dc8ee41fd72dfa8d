# Per-kernel durations inside the training step for an LTX_* switch (rocprofv3 --stats of a short
# bench.py run per value): step_kernel_ab.sh VAR KERNEL_SUBSTRING v1 v2 ...  (@path = repo-relative path)
set -e
R=$GRAFT_REPO_ROOT
VAR=$1; KSUB=$2; shift 2
cd /tmp; export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  case "$v" in @*) v="$R/${v#@}" ;; esac  # @path: relative to the repo root (LTX_HIP_LIB A/B)
  export "$VAR=$v"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sk_$i -o run -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $R/gpurun_out/sk_bench_$i.jsonl 2>> $R/gpurun_out/sk.log
  python3 -c "
import csv
for r in csv.DictReader(open('/tmp/sk_$i/run_kernel_stats.csv')):
    if '$KSUB' in r['Name']: print('$VAR=$v', r['Name'][:48], r['Calls'], r['AverageNs'])" >> $R/gpurun_out/sk_sum.log
done
