set -e
cd /tmp; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 256 512 1024; do
  LTX_GEMM_SMALL_BLOCKS=$v timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tg_$v -o run -- python3 $R/tools/text_gemm_bench.py >> $R/gpurun_out/tg.log 2>&1
  cp /tmp/tg_$v/run_kernel_stats.csv $R/gpurun_out/tg_stats_$v.csv
done
