#!/bin/bash
# Round-end measurement on the GPU box: default bench line, kernel-trace stats, two PMC passes.
# Raw profiler output stays under /tmp (too large for gpurun_out); only summaries are kept.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/final
RAW=/tmp/ltx_prof
mkdir -p $OUT $RAW
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 python3 -u $R/bench.py > $OUT/bench_default.jsonl 2> $OUT/bench_default.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $RAW/trace -o run -- \
    python3 $R/bench.py --steps 16 --warmup 2 --no-cpu-baseline > $OUT/bench_under_rocprof.jsonl 2> $RAW/trace.err
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $RAW/pmc_f -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $RAW/pmc_f.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $RAW/pmc_w -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $RAW/pmc_w.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $RAW/short -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $RAW/short.log 2>&1
python3 $R/tools/rocpd_summary.py $RAW/trace/run_results.db 23 60 > $OUT/trace_summary.txt  # 2 warm-up + 16 timed + 1 + 4 timer steps
python3 $R/tools/pmc_summary.py stats $RAW/trace/run_kernel_stats.csv $OUT/kernel_stats.md > /dev/null
cp $RAW/trace/run_kernel_stats.csv $OUT/kernel_stats.csv
python3 $R/tools/pmc_summary.py traffic $RAW/pmc_f/run_counter_collection.csv $RAW/pmc_w/run_counter_collection.csv \
    $OUT/pmc_dominant_gemm.json > /dev/null
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT \
    --kernel-trace --output-format csv -d $RAW/pmc_sq -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $RAW/pmc_sq.log 2>&1
python3 $R/tools/pmc_table.py $RAW/pmc_sq/run_counter_collection.csv > $OUT/pmc_sq.md
python3 $R/tools/kernel_traffic.py $RAW/pmc_f/run_counter_collection.csv $RAW/pmc_w/run_counter_collection.csv \
    $OUT/traffic.json > /dev/null
python3 $R/tools/hbm_table.py $RAW/pmc_f/run_counter_collection.csv $RAW/pmc_w/run_counter_collection.csv \
    $RAW/short/run_results.db 8 $OUT/hbm_per_kernel.md > /dev/null
ls -la $OUT
