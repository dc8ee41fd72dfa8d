#!/bin/bash
# The attn2 cross-attention kernels at config A (tools/cross_bench.py): HIP-event timing, a kernel
# trace, and SQ / HBM counter passes (one rocprofv3 run each, the program directly after --).
# Summaries -> gpurun_out/cross_<tag>/.   usage: tools/cross_prof.sh TAG [extra cross_bench args]
set -e
R=$GRAFT_REPO_ROOT
TAG=$1; shift
OUT=$R/gpurun_out/cross_$TAG
RAW=/tmp/cross_$TAG
mkdir -p $OUT $RAW
cd /tmp
export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/cross_bench.py "$@" > $OUT/bench.txt 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $RAW/t -o run -- \
    python3 $R/tools/cross_bench.py --iters 10 --rounds 1 > $RAW/t.log 2>&1
python3 -c "
import csv
for r in csv.DictReader(open('$RAW/t/run_kernel_stats.csv')):
    if 'attn' in r['Name']: print(r['Name'][:60], r['Calls'], r['AverageNs'])" > $OUT/trace.txt
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $RAW/p1 -o run -- \
    python3 $R/tools/cross_bench.py --iters 3 --rounds 1 > $RAW/p1.log 2>&1
python3 $R/tools/pmc_table.py $RAW/p1/run_counter_collection.csv | grep "attn" > $OUT/pmc_sq.md || true
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $RAW/$C -o run -- \
      python3 $R/tools/cross_bench.py --iters 3 --rounds 1 > $RAW/$C.log 2>&1
  python3 $R/tools/pmc_table.py $RAW/$C/run_counter_collection.csv | grep "attn" > $OUT/pmc_$C.md || true
done
cat $OUT/bench.txt $OUT/trace.txt
