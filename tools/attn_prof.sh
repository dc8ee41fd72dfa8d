#!/bin/bash
# Kernel trace + two SQ counter passes over the self-attention microbenchmark, for one env setting
#   tools/attn_prof.sh TAG [VAR=VALUE ...]    -> gpurun_out/aprof_TAG/{stats.csv,summary.md}
set -e
R=$GRAFT_REPO_ROOT
TAG=$1; shift
OUT=$R/gpurun_out/aprof_$TAG; RAW=/tmp/aprof_$TAG
mkdir -p $OUT $RAW
cd /tmp; export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $RAW/kt -o run -- \
    python3 $R/tools/attn_bench.py --iters 5 --which ${WHICH:-self} > $RAW/kt.log 2>&1
cp $RAW/kt/run_kernel_stats.csv $OUT/stats.csv 2>/dev/null || find $RAW/kt -name '*kernel_stats.csv' -exec cp {} $OUT/stats.csv \;
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $RAW/a$i -o run -- \
      python3 $R/tools/attn_bench.py --iters 3 --which ${WHICH:-self} > $RAW/a$i.log 2>&1
  echo "## pass $i" >> $OUT/summary.md
  python3 $R/tools/pmc_table.py $RAW/a$i/run_counter_collection.csv | grep -v "at::native\|fillBuffer\|distribution\|elementwise" >> $OUT/summary.md
done
