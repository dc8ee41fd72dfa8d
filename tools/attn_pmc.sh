#!/bin/bash
# Counter passes over the attention microbenchmark (tools/attn_bench.py, config-A shapes), one
# rocprofv3 run per pass, program directly after --. Summary -> gpurun_out/apmc_<tag>/summary.md
#   usage: tools/attn_pmc.sh TAG [LIB]   (LIB: optional LTX_HIP_LIB override for an A/B build)
set -e
R=$GRAFT_REPO_ROOT
TAG=$1
OUT=$R/gpurun_out/apmc_$TAG
RAW=/tmp/apmc_$TAG
mkdir -p $OUT $RAW
cd /tmp
export TMPDIR=/tmp
[ -n "$2" ] && export LTX_HIP_LIB=$2
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $RAW/a$i -o run -- \
      python3 $R/tools/attn_bench.py --iters 3 --which ${WHICH:-self} > $RAW/a$i.log 2>&1
  echo "## pass $i" >> $OUT/summary.md
  python3 $R/tools/pmc_table.py $RAW/a$i/run_counter_collection.csv | grep -v "at::native\|fillBuffer\|distribution\|elementwise" >> $OUT/summary.md
done
ls -la $OUT
