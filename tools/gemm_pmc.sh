#!/bin/bash
# Counter pass (SQ + GRBM) over gemm_variants.py --only V for each variant given; summary per variant.
#   usage: tools/gemm_pmc.sh TAG "14 32" qkv,n2048_k2048
set -e
R=$GRAFT_REPO_ROOT
TAG=$1; VARS=$2; SHAPES=$3
OUT=$R/gpurun_out/gpmc_$TAG
RAW=/tmp/gpmc_$TAG
mkdir -p $OUT $RAW
cd /tmp
export TMPDIR=/tmp
P1=${PMC:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"}
for V in $VARS; do
  LTX_GEMM_BLASLT=0 timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $RAW/v$V -o run -- \
      python3 $R/tools/gemm_variants.py --only $V --shapes $SHAPES --iters 4 > $RAW/v$V.log 2>&1
  echo "## variant $V ($P1)" >> $OUT/summary.md
  python3 $R/tools/pmc_table.py $RAW/v$V/run_counter_collection.csv | grep -v "at::native\|fillBuffer" >> $OUT/summary.md
done
