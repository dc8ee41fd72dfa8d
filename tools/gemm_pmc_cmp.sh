#!/bin/bash
# Counter passes (one rocprofv3 run per counter group, program right after --) comparing GEMM
# variants and torch (hipBLASLt) on one training shape. Summaries -> gpurun_out/gcmp_<tag>/.
#   usage: tools/gemm_pmc_cmp.sh TAG SHAPE "0 40" [torch]
set -e
R=$GRAFT_REPO_ROOT
TAG=$1; SHAPE=$2; VARS=$3; TORCH=${4:-}
OUT=$R/gpurun_out/gcmp_$TAG
RAW=/tmp/gcmp_$TAG
mkdir -p $OUT $RAW
cd /tmp
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT"
P4="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P5="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"
P6="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
run() {  # name args...
  local name=$1; shift
  local i=0
  for PN in ${PASSES:-P1 P2 P3}; do
    P=${!PN}
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $RAW/$name$i -o run -- \
        python3 $R/tools/gemm_variants.py "$@" --shape $SHAPE --iters 4 > $RAW/$name$i.log 2>&1
    echo "## $name pass $i" >> $OUT/summary.md
    python3 $R/tools/pmc_table.py $RAW/$name$i/run_counter_collection.csv | grep -v "at::native\|fillBuffer\|distribution\|elementwise" >> $OUT/summary.md
  done
}
for V in $VARS; do run v$V --only $V; done
if [ -n "$TORCH" ]; then run torch --only 0 --torch; fi
ls -la $OUT
