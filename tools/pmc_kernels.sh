#!/bin/bash
# Counter passes (one rocprofv3 run per counter group, program directly after --) over the GEMM and
# attention microbenchmarks at the config-A shapes. Raw CSVs stay under /tmp; the per-kernel
# summary (tools/pmc_table.py) goes to gpurun_out/pmc/.
#   usage: tools/pmc_kernels.sh [tag]
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r02}
OUT=$R/gpurun_out/pmc_$TAG
RAW=/tmp/ltx_pmc_$TAG
mkdir -p $OUT $RAW
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1"; do
  i=$((i+1))
  LTX_GEMM_BLASLT=0 timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $RAW/g$i -o run -- \
      python3 $R/tools/gemm_variants.py --only 0 --shapes qkv,ff_up_gelu,n2048_k8192,out1_gres --iters 4 > $RAW/g$i.log 2>&1
  LTX_GEMM_BLASLT=1 timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $RAW/b$i -o run -- \
      python3 $R/tools/gemm_variants.py --only 0 --shapes qkv,n2048_k8192 --iters 4 > $RAW/b$i.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $RAW/a$i -o run -- \
      python3 $R/tools/attn_bench.py --iters 3 > $RAW/a$i.log 2>&1
  python3 $R/tools/pmc_table.py $RAW/g$i/run_counter_collection.csv $RAW/b$i/run_counter_collection.csv \
      $RAW/a$i/run_counter_collection.csv > $OUT/pass$i.md
done
ls -la $OUT
