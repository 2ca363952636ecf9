#!/bin/bash
# PMC passes over the conv microbenchmark (one counter group per pass).
# usage: [MICRO_PREC=1] tools/pmc_conv.sh OUTDIR "B H Cin Cout k s iters" [TILE]
#   TILE: a po_conv tile index (1..45) or "BMxBNxBK[g]"
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/pmc_conv}
SHAPE=${2:-"16 76 128 256 3 1 30"}
TILE=${3:-128x128x16}
if [[ "$TILE" =~ ^[0-9]+$ ]]; then export MICRO_TILE=$TILE; else export ADVPATCH_CONV_TILE=$TILE; fi
mkdir -p $OUT
timeout -k 10 120 python tools/conv_micro.py $SHAPE > $OUT/plain.txt 2>&1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_COUNT" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_THREAD_CYCLES_VALU TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --kernel-include-regex 'conv_' --output-format csv -d $OUT/p$i -o p$i -- python tools/conv_micro.py $SHAPE > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
