#!/bin/bash
# PMC passes over the first-layer pooled conv (direct and F(2x2)), B=256 @416 3->16
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-True wino}; do
OUT=gpurun_out/pmc_first_$v
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_COUNT" \
           "SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_BUSY TD_TC_STALL"; do
  i=$((i+1))
  FIRST_ONLY=$v timeout -k 10 120 rocprofv3 --pmc $grp --kernel-include-regex 'first_pool' --output-format csv -d $OUT/p$i -o p$i -- python tools/first_micro.py 10 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail $OUT/p$i.log; exit 1; }
done
echo "== $v"; python3 tools/pmc_read.py $OUT | tee $OUT/summary.txt
done
