#!/bin/bash
# PMC passes over the training step's warp kernels (box forward with saved
# factors, factor -> gradient pass, phase B gather) at config 5 (tiny B=256 @416)
# and config 2 (yolov3 B=16 @608): what bounds them.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for cfg in ${CONFIGS:-tiny yolov3}; do
OUT=gpurun_out/pmc_warp_$cfg
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_COUNT" \
           "SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_BUSY TD_TC_STALL" \
           "FETCH_SIZE TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex 'warp_box|warp_bwd_b' --output-format csv -d $OUT/p$i -o p$i \
    -- python bench.py --config $cfg --steps 3 --warmup 2 --no-cpu-baseline --no-tiny > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail $OUT/p$i.log; exit 1; }
done
echo "== $cfg"; PMC_BY_KERNEL=1 python3 tools/pmc_read.py $OUT | tee $OUT/summary.txt
done
