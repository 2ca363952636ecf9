#!/bin/bash
# PMC of tile 71 (conv_wino6_k, F(4x4,3x3)) on bench shapes (TILES="71 70" to compare)
set -e
cd "$GRAFT_REPO_ROOT"
for shape in "16 76 128 256 3 1 20" "16 19 512 1024 3 1 20"; do
  tag=$(echo $shape | awk '{print $2}')
  for t in ${TILES:-71}; do
    O=gpurun_out/pmc_t${t}_$tag
    MICRO_RES=1 bash tools/pmc_conv.sh $O "$shape" $t
    MICRO_TILE=$t MICRO_RES=1 timeout -k 10 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-include-regex 'conv_' \
        --output-format csv -d $O/p4 -o p4 -- python tools/conv_micro.py $shape > $O/p4.log 2>&1
    MICRO_TILE=$t MICRO_RES=1 timeout -k 10 180 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TD_BUSY_sum TD_TC_STALL_sum --kernel-include-regex 'conv_' \
        --output-format csv -d $O/p5 -o p5 -- python tools/conv_micro.py $shape > $O/p5.log 2>&1 || echo "tcp pass failed"
    python3 tools/pmc_read.py $O > $O/summary.txt
    echo "== tile $t $shape"; cat $O/plain.txt; cat $O/summary.txt
  done
done
