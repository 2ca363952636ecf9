#!/bin/bash
# PMC of tile 71 (conv_wino6_k, F(4x4,3x3)) beside tile 70 on bench shapes
set -e
cd "$GRAFT_REPO_ROOT"
for shape in "16 76 128 256 3 1 20" "16 19 512 1024 3 1 20"; do
  tag=$(echo $shape | awk '{print $2}')
  for t in 71 70; do
    MICRO_RES=1 bash tools/pmc_conv.sh gpurun_out/pmc_t${t}_$tag "$shape" $t
    MICRO_TILE=$t MICRO_RES=1 timeout -k 10 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-include-regex 'conv_' \
        --output-format csv -d gpurun_out/pmc_t${t}_$tag/p4 -o p4 -- python tools/conv_micro.py $shape > gpurun_out/pmc_t${t}_$tag/p4.log 2>&1
    python3 tools/pmc_read.py gpurun_out/pmc_t${t}_$tag > gpurun_out/pmc_t${t}_$tag/summary.txt
    echo "== tile $t $shape"; cat gpurun_out/pmc_t${t}_$tag/plain.txt; cat gpurun_out/pmc_t${t}_$tag/summary.txt
  done
done
