#!/bin/bash
# Per-shape PMC of the dominant kernels at the round-3 head: tile 68 (yolov3 Winograd) at
# 152^2 64->128, 76^2 128->256, 38^2 256->512; tile 69 (tiny 208^2 16->32 + pool).
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_pmc
mkdir -p $OUT
for s in "152 64 128" "76 128 256" "38 256 512"; do
  set -- $s
  bash tools/pmc_conv.sh $OUT/t68_$1 "16 $1 $2 $3 3 1 20" 68 > $OUT/t68_$1.log 2>&1 || exit 1
  python tools/pmc_read.py $OUT/t68_$1 > $OUT/t68_$1.txt
done
MICRO_POOL=1 bash tools/pmc_conv.sh $OUT/t69_208 "256 208 16 32 3 1 10" 69 > $OUT/t69_208.log 2>&1 || exit 1
python tools/pmc_read.py $OUT/t69_208 > $OUT/t69_208.txt
ls $OUT
