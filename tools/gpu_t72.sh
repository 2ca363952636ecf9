#!/bin/bash
# tile 72 (pre-transformed F(4x4)) beside tile 71 on the bench's shapes, interleaved
cd "$GRAFT_REPO_ROOT"
OUT=$1
: > $OUT
for rnd in 1 2; do
  for shape in "16 304 32 64 3 1 20" "16 152 64 128 3 1 20" "16 76 128 256 3 1 20" "16 76 256 128 3 1 20" "16 38 256 512 3 1 20" "16 38 512 256 3 1 20" "16 19 512 1024 3 1 20" "16 19 1024 512 3 1 20"; do
    for t in 71 72; do
      r=$(MICRO_TILE=$t MICRO_RES=1 timeout -k 10 120 python tools/conv_micro.py $shape 2>/dev/null | tail -1) || exit 1
      echo "r$rnd t$t $r" | tee -a $OUT
    done
  done
done
