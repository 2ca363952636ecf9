#!/bin/bash
# Interleaved micro timings of tile-71 variant libraries (tools/abl_now/libadvpatch_<tag>.so)
# on the bench's F(4x4) shapes:  TAGS="w6base w6v1" bash tools/gpu_w6_variants.sh OUTFILE
cd "$GRAFT_REPO_ROOT"
OUT=$1
: > $OUT
for rnd in 1 2; do
  for shape in "16 304 64 64 3 1 20" "16 152 128 128 3 1 20" "16 76 128 256 3 1 20" "16 76 256 128 3 1 20" "16 38 256 512 3 1 20" "16 19 512 1024 3 1 20"; do
    for tag in $TAGS; do
      r=$(MICRO_LIB=tools/abl_now/libadvpatch_$tag.so MICRO_TILE=71 MICRO_RES=1 timeout -k 10 120 python tools/conv_micro.py $shape 2>/dev/null | tail -1) || exit 1
      echo "r$rnd $tag $r" | tee -a $OUT
    done
  done
done
