#!/bin/bash
# Direct conv_k tiles on the yolov3@608 B=16 stride-2 3x3 and 1x1 shapes: the
# current library against tools/bin/libadvpatch_oldk.so (the previous conv_k).
# Usage: OUT=file bash tools/direct_cmp.sh
OUT=${OUT:-/dev/stdout}
for shp in "16 608 32 64 3 2" "16 304 64 128 3 2" "16 152 128 256 3 2" "16 76 256 512 3 2" "16 38 512 1024 3 2" \
           "16 304 64 32 1 1" "16 152 128 64 1 1" "16 76 256 128 1 1" "16 38 512 256 1 1"; do
  for t in 3 4 5 6 7 9 13 14 15 16 17 19; do
    for lib in new old; do
      if [ $lib = old ]; then L=tools/bin/libadvpatch_oldk.so; else L=""; fi
      r=$(MICRO_LIB=$L MICRO_TILE=$t timeout -k 5 60 python3 tools/conv_micro.py $shp 20 2>&1 | tail -1) || exit 1
      echo "$shp tile $t $lib: $r" >> $OUT
    done
  done
done
