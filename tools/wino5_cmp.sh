#!/bin/bash
# Tile 70 (persistent conv_wino5_k) against tile 68 on the yolov3@608 B=16 Winograd shapes (tools/conv_micro.py),
# interleaved; MICRO_RES=1 adds the fused-shortcut epilogue.  Usage: bash tools/wino5_cmp.sh
for shp in "16 304 32 64" "16 152 64 128" "16 76 128 256" "16 38 256 512" "16 19 512 1024" "16 19 1024 512"; do
  for t in 68 70 68 70; do
    echo -n "$shp tile $t: "; MICRO_TILE=$t timeout -k 5 60 python3 tools/conv_micro.py $shp 3 1 20 2>&1 | tail -1
  done
done
