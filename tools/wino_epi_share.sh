#!/bin/bash
# Share of the Winograd tile-65 launch time spent outside the k-loop (GPU box):
# builds the PO_ABLATE_WINO_NOEPI variant (prologue + k-loop only) and times
# both libraries on the yolov3@608 B=16 stride-1 3x3 shapes (MICRO_RES=1: the
# fused-shortcut epilogue of the residual convs).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
LIB=$(bash "$ROOT/tools/build_ablate.sh" noepi -DPO_ABLATE_WINO_NOEPI | tail -1)
for shp in "16 152 64 128" "16 76 128 256" "16 38 256 512" "16 19 512 1024"; do
  full=$(MICRO_RES=1 MICRO_TILE=65 timeout -k 5 60 python3 "$ROOT/tools/conv_micro.py" $shp 3 1 20 2>&1 | tail -1)
  kl=$(MICRO_LIB=$LIB MICRO_RES=1 MICRO_TILE=65 timeout -k 5 60 python3 "$ROOT/tools/conv_micro.py" $shp 3 1 20 2>&1 | tail -1)
  echo "full:   $full"
  echo "k-loop: $kl"
done
