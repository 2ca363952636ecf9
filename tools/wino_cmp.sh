# Winograd tile timings (tools/conv_micro.py) on the yolov3@608 B=16 3x3 stride-1 shapes; MICRO_RES=1 adds
# the fused shortcut epilogue.  Usage: TILES="63 64" bash tools/wino_cmp.sh
set -e
for shp in "16 152 64 128" "16 76 128 256" "16 76 256 128" "16 38 256 512" "16 38 512 256" "16 19 512 1024" "16 19 1024 512"; do
  for t in ${TILES:-63 64}; do
    echo -n "$shp tile $t res=${MICRO_RES:-0}: "; MICRO_TILE=$t timeout -k 5 60 python3 tools/conv_micro.py $shp 3 1 20 2>&1 | tail -1
  done
done
