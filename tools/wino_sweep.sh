# Winograd (tile 61) vs direct tiles on the yolov3@608 B=16 3x3 stride-1 shapes
set -e
for shp in "16 304 32 64" "16 304 64 32" "16 152 64 128" "16 152 128 64" "16 76 128 256" "16 76 256 128" "16 38 256 512" "16 38 512 256" "16 19 512 1024" "16 19 1024 512"; do
  for t in ${TILES:-61 62 1 4 5 11 13 15 17}; do
    echo -n "tile $t: "; MICRO_TILE=$t timeout -k 5 60 python3 tools/conv_micro.py $shp 3 1 20 2>&1 | tail -1
  done
done
