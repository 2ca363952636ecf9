# tile 66 with 1/2/3 input-channel slices (split-K + conv_reduce_k) against tile 65 on the
# yolov3@608 B=16 Winograd shapes.  Usage: bash tools/wino_split_cmp.sh
set -e
for shp in "16 19 512 1024" "16 19 1024 512" "16 38 512 256" "16 38 256 512" "16 76 256 128"; do
  echo -n "$shp tile 65: "; MICRO_TILE=65 timeout -k 5 60 python3 tools/conv_micro.py $shp 3 1 20 2>&1 | tail -1
  for k in 1 2 3; do
    echo -n "$shp tile 66 ksplit $k: "; MICRO_TILE=66 MICRO_KSPLIT=$k timeout -k 5 60 python3 tools/conv_micro.py $shp 3 1 20 2>&1 | tail -1
  done
done
