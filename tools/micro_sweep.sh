set -e
for T in 128x128x16 128x128x16g 128x128x32 128x128x32g 64x128x16g; do
for SH in "16 64 128 256 3 1 20" "32 64 128 256 3 1 20" "16 76 128 256 3 1 20" "8 64 128 256 3 1 20" "16 64 256 256 3 1 20" "16 64 512 512 3 1 20"; do
  ADVPATCH_CONV_TILE=$T timeout -k 10 60 python tools/conv_micro.py $SH | grep -v amdgpu.ids | sed "s/^/$T /"
done; done
