set -e
for T in 128x128x16 128x128x16g 128x128x32g; do
for SH in "16 64 128 256 3 1 20" "16 64 512 512 3 1 20" "16 76 128 256 3 1 20"; do
  ADVPATCH_CONV_TILE=$T timeout -k 10 60 python tools/conv_micro.py $SH | grep -v amdgpu.ids | sed "s/^/$T full   /"
  MICRO_LIB=tools/bin/libadvpatch_noload.so ADVPATCH_CONV_TILE=$T timeout -k 10 60 python tools/conv_micro.py $SH | grep -v amdgpu.ids | sed "s/^/$T noload /"
done; done
