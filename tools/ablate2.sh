set -e
for T in 128x128x16; do
for SH in "16 64 16 256 1 1 20" "16 64 64 256 1 1 20" "16 64 256 256 1 1 20" "16 64 1024 256 1 1 20" "16 64 128 256 3 1 20"; do
  ADVPATCH_CONV_TILE=$T timeout -k 10 60 python tools/conv_micro.py $SH | grep -v amdgpu.ids | sed "s/^/$T full   /"
  MICRO_LIB=tools/bin/libadvpatch_noload.so ADVPATCH_CONV_TILE=$T timeout -k 10 60 python tools/conv_micro.py $SH | grep -v amdgpu.ids | sed "s/^/$T noload /"
done; done
