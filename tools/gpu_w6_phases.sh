#!/bin/bash
# phase stamps of tiles 71 and 72 on bench shapes (stamp build in tools/abl_now)
cd "$GRAFT_REPO_ROOT"
for shape in "16 76 128 256" "16 38 256 512" "16 19 512 1024" "16 76 256 128"; do
  for t in 71 72; do
    echo "== tile $t $shape"
    W6_TILE=$t W6_MODE=res MICRO_LIB=tools/abl_now/libadvpatch_w6stamp.so timeout -k 10 120 python tools/w6_phases.py $shape 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
