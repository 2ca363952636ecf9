#!/bin/bash
# Build A/B variants of one HIP source into tools/var/<name>/libadvpatch_hip.so
# (the other objects from csrc/build), for ADVPATCH_LIB=... runs on the GPU box.
# Usage: tools/build_variants.sh SOURCE "name:-DFLAG=1 -DOTHER" ["name2:..."]
set -e
PKG=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd
SRC=$1; shift
C=$PKG/csrc
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -Wno-inline-asm -munsafe-fp-atomics"
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}
  mkdir -p tools/var/$name
  (/opt/rocm/bin/hipcc $FLAGS $defs -c ${SRCFILE:-$C/$SRC.hip} -o tools/var/$name/$SRC.o &&
   objs=$(ls $C/build/*.o | grep -v "/$SRC.o") &&
   /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/var/$name/libadvpatch_hip.so tools/var/$name/$SRC.o $objs &&
   rm tools/var/$name/$SRC.o && echo "built $name") &
done
wait
