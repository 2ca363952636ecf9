#!/bin/bash
# Ablation builds of libadvpatch_hip.so into tools/bin/ (git-ignored):
#   tools/build_ablate.sh TAG -DMACRO [...]  ->  tools/bin/libadvpatch_TAG.so
set -e
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/csrc
OUT=${OUT:-$ROOT/tools/abl}; case $OUT in /*) ;; *) OUT=$ROOT/$OUT;; esac
TMP=$(mktemp -d)
mkdir -p "$OUT"
for f in "$SRC"/*.hip; do
  b=$(basename "$f" .hip)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Wno-inline-asm "$@" -c "$f" -o "$TMP/$b.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libadvpatch_$TAG.so" "$TMP"/*.o
rm -rf "$TMP"
echo "$OUT/libadvpatch_$TAG.so"
