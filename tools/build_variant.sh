#!/bin/bash
# Build libadvpatch_TAG.so into tools/abl/ from the package sources with some
# files replaced (ablation against another revision):
#   tools/build_variant.sh TAG [REV:file.hip | /path/to/file.hip] ... [-- -DMACRO ...]
set -e
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd
SRC=$ROOT/$PKG/csrc
TMP0=$(mktemp -d); TMP=$TMP0/a/b; mkdir -p $TMP $TMP0/include; cp $ROOT/include/*.h $TMP0/include/
cp "$SRC"/*.hip "$SRC"/*.h "$TMP"/
FLAGS=()
while [ $# -gt 0 ]; do
  case "$1" in
    --) shift; FLAGS=("$@"); break ;;
    *:*) rev=${1%%:*}; f=${1#*:}; git -C "$ROOT" show "$rev:$PKG/csrc/$f" > "$TMP/$f" ;;
    *) cp "$1" "$TMP/$(basename "$1")" ;;
  esac
  shift
done
mkdir -p "$ROOT/tools/abl"
for f in "$TMP"/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Wno-inline-asm "${FLAGS[@]}" \
      -c "$f" -o "${f%.hip}.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/tools/abl/libadvpatch_$TAG.so" "$TMP"/*.o
rm -rf "$TMP0"
echo "$ROOT/tools/abl/libadvpatch_$TAG.so"
