#!/bin/bash
# Tile 69 (halo pool conv): bit-identity tests, pooled-launch timings against the generic tiles.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03s
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_halo.py \
    "tests/test_gpu_wino.py::test_wino_fused_pool" > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for t in 69 9 19 5 66; do
  echo -n "tile $t: " >> $OUT/micro.txt
  MICRO_POOL=1 MICRO_TILE=$t timeout -k 5 60 python3 tools/conv_micro.py 256 208 16 32 3 1 20 2>&1 | tail -1 >> $OUT/micro.txt || exit 1
done
cat $OUT/micro.txt
