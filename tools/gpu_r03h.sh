#!/bin/bash
# Footprint-box warp kernels: patch-op tests + the tiny step parity; warp
# micro-benchmark; PMC of Winograd tile 68 on a long-K and a short-K shape.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_patch_ops.py \
    tests/test_gpu_first_conv.py "tests/test_gpu_step.py::test_step_tiny_416" > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/warp_micro.py > $OUT/warp_micro.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/warp_micro.py 256 416 224 20 > $OUT/warp_micro_tiny.txt 2>&1 || exit 1
MICRO_TILE=68 bash tools/pmc_conv.sh $OUT/pmc68_76 "16 76 128 256 3 1 30" 68 > $OUT/pmc68_76.log 2>&1 || exit 1
MICRO_TILE=68 bash tools/pmc_conv.sh $OUT/pmc68_304 "16 304 32 64 3 1 10" 68 > $OUT/pmc68_304.log 2>&1 || exit 1
python tools/pmc_read.py $OUT/pmc68_76 > $OUT/pmc68_76.txt
python tools/pmc_read.py $OUT/pmc68_304 > $OUT/pmc68_304.txt
