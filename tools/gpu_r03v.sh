#!/bin/bash
# First layer on the matrix cores: first-conv tests, timings against HEAD's VALU kernels.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03v
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_first_conv.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for lib in head new head new; do
  L=tools/abl/libadvpatch_head.so; [ $lib = new ] && L=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/libadvpatch_hip.so
  echo "$lib:" >> $OUT/micro.txt
  MICRO_LIB=$L timeout -k 5 60 python3 tools/first_micro.py 20 2>&1 | grep -v amdgpu >> $OUT/micro.txt || exit 1
done
cat $OUT/micro.txt
