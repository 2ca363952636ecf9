#!/bin/bash
# Head tails on a second stream: bit-identity tests, then interleaved A/B (A: streams, B: ADVPATCH_STREAMS=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAGOUT:-r04f}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino5.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_w5.log 2>&1
rc=$?; tail -2 $OUT/tests_w5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_step.py -x -v -s --timeout 600 --timeout-method thread -k "head_tails or windowed or tiny_416" > $OUT/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|patch grad|plan:" $OUT/tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
AB_ENV="ADVPATCH_STREAMS=0" timeout -k 10 900 tools/gpu_ab.sh ${TAGOUT:-r04f}/ab 2
