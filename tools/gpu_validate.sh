#!/bin/bash
# Full -m gpu suite, default bench line, boxed-launch split probe (yolov3, tiny).
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-r03u}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cut -c1-300 $OUT/bench.json
