#!/bin/bash
# Re-entry check of the round-3 head: full -m gpu suite, then the default bench line.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03i
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json | cut -c1-400
