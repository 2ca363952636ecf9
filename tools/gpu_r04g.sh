#!/bin/bash
# Round-4 checkpoint: the full -m gpu suite, the default bench line, then the
# rocprof profile of both bench configs (tools/profile_round.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAGOUT:-r04g}
mkdir -p $OUT
(while sleep 45; do echo "tick $(date +%T)"; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread ${TESTSEL:-} > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
[ "${PROFILE:-1}" = 1 ] || exit 0
bash tools/profile_round.sh r04 yolov3 16 fp32 > $OUT/prof_y.log 2>&1 || { echo "profile yolov3 failed"; tail -20 $OUT/prof_y.log; exit 1; }
bash tools/profile_round.sh r04 tiny 256 fp32 > $OUT/prof_t.log 2>&1 || { echo "profile tiny failed"; tail -20 $OUT/prof_t.log; exit 1; }
echo done
