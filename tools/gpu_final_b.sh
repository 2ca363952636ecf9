#!/bin/bash
# round-end: full -m gpu suite, default bench line, steady-state profiles of both configs
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${FINAL_OUT:-final2}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_full.txt 2>&1 || { tail -30 $OUT/tests_full.txt; exit 1; }
tail -1 $OUT/tests_full.txt
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -1 $OUT/bench.json | cut -c1-300
bash tools/profile_round.sh r05 yolov3 16 fp32
bash tools/profile_round.sh r05 tiny 256 fp32
