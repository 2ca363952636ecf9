#!/bin/bash
# round-end: printed parity of the bench-path step tests + the default bench line
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/final
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_train.py -m gpu -s -v --timeout 300 --timeout-method thread \
  -k "headline_plan or tiny_bench_plan or targeted or objectives or tiny_416 or empty_shard" > $OUT/parity.txt 2>&1
grep -E "plan|targeted|tiny|PASSED|FAILED|passed|failed" $OUT/parity.txt | tail -40
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -1 $OUT/bench.json | cut -c1-400
