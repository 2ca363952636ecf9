#!/bin/bash
# Round-3 profile of the bench workload with the committed tile caches:
# per-launch conv dump, rocprofv3 kernel trace + stats (yolov3 B=16 and tiny
# B=256), the MFMA counter pass, FETCH/WRITE passes for the traffic figure.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03g
mkdir -p $OUT
ADVPATCH_LAUNCH_DUMP=$OUT/launches_yolov3.jsonl timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-tiny \
    --prec fp32 > $OUT/bench_dump.json 2> $OUT/bench_dump.err || exit 1
ADVPATCH_LAUNCH_DUMP=$OUT/launches_tiny.jsonl timeout -k 10 300 python -u bench.py --config tiny --no-cpu-baseline \
    --no-tiny --prec fp32 > $OUT/bench_dump_tiny.json 2> $OUT/bench_dump_tiny.err || exit 1
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-tiny --prec fp32"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python $B \
    > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_tiny -o run -- python $B \
    --config tiny > $OUT/bench_trace_tiny.json 2> $OUT/trace_tiny.err || exit 1
bash tools/pmc_mfma_bench.sh $OUT/mfma yolov3 16 || exit 1
bash tools/pmc_mfma_bench.sh $OUT/mfma_tiny tiny 256 || exit 1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'conv_' --output-format csv -d $OUT/pmc_fetch \
    -o run -- python $B > $OUT/bench_fetch.json 2> $OUT/pmc_fetch.err || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'conv_' --output-format csv -d $OUT/pmc_write \
    -o run -- python $B > $OUT/bench_write.json 2> $OUT/pmc_write.err || exit 1
