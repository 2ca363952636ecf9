#!/bin/bash
# Round-3 final profiles of the tiny B=256 workload (tile 69 changed it): kernel trace + stats,
# FETCH/WRITE passes (tools/profile_round.sh), MFMA busy counters, per-launch conv timings.
cd "$GRAFT_REPO_ROOT"
PKG=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd
OUT=gpurun_out/r03_final
mkdir -p $OUT
bash tools/profile_round.sh r03 tiny 256 fp32 > $OUT/profile_tiny.log 2>&1 || { tail -5 $OUT/profile_tiny.log; exit 1; }
bash tools/pmc_mfma_bench.sh gpurun_out/r03_final/mfma_tiny tiny 256 > $OUT/mfma_tiny.log 2>&1 || { tail -5 $OUT/mfma_tiny.log; exit 1; }
ADVPATCH_LAUNCH_DUMP=$OUT/launches_tiny.jsonl timeout -k 10 300 python -u bench.py --config tiny --batch 256 --steps 5 \
    --warmup 2 --no-cpu-baseline --prec fp32 > $OUT/bench_tiny_dump.json 2> $OUT/bench_tiny_dump.err || exit 1
ls $OUT
