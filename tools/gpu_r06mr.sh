# multi-rank rehearsal on one GPU: bench.py's rank launch, per-rank shards and the fused all-reduce (gloo),
# two ranks sharing cuda:0 (the RCCL path needs one GPU per rank)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06mr; mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-cpu-baseline --no-tiny \
  > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { tail -20 $O/bench_gloo2.err; exit 1; }
cut -c1-400 $O/bench_gloo2.json
