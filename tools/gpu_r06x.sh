# head tails on a second stream (ADVPATCH_STREAMS=1) vs one stream: interleaved bench A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06x}; mkdir -p $O
for rep in 1 2 3; do
  for v in 1 0; do
    ADVPATCH_STREAMS=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 \
      > $O/bench_st$v.$rep.json 2> $O/bench_st$v.$rep.err || { tail $O/bench_st$v.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3), round(d.get('value_tiny',0)), round(d.get('ms_per_step_tiny',0),3))" $O/bench_st$v.$rep.json
  done
done
