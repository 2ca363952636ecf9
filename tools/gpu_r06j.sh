set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06j
ADVPATCH_GEOMETRY=ref timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06j/ref -o run -- \
  python bench.py --config tiny --no-cpu-baseline --no-tiny --steps 5 --warmup 2 > gpurun_out/r06j/ref.json 2> gpurun_out/r06j/ref.err && \
ADVPATCH_GEOMETRY=f64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06j/f64 -o run -- \
  python bench.py --config tiny --no-cpu-baseline --no-tiny --steps 5 --warmup 2 > gpurun_out/r06j/f64.json 2> gpurun_out/r06j/f64.err
