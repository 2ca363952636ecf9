set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06g
timeout -k 10 400 python -u bench.py > gpurun_out/r06g/bench.json 2> gpurun_out/r06g/bench.err
for i in 1 2; do
  for f in 0 1; do
    ADVPATCH_WARP_FLAT=$f timeout -k 10 200 python -u bench.py --config tiny --no-cpu-baseline --no-tiny --steps 20 \
      > gpurun_out/r06g/tiny_flat$f.$i.json 2> gpurun_out/r06g/tiny_flat$f.$i.err
  done
done
timeout -k 10 300 python -u tools/step_breakdown.py --config yolov3 --steps 5 > gpurun_out/r06g/step_breakdown_yolov3_b16.txt 2>&1
timeout -k 10 300 python -u tools/step_breakdown.py --config tiny --steps 5 > gpurun_out/r06g/step_breakdown_tiny_b256.txt 2>&1
true
