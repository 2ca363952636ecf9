# Round measurement on one GPU box: benches (yolov3 B=16 with the CPU baseline,
# tiny B=256), tile caches copied out (profiles: tools/profile_round.sh, one call each).
set -o pipefail
R=${1:-r02}
PKG=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd
mkdir -p gpurun_out/meas_$R/tiles
echo "bench yolov3"; timeout -k 10 600 python3 -u bench.py > gpurun_out/meas_$R/bench_yolov3_b16.json 2> gpurun_out/meas_$R/bench_yolov3.err || exit 1
echo "bench tiny"; timeout -k 10 600 python3 -u bench.py --config tiny --no-cpu-baseline > gpurun_out/meas_$R/bench_tiny_b256.json 2> gpurun_out/meas_$R/bench_tiny.err || exit 1
cp $PKG/tiles/*.json gpurun_out/meas_$R/tiles/
echo done
