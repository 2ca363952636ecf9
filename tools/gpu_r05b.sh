# tile 71 (F(4x4,3x3)): diagnostics, correctness tests, then per-shape timing against tile 70
set -o pipefail
mkdir -p gpurun_out/r05b

timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_wino6.py \
  > gpurun_out/r05b/tests.log 2>&1 || exit 1
for shp in "16 304 32 64" "16 152 64 128" "16 76 128 256" "16 38 256 512" "16 19 512 1024" "16 38 512 256"; do
  for t in 70 71; do
    for ks in 1 2 3; do
      echo "tile $t ks $ks: $(MICRO_TILE=$t MICRO_KSPLIT=$ks MICRO_RES=1 timeout -k 5 60 python tools/conv_micro.py $shp 3 1 30 2>&1 | tail -1)" >> gpurun_out/r05b/micro.txt || exit 1
    done
  done
done
