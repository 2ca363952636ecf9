set -o pipefail
mkdir -p gpurun_out/w4
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -q --timeout 200 --timeout-method thread > gpurun_out/w4/wino.log 2>&1
rc=$?
tail -3 gpurun_out/w4/wino.log
[ $rc -eq 0 ] || exit $rc
for shp in "16 38 512 256" "16 38 256 512" "16 76 256 128" "16 76 128 256" "16 19 1024 512" "16 19 512 1024" "16 152 128 64" "16 152 64 128"; do
  for t in 62 63; do echo -n "$t: "; MICRO_TILE=$t timeout -k 5 60 python3 tools/conv_micro.py $shp 3 1 20 2>&1 | tail -1; done
done
