set -o pipefail
mkdir -p gpurun_out/w3
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wino.py -x -q --timeout 200 --timeout-method thread > gpurun_out/w3/wino.log 2>&1
rc=$?
tail -3 gpurun_out/w3/wino.log
[ $rc -eq 0 ] || exit $rc
for shp in "16 38 512 256" "16 76 256 128" "16 19 1024 512" "16 76 128 256" "16 152 128 64"; do
  echo -n "62: "; MICRO_TILE=62 timeout -k 5 60 python3 tools/conv_micro.py $shp 3 1 20 2>&1 | tail -1
done
