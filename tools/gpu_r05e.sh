set -o pipefail
mkdir -p gpurun_out/r05e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wino6.py > gpurun_out/r05e/tests.log 2>&1 || exit 1
for m in res y resy; do for s in "16 76 128 256" "16 152 64 128" "16 19 512 1024"; do W6_MODE=$m MICRO_LIB=tools/abl_push/libadvpatch_w6stamp.so timeout -k 5 60 python tools/w6_phases.py $s || exit 1; done; done > gpurun_out/r05e/phases.txt 2>&1
for shp in "16 304 32 64" "16 152 64 128" "16 76 128 256" "16 38 256 512" "16 19 512 1024"; do
  for t in 70 71; do
    echo "tile $t: $(MICRO_TILE=$t MICRO_RES=1 timeout -k 5 60 python tools/conv_micro.py $shp 3 1 30 2>&1 | tail -1)" >> gpurun_out/r05e/micro.txt || exit 1
  done
done
