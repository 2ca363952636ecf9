# tiles 71/72 with the fused pool (EF_POOL): bit-identity tests, then micro vs tile 70 on tiny's pooled launches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06t71p2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wino6.py -k "fused_pool" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for shape in "256 104 32 64 3 1 20" "256 52 64 128 3 1 20"; do
  for t in 70 71 72 70 71 72; do
    r=$(MICRO_TILE=$t MICRO_POOL=1 timeout -k 10 120 python -u tools/conv_micro.py $shape 2>&1 | grep -v amdgpu.ids | tail -1) || { echo "$shape $t failed: $r"; exit 1; }
    echo "$shape tile ${t}p: $r" | tee -a $O/micro.txt
  done
done
