# would F(4x4) (tiles 71/72) beat tile 70 on tiny's pooled 104^2 32->64 and 52^2 64->128 launches? (unpooled proxies)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06t71p; mkdir -p $O
for shape in "256 104 32 64 3 1 20" "256 52 64 128 3 1 20" "256 208 16 32 3 1 20"; do
  for t in 70p 70 71 72 73p; do
    tile=${t%p}; pool=0; [ "$t" != "$tile" ] && pool=1
    if [ "$tile" = 73 ] && [ "${shape:4:3}" != "208" ]; then continue; fi
    r=$(MICRO_TILE=$tile MICRO_POOL=$pool timeout -k 10 120 python -u tools/conv_micro.py $shape 2>&1 | grep -v amdgpu.ids | tail -1) || { echo "$shape $t failed: $r"; continue; }
    echo "$shape tile $t: $r" | tee -a $O/micro.txt
  done
done
