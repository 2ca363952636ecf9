cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export MICRO_PREC=1
for shape in "16 76 128 256 3 1 30" "16 38 256 512 3 1 30" "16 304 32 64 3 1 20" "16 19 512 1024 3 1 30"; do
  for t in 34 36 53 55 56 57 58 59 60; do
    MICRO_TILE=$t timeout -k 5 60 python tools/conv_micro.py $shape 2>&1 | tail -n 1 | sed "s/^/tile $t: /"
  done
done
