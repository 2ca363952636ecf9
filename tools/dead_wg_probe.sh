cd "$GRAFT_REPO_ROOT"
for f in 0 0.1 0.25 0.5 1.0; do
  echo "box $f"; MICRO_TILE=9 MICRO_BOX=$f timeout -k 5 60 python tools/conv_micro.py 16 304 64 32 1 1 30 || exit 1
  MICRO_TILE=11 MICRO_BOX=$f timeout -k 5 60 python tools/conv_micro.py 16 76 256 128 1 1 30 || exit 1
done
echo "no box"; MICRO_TILE=9 timeout -k 5 60 python tools/conv_micro.py 16 304 64 32 1 1 30
