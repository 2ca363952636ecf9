"""Drop the Winograd choices of a committed tile cache so the next bench run
re-times those launch shapes against every tile: mode "unboxed" (default)
drops the full-map ones (tiles 65-68, 70-72), to weigh the persistent tiles 70
(F(2x2,3x3)), 71 and 72 (F(4x4,3x3)); mode "boxed" the gradient-cone ones
(tiles 65-68, 71, 72), to weigh tiles 71/72 on boxed launches.
Usage: python tools/retune_wino.py IN.json OUT.json [unboxed|boxed]"""
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
mode = sys.argv[3] if len(sys.argv) > 3 else "unboxed"
cache = json.load(open(src))
keep = {}
for k, v in cache.items():
    key = json.loads(k)
    tile = v[0] if isinstance(v, list) else v
    boxed = bool(key[15])
    if tile in (65, 66, 67, 68, 70, 71, 72) and boxed == (mode == "boxed"):
        continue
    keep[k] = v
json.dump(keep, open(dst, "w"))
print("kept %d of %d entries" % (len(keep), len(cache)))
