"""Drop the unboxed Winograd choices (tiles 65-68, 70) of a committed tile
cache so the next bench run re-times those launch shapes against every tile,
the persistent tiles 70 (F(2x2,3x3)) and 71 (F(4x4,3x3)) included; boxed
launches (gradient cones) keep their choice (tiles 70/71 run full maps only).
Usage: python tools/retune_wino.py IN.json OUT.json"""
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
cache = json.load(open(src))
keep = {}
for k, v in cache.items():
    key = json.loads(k)
    tile = v[0] if isinstance(v, list) else v
    boxed = bool(key[15])
    if tile in (65, 66, 67, 68, 70) and not boxed:
        continue
    keep[k] = v
json.dump(keep, open(dst, "w"))
print("kept %d of %d entries" % (len(keep), len(cache)))
