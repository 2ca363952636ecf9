"""Drop entries from the committed conv tile caches so that the next bench run
re-times them.  Usage:
    python tools/retune_boxed.py [--wino] <cache.json> [...]
Default: the boxed (gradient-cone gbox / support-grid) launches (re-timed on
the tuner's training-like footprints, NetPlan.tuning_rois).  --wino: also
every launch whose cached choice is a Winograd tile (a new Winograd tile
competes)."""
import json
import sys

wino = "--wino" in sys.argv
for path in [a for a in sys.argv[1:] if not a.startswith("--")]:
    with open(path) as f:
        c = json.load(f)
    keep = {}
    for k, v in c.items():
        key = json.loads(k)
        boxed = bool(key[15]) or "mrows" in key
        tile = v[0] if isinstance(v, list) else v
        if not boxed and not (wino and 61 <= tile <= 68):
            keep[k] = v
    with open(path, "w") as f:
        json.dump(keep, f)
    print("%s: %d -> %d entries" % (path, len(c), len(keep)))
