"""Builtin darknet network definitions, emitted as darknet-format cfg text.

The reference ships its networks as cfg files (`cfg/yolov3-dota.cfg`,
`cfg/yolov3-tiny.cfg`) that `darknet_v3.Darknet(path)` parses through
`cfg.parse_model_config` (reference `cfg.py:37-56`).  This module *generates*
equivalent definitions from the architecture recipe instead of carrying copies
of those files:

* ``yolov3(classes)``  - Darknet-53 backbone + 3 YOLO heads (19/38/76 at 608),
  the layer sequence of reference `cfg/yolov3-dota.cfg` (107 blocks: 75 conv,
  23 shortcut, 4 route, 2 upsample, 3 yolo; heads at blocks 82/94/106).
* ``yolov3_tiny(classes)`` - the 24-block tiny network of reference
  `cfg/yolov3-tiny.cfg` (2 heads at 13/26 for 416 input), generalised to any
  class count (the 80-class file cannot feed the 20-channel loss
  head, config 5 uses classes=15).
* ``mini3(classes)`` - a 34-block test network with every block kind of the
  yolov3 path (3x3 s1/s2, 1x1, shortcut, 1- and 2-input route, upsample,
  3 yolo heads) used for fast parity fixtures.

`Darknet` accepts either a filesystem path or one of ``builtin:<name>``.
"""

DOTA_ANCHORS = "15,31, 19,12, 28,40, 40,20, 43,38, 42,87, 78,54, 95,102, 181,206"
TINY_ANCHORS = "10,14, 23,27, 37,58, 81,82, 135,169, 344,319"


def _net(width, height=None):
    height = width if height is None else height
    # create_modules (reference darknet_v3.py:14-29) requires all of these keys.
    return ("[net]\nbatch=1\nsubdivisions=1\nwidth=%d\nheight=%d\nchannels=3\n"
            "momentum=0.9\ndecay=0.0005\nlearning_rate=0.001\nburn_in=1000\n"
            "max_batches=500200\npolicy=steps\nsteps=400000,450000\nscales=.1,.1\n\n"
            % (width, height))


def _conv(filters, size, stride=1, bn=True, act="leaky"):
    s = "[convolutional]\n"
    if bn:
        s += "batch_normalize=1\n"
    s += "filters=%d\nsize=%d\nstride=%d\npad=1\nactivation=%s\n\n" % (filters, size, stride, act)
    return s


def _shortcut(frm=-3):
    return "[shortcut]\nfrom=%d\nactivation=linear\n\n" % frm


def _route(*layers):
    return "[route]\nlayers=%s\n\n" % ",".join(str(l) for l in layers)


def _upsample(stride=2):
    return "[upsample]\nstride=%d\n\n" % stride


def _maxpool(size, stride):
    return "[maxpool]\nsize=%d\nstride=%d\n\n" % (size, stride)


def _yolo(mask, anchors, classes, num):
    return ("[yolo]\nmask=%s\nanchors=%s\nclasses=%d\nnum=%d\njitter=.3\n"
            "ignore_thresh=.7\ntruth_thresh=1\nrandom=1\n\n" % (mask, anchors, classes, num))


def yolov3(classes=15, width=608):
    head = 3 * (5 + classes)
    t = _net(width)
    t += _conv(32, 3)
    for filters, nblocks in ((64, 1), (128, 2), (256, 8), (512, 8), (1024, 4)):
        t += _conv(filters, 3, 2)
        for _ in range(nblocks):
            t += _conv(filters // 2, 1) + _conv(filters, 3) + _shortcut(-3)
    for _ in range(3):
        t += _conv(512, 1) + _conv(1024, 3)
    t += _conv(head, 1, bn=False, act="linear") + _yolo("6,7,8", DOTA_ANCHORS, classes, 9)
    t += _route(-4) + _conv(256, 1) + _upsample(2) + _route(-1, 61)
    for _ in range(3):
        t += _conv(256, 1) + _conv(512, 3)
    t += _conv(head, 1, bn=False, act="linear") + _yolo("3,4,5", DOTA_ANCHORS, classes, 9)
    t += _route(-4) + _conv(128, 1) + _upsample(2) + _route(-1, 36)
    for _ in range(3):
        t += _conv(128, 1) + _conv(256, 3)
    t += _conv(head, 1, bn=False, act="linear") + _yolo("0,1,2", DOTA_ANCHORS, classes, 9)
    return t


def yolov3_tiny(classes=15, width=416):
    head = 3 * (5 + classes)
    t = _net(width)
    for i, f in enumerate((16, 32, 64, 128, 256)):
        t += _conv(f, 3) + _maxpool(2, 2)
    t += _conv(512, 3) + _maxpool(2, 1)
    t += _conv(1024, 3) + _conv(256, 1) + _conv(512, 3)
    t += _conv(head, 1, bn=False, act="linear") + _yolo("3,4,5", TINY_ANCHORS, classes, 6)
    t += _route(-4) + _conv(128, 1) + _upsample(2) + _route(-1, 8)
    t += _conv(256, 3) + _conv(head, 1, bn=False, act="linear") + _yolo("0,1,2", TINY_ANCHORS, classes, 6)
    return t


def mini3(classes=15, width=64):
    head = 3 * (5 + classes)
    t = _net(width)
    t += _conv(16, 3)                                         # 0
    t += _conv(32, 3, 2) + _conv(16, 1) + _conv(32, 3) + _shortcut()    # 1-4
    t += _conv(64, 3, 2) + _conv(32, 1) + _conv(64, 3) + _shortcut()    # 5-8
    t += _conv(128, 3, 2) + _conv(64, 1) + _conv(128, 3) + _shortcut()  # 9-12
    t += _conv(128, 3, 2) + _conv(64, 1) + _conv(128, 3)       # 13-15
    t += _conv(head, 1, bn=False, act="linear") + _yolo("6,7,8", DOTA_ANCHORS, classes, 9)  # 16-17
    t += _route(-4) + _conv(32, 1) + _upsample(2) + _route(-1, 12)       # 18-21
    t += _conv(64, 1) + _conv(128, 3)                                      # 22-23
    t += _conv(head, 1, bn=False, act="linear") + _yolo("3,4,5", DOTA_ANCHORS, classes, 9)  # 24-25
    t += _route(-4) + _conv(32, 1) + _upsample(2) + _route(-1, 8)         # 26-29
    t += _conv(32, 1) + _conv(64, 3)                                       # 30-31
    t += _conv(head, 1, bn=False, act="linear") + _yolo("0,1,2", DOTA_ANCHORS, classes, 9)  # 32-33
    return t


BUILTIN = {
    "yolov3-dota": lambda: yolov3(15, 608),
    "yolov3-dota-416": lambda: yolov3(15, 416),
    "yolov3-tiny-dota": lambda: yolov3_tiny(15, 416),
    "mini3": lambda: mini3(15, 64),
    "mini3-96": lambda: mini3(15, 96),
}


def cfg_text(name_or_path):
    """Return cfg text for ``builtin:<name>`` or read it from a file path."""
    if isinstance(name_or_path, str) and name_or_path.startswith("builtin:"):
        key = name_or_path[len("builtin:"):]
        if key not in BUILTIN:
            raise KeyError("unknown builtin network %r (have %s)" % (key, sorted(BUILTIN)))
        return BUILTIN[key]()
    with open(name_or_path, "r") as f:
        return f.read()
