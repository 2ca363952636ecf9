"""Run configurations — drop-in for reference ``patch_config.py:5-174``.

Same class names, fields, defaults and registry keys.  Differences, all about
files this environment does not have:

* ``cfgfile`` defaults to ``builtin:yolov3-dota`` (generated, see cfg_gen.py);
  a path to the reference's ``cfg/yolov3-dota.cfg`` works the same way;
* ``weightfile`` defaults to a synthetic darknet ``.weights`` file generated
  on first use (weights.py) because the pretrained file is absent;
* ``printfile`` defaults to ``builtin:30values`` (printability.py);
* ``img_dir``/``lab_dir`` keep the reference's paths and can be overridden
  with ``ADVPATCH_IMG_DIR`` / ``ADVPATCH_LAB_DIR``.
"""
import os

import torch
from torch import optim

_HERE = os.path.dirname(os.path.abspath(__file__))
SYNTH_WEIGHTS_DIR = os.environ.get("ADVPATCH_WEIGHTS_DIR", os.path.join(os.path.dirname(_HERE), "weights"))


def synthetic_weights_path(cfg_name="yolov3-dota"):
    return os.path.join(SYNTH_WEIGHTS_DIR, "%s-synthetic-seed4.weights" % cfg_name)


class BaseConfig(object):
    """Default parameters for all config files (patch_config.py:5-53)."""

    def __init__(self):
        self.img_dir = os.environ.get(
            "ADVPATCH_IMG_DIR", "/mnt/jfs/tangguijian/Data_storage/creation_patch_attackSet/trainset/images")
        self.lab_dir = os.environ.get(
            "ADVPATCH_LAB_DIR", "/mnt/jfs/tangguijian/Data_storage/creation_patch_attackSet/trainset/yolo-labels")
        self.img_dir_test = "/mnt/jfs/tangguijian/Data_storage/creation_patch_attackSet/testset/images"
        self.lab_dir_test = "/mnt/jfs/tangguijian/Data_storage/creation_patch_attackSet/testset/yolo-labels"
        self.cfgfile = "builtin:yolov3-dota"
        self.weightfile = synthetic_weights_path("yolov3-dota")
        self.printfile = "builtin:30values"
        self.patch_size = 224
        self.start_learning_rate = 0.03
        self.patch_name = "base"
        self.scheduler_factory = lambda x: optim.lr_scheduler.ReduceLROnPlateau(x, "min", patience=50)
        self.max_tv = 0
        self.batch_size = 16
        self.loss_target = lambda obj, cls: obj * cls
        self.target_loc = torch.tensor([0., 0., 0.01, 0.01])


class Experiment1(BaseConfig):
    """Model that uses a maximum total variation, tv cannot go below this point."""

    def __init__(self):
        super().__init__()
        self.patch_name = "Experiment1"
        self.max_tv = 0.165


class Experiment2HighRes(Experiment1):
    """Higher res"""

    def __init__(self):
        super().__init__()
        self.max_tv = 0.165
        self.patch_size = 400
        self.patch_name = "Exp2HighRes"


class Experiment3LowRes(Experiment1):
    """Lower res"""

    def __init__(self):
        super().__init__()
        self.max_tv = 0.165
        self.patch_size = 100
        self.patch_name = "Exp3LowRes"


class Experiment4ClassOnly(Experiment1):
    """Only minimise class score."""

    def __init__(self):
        super().__init__()
        self.batch_size = 8
        self.patch_size = 224
        self.max_tv = 0.165
        self.patch_name = "Experiment4ClassOnly"
        self.loss_target = lambda obj, cls: cls


class ObjectAndClass(BaseConfig):
    """obj_conf+cls_conf"""

    def __init__(self):
        super().__init__()
        self.batch_size = 12
        self.patch_size = 224
        self.patch_name = "ObjectAndClass"
        self.max_tv = 0.165
        self.loss_target = lambda obj, cls: (0.2 * obj + 0.8 * cls)


class ReproducePaperObj(BaseConfig):
    """Reproduce the results from the paper: Generate a patch that minimises object score."""

    def __init__(self):
        super().__init__()
        self.batch_size = 24
        self.patch_size = 224
        self.patch_name = "ObjectOnlyPaper"
        self.max_tv = 0.165
        self.loss_target = lambda obj, cls: obj


patch_configs = {
    "base": BaseConfig,
    "exp1": Experiment1,
    "obj_cls": ObjectAndClass,
    "exp2_high_res": Experiment2HighRes,
    "exp3_low_res": Experiment3LowRes,
    "exp4_class_only": Experiment4ClassOnly,
    "paper_obj": ReproducePaperObj,
}
