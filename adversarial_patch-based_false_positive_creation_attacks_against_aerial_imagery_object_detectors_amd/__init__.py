"""MI355X-native adversarial-patch training loop (drop-in for the hot path of
tang-agui/Adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors).

Modules mirror the reference's module names so existing code can switch by
import: ``load_data``, ``median_pool``, ``darknet_v3``, ``cfg``,
``patch_config``, ``train_patch`` (plus ``eval_patch``, the folder
evaluation of test_patch_DOTA.py).  ``install_dropin()`` registers them under
those top-level names in ``sys.modules`` (``import load_data`` then resolves
here).  The compute runs in ``libadvpatch_hip.so`` (csrc/, C ABI in
include/advpatch.h); see DESIGN.md.
"""
import importlib
import sys

DROPIN_MODULES = ("cfg", "median_pool", "load_data", "darknet_v3", "patch_config", "train_patch", "utils",
                  "utils_self", "eval_patch")


def install_dropin():
    """Make ``import load_data`` / ``from darknet_v3 import Darknet`` / ... resolve
    to this package's HIP-backed modules."""
    for name in DROPIN_MODULES:
        sys.modules[name] = importlib.import_module(__name__ + "." + name)
    return [sys.modules[n] for n in DROPIN_MODULES]


def native():
    """The loaded ctypes library (raises if libadvpatch_hip.so is not built)."""
    from . import _native
    return _native.load()
