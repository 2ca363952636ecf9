"""Darknet cfg parsing — mirror of reference ``cfg.py:37-56`` (``parse_model_config``).

Only the parser the training path uses is provided (the reference's legacy
``parse_cfg``/``print_cfg``/load/save helpers, cfg.py:4-35,58-247, are unused
by ``darknet_v3`` and out of scope).
"""
from .cfg_gen import cfg_text

__all__ = ["parse_model_config", "parse_model_config_text"]


def parse_model_config_text(text):
    """Same semantics as reference cfg.py:37-56: comment lines dropped, one
    dict per ``[section]`` with ``type``; convolutional blocks get
    ``batch_normalize = 0`` (int) unless the cfg sets it (then the raw string)."""
    lines = [x for x in text.split("\n") if x and not x.startswith("#")]
    lines = [x.rstrip().lstrip() for x in lines]
    module_defs = []
    for line in lines:
        if not line:
            continue
        if line.startswith("["):
            module_defs.append({"type": line[1:-1].rstrip()})
            if module_defs[-1]["type"] == "convolutional":
                module_defs[-1]["batch_normalize"] = 0
        else:
            key, value = line.split("=", 1)
            module_defs[-1][key.rstrip()] = value.strip()
    return module_defs


def parse_model_config(path):
    """``path`` is a cfg file or ``builtin:<name>`` (see cfg_gen.BUILTIN)."""
    return parse_model_config_text(cfg_text(path))
