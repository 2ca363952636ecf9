"""Generate the committed golden fixtures from the oracle (PyTorch-CPU
restatement of the reference path).  Inputs are seeded synthetic data, so a
fixture stores the seeds plus the outputs:

    python tests/golden/make_golden.py

golden_mini3.npz       mini3 net, S=64, P=32, B=4, seeds frames 0 / labels 1 / patch 2 / draws 3 / weights 4
golden_yolov3_608.npz  yolov3-dota, S=608, P=224, B=1, seeds 40/41/42/43, weights 4
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import __graft_entry__ as ge  # noqa: E402
import oracle  # noqa: E402

CASES = {
    "mini3": dict(cfg="builtin:mini3", B=4, P=32, seeds=(0, 1, 2, 3), full_grad=True),
    "yolov3_608": dict(cfg="builtin:yolov3-dota", B=1, P=224, seeds=(40, 41, 42, 43), full_grad=False),
}


def compute(name):
    c = CASES[name]
    sy, W, G, ld = ge._pkg("synthetic"), ge._pkg("weights"), ge._pkg("cfg_gen"), ge._pkg("load_data")
    net = oracle.OracleDarknet(G.cfg_text(c["cfg"]), W.synthesize(c["cfg"], seed=4))
    S, B, P = net.height, c["B"], c["P"]
    sf, sl, sp, sd = c["seeds"]
    img, lab, patch, dr = sy.frames(B, S, seed=sf), sy.labels(B, seed=sl), sy.patch(P, seed=sp), sy.draws(B, P, seed=sd)
    r = oracle.train_step(patch, img, lab, dr, net, ld.load_printability_colors("builtin:30values"))
    g = r["grad"].numpy()
    out = {k: np.float32(float(r[k])) for k in ("loss", "nps_loss", "tv_loss", "no_obj_loss", "no_cls_loss",
                                                "colorful_loss")}
    out.update(patch_center=r["patch_center"].numpy(), cells=np.asarray(r["cells"], np.int32),
               obj=r["obj"].numpy(), cls=r["cls"].numpy(), grad_absmax=np.float32(np.abs(g).max()),
               grad_l2=np.float32(np.linalg.norm(g.ravel())), grad_sample=g.ravel()[::37].copy())
    if c["full_grad"]:
        out["grad"] = g
    return out


if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for name in CASES:
        np.savez_compressed(os.path.join(HERE, "golden_%s.npz" % name), **compute(name))
        print("wrote", name)
