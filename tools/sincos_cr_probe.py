"""How much the reference's own gradient moves when its sin/cos (or sqrt) are
correctly rounded instead of MKL VML's (oracle only, CPU):
    python tools/sincos_cr_probe.py builtin:yolov3-tiny-dota 416 16 4 [all|trig|sqrt]
(config, S, B, keys, which functions are replaced).  DESIGN.md §4."""
import os, sys, time, torch, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle, oracle.reference_path as R
from oracle import draws_ref
P_ = 'adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd'
import importlib
sy = importlib.import_module(P_ + '.synthetic'); W = importlib.import_module(P_ + '.weights'); G = importlib.import_module(P_ + '.cfg_gen')
ld = importlib.import_module(P_ + '.load_data')
MODE = sys.argv[5] if len(sys.argv) > 5 else 'all'
cfg, S, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
import tempfile
path = os.path.join(tempfile.gettempdir(), 'w_%s.weights' % cfg.split(':')[1])
W.write_weights(path, W.synthesize(cfg, seed=4))
net = oracle.OracleDarknet(G.cfg_text(cfg), path)
colors = ld.load_printability_colors("builtin:30values")
P = 224
img, lab, patch = sy.frames(B, S, seed=0), sy.labels(B, seed=1), sy.patch(P, seed=2)
osin, ocos, osqrt = torch.sin, torch.cos, torch.sqrt
cr = lambda f: (lambda x: f(x.double()).float() if x.dtype == torch.float32 else f(x))
class CRTorch:
    def __getattr__(self, k):
        if k == 'sin' and MODE != 'sqrt': return cr(osin)
        if k == 'cos' and MODE != 'sqrt': return cr(ocos)
        if k == 'sqrt' and MODE != 'trig': return cr(osqrt)
        return getattr(torch, k)
for key in range(int(sys.argv[4])):
    d = {k: torch.from_numpy(v) for k, v in draws_ref.draws(3, key, 0, B, P).items()}
    t0 = time.time()
    R.torch = torch
    g0 = oracle.train_step(patch, img, lab, d, net, colors)["grad"]
    R.torch = CRTorch()
    g1 = oracle.train_step(patch, img, lab, d, net, colors)["grad"]
    R.torch = torch
    sn = torch.sin(d['angle']); cs = torch.cos(d['angle'])
    nm = int((sn != cr(osin)(d['angle'])).sum() + (cs != cr(ocos)(d['angle'])).sum())
    print('key', key, 'CR-vs-MKL rel %.3g' % float((g1 - g0).abs().max() / g0.abs().max()), 'sincos mismatches', nm, '%.0fs' % (time.time() - t0), flush=True)
