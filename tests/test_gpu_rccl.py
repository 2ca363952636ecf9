"""The data-parallel reduction over RCCL on the MI355X.

The gloo tests (tests/test_dist_gloo.py) pin the semantics of
train_patch.allreduce_patch_grad at world 2-4 on the CPU; the driver's
8-GPU node runs it over xGMI.  This test runs the same function through a
real ``nccl`` (= RCCL) process group on the one GPU of the box, world 1, in a
child process (RCCL state never enters the pytest process): the fused buffer
[patch grad | 6 loss scalars] is all-reduced on the device, the gradient comes
back unchanged (SUM over one rank) and the loss scalars are replaced by the
reduced device values.  It is the communicator bring-up, the device_id binding
bench.py uses and the fused-buffer layout on hardware, not a scaling figure."""
import os
import socket
import subprocess
import sys

import pytest

from conftest import PKG_NAME, ROOT

pytestmark = pytest.mark.gpu

_CHILD = r"""
import importlib, os, sys, time
import torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
tp = importlib.import_module(sys.argv[2] + ".train_patch")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
assert dist.get_backend() == "nccl"
g = torch.Generator(device="cpu").manual_seed(7)
grad = torch.randn(3, 224, 224, generator=g).to(dev)
want = grad.clone()
terms = {k: torch.tensor(0.25 * (i + 1), device=dev) for i, k in enumerate(tp.LOSS_KEYS)}
out = tp.allreduce_patch_grad(grad, terms)
torch.cuda.synchronize()
assert out is grad
assert torch.equal(grad, want), "RCCL world-1 SUM changed the gradient"
for i, k in enumerate(tp.LOSS_KEYS):
    assert terms[k].device == dev and float(terms[k]) == 0.25 * (i + 1), k
for _ in range(5):
    tp.allreduce_patch_grad(grad, terms)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    tp.allreduce_patch_grad(grad, terms)
torch.cuda.synchronize()
print("rccl world-1 fused all-reduce (%d floats): %.1f us/step" % (grad.numel() + len(tp.LOSS_KEYS),
      (time.perf_counter() - t0) / 50 * 1e6))
assert torch.equal(grad, want)
dist.destroy_process_group()
print("rccl ok")
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_allreduce_patch_grad_over_rccl_world1():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, PKG_NAME], env=env, capture_output=True, text=True,
                       timeout=100)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl ok" in r.stdout
