"""Multi-process data-parallel semantics on CPU (gloo): N ranks each compute
the oracle step on their shard of the global batch; the single fused
all-reduce of train_patch.allreduce_patch_grad must reproduce the
global-batch gradient and loss terms.  World sizes 2 and 4."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case():
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    import oracle
    sy, W, G, ld = ge._pkg("synthetic"), ge._pkg("weights"), ge._pkg("cfg_gen"), ge._pkg("load_data")
    net = oracle.OracleDarknet(G.cfg_text("builtin:mini3"), W.synthesize("builtin:mini3", seed=4))
    B, P, S = 8, 32, 64
    data = (sy.frames(B, S, seed=60), sy.labels(B, seed=61), sy.patch(P, seed=62), sy.draws(B, P, seed=63))
    return net, data, ld.load_printability_colors("builtin:30values")


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    import oracle
    sy, tp = ge._pkg("synthetic"), ge._pkg("train_patch")
    net, (img, lab, patch, dr), colors = _case()
    r = oracle.train_step(patch, sy.shard(img, rank, world), sy.shard(lab, rank, world),
                          sy.shard_draws(dr, rank, world), net, colors)
    terms = {k: r[k] for k in tp.LOSS_KEYS}
    g = r["grad"].clone()
    tp.allreduce_patch_grad(g, terms)
    if rank == 0:
        out_q.put((g.numpy(), {k: float(v) for k, v in terms.items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_allreduce_equals_full_batch(world):
    import oracle
    net, (img, lab, patch, dr), colors = _case()
    full = oracle.train_step(patch, img, lab, dr, net, colors)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    g, terms = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = full["grad"].numpy()
    rel = abs(g - ref).max() / abs(ref).max()
    assert rel < 1e-5, rel
    for k, v in terms.items():
        assert abs(v - float(full[k])) <= 1e-5 * max(1.0, abs(float(full[k]))), k
