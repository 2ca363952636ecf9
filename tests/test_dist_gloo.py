"""Multi-process data-parallel semantics on CPU (gloo), SURVEY.md §8e.

N ranks each run the oracle step on their contiguous shard of the global
batch, with the loss assembled by the PRODUCT's weighting
(train_patch.combine_terms + shard_weights) and reduced by the product's
single fused all-reduce (train_patch.allreduce_patch_grad).  The result must
equal the single-process full-batch step: gradient and every loss term, for
the CE objective and the batch-SUM targeted objective (config 4), with equal
and ragged shards.  The GlobalBatchSampler must give every global batch the
same images for any number of ranks, and draws keyed by global image index
(oracle/draws_ref.py, the restatement of po_draws) must not depend on the
split."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT, pkg_mod


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case(B):
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    import oracle
    sy, W, G, ld = ge._pkg("synthetic"), ge._pkg("weights"), ge._pkg("cfg_gen"), ge._pkg("load_data")
    net = oracle.OracleDarknet(G.cfg_text("builtin:mini3"), W.synthesize("builtin:mini3", seed=4))
    P, S = 32, 64
    data = (sy.frames(B, S, seed=60), sy.labels(B, seed=61), sy.patch(P, seed=62), sy.draws(B, P, seed=63))
    return net, data, ld.load_printability_colors("builtin:30values")


def _bounds(B, rank, world):
    return rank * B // world, (rank + 1) * B // world


def _worker(rank, world, port, B, objective, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    import oracle
    tp = ge._pkg("train_patch")
    net, (img, lab, patch, dr), colors = _case(B)
    lo, hi = _bounds(B, rank, world)
    w = tp.shard_weights(hi - lo, B, world, objective)
    if hi > lo:
        r = oracle.train_step(patch, img[lo:hi], lab[lo:hi], {k: v[lo:hi] for k, v in dr.items()}, net, colors,
                              objective=objective,
                              combine=lambda *t: tp.combine_terms(*t, objective=objective, weights=w))
        terms = {k: r[k] for k in tp.LOSS_KEYS}
        g = r["grad"].clone()
    else:
        # an empty shard (fewer images than ranks): PatchTrainer._patch_terms_only —
        # no image terms, this rank's 1/world share of NPS/TV/colour
        leaf = patch.detach().clone().requires_grad_(True)
        z = torch.zeros(())
        loss, terms = tp.combine_terms(z, z, oracle.nps_score(leaf, colors), oracle.total_variation(leaf),
                                       oracle.colorful_loss(leaf), objective=objective, weights=w)
        loss.backward()
        terms = {k: v.detach() for k, v in terms.items()}
        g = leaf.grad.clone()
    tp.allreduce_patch_grad(g, terms)
    if rank == 0:
        out_q.put((g.numpy(), {k: float(v) for k, v in terms.items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,B,objective", [(2, 8, "ce"), (4, 8, "ce"), (2, 8, "targeted"), (4, 8, "targeted"),
                                               (3, 8, "ce"), (3, 8, "targeted"), (4, 3, "ce"), (3, 2, "targeted")])
def test_sharded_allreduce_equals_full_batch(world, B, objective):
    """world 3 with B=8 gives ragged shards (2, 3, 3); world 4 with B=3 and
    world 3 with B=2 give EMPTY shards (a ragged last global batch with fewer
    images than ranks), which contribute only their share of the patch terms."""
    import oracle
    net, (img, lab, patch, dr), colors = _case(B)
    full = oracle.train_step(patch, img, lab, dr, net, colors, objective=objective)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, objective, q)) for r in range(world)]
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
        assert abs(v - float(full[k])) <= 1e-5 * max(1.0, abs(float(full[k]))), (k, v, float(full[k]))


@pytest.mark.parametrize("n,G", [(37, 8), (32, 8), (9, 4), (10, 4)])
def test_global_batch_sampler_is_rank_count_independent(n, G):
    """For every world size, the union of the ranks' slices of global batch k
    (concatenated in rank order) is the single-process batch k, and the shard
    bounds are the ones shard_of reports."""
    tp = pkg_mod("train_patch")
    one = list(tp.GlobalBatchSampler(n, G, 0, 1, shuffle=True, seed=5))
    for world in (2, 3, 4):
        samplers = [tp.GlobalBatchSampler(n, G, r, world, shuffle=True, seed=5) for r in range(world)]
        per = [list(s) for s in samplers]
        assert all(len(p) == len(samplers[0]) for p in per)
        for k in range(len(samplers[0])):
            merged = sum((per[r][k] for r in range(world)), [])
            assert merged == one[k]
            for r in range(world):
                lo, hi, ng = samplers[r].shard_of(k)
                assert ng == len(one[k]) and per[r][k] == one[k][lo:hi]
        # nothing is dropped: a final batch smaller than the world leaves some ranks an empty shard
        assert len(samplers[0]) == len(one)
    # set_epoch reshuffles, identically on every rank
    s0, s1 = tp.GlobalBatchSampler(n, G, 0, 2, seed=5), tp.GlobalBatchSampler(n, G, 1, 2, seed=5)
    s0.set_epoch(3)
    s1.set_epoch(3)
    merged = [x + y for x, y in zip(s0, s1)]
    assert merged != one[:len(merged)]
    assert len(set(sum(merged, []))) == sum(len(b) for b in merged)      # still a permutation slice


def test_draws_keyed_by_global_index():
    """oracle/draws_ref.py (the po_draws restatement): the rows of images
    [b0, b0+B) are the same whether drawn as one batch or as shards."""
    from oracle import draws_ref
    full = draws_ref.draws(0x1234, 7, 0, 8, 16)
    for world in (2, 4):
        for r in range(world):
            part = draws_ref.draws(0x1234, 7, r * 8 // world, 8 // world, 16)
            for k in full:
                assert np.array_equal(part[k], full[k][r * 8 // world:(r + 1) * 8 // world]), k
    other = draws_ref.draws(0x1234, 8, 0, 8, 16)
    assert not np.array_equal(other["noise"], full["noise"])        # a new step draws anew
    # distributions (load_data.py:548-707)
    assert full["contrast"].min() >= 0.8 and full["contrast"].max() < 1.2
    assert full["bright"].min() >= -0.1 and full["bright"].max() < 0.1
    assert full["noise"].min() >= -1.0 and full["noise"].max() < 1.0
    assert abs(float(full["angle"].max())) <= np.pi
    assert full["ux"].min() >= 0 and full["uy"].max() < 1


def test_philox_known_answers():
    """Random123 known-answer vectors of Philox4x32-10."""
    from oracle.draws_ref import philox4x32_10
    cases = [((0, 0, 0, 0, 0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
             ((0xffffffff,) * 6, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
             ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0),
              (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for args, want in cases:
        assert tuple(int(x) for x in philox4x32_10(*args)) == want
