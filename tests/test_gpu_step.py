"""GPU parity of one full training iteration (train_patch.py:164-330) against
the oracle: loss terms, bit-exact cell indices, objectness/class extraction,
and the fp32 patch gradient within 1e-4 relative (north_star tolerance:
max|g_hip - g_ref| / max|g_ref| <= 1e-4).

On yolov3-dota@608 the comparison is branch-aligned: the oracle runs on the
LeakyReLU/maxpool decisions the HIP forward took, and every decision where
the two disagree must be a rounding tie (assert_branch_ties_only) — a kernel
that flips a real branch fails.  The trainer's placement is the reference's
own fp32 arithmetic (po_patch_params geometry 1), so the bound is
north_star's, literally: the HIP gradient within 1e-4 of the fp32 oracle.
The float64 evaluation at the same sample points is the accuracy yardstick
(HIP within 1e-5 of it)."""
import pytest
import torch

import oracle
from conftest import assert_branch_ties_only, pkg_mod, plan_branches

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _trainer(cfg, tmp_path, objective="ce", prec="fp16x3"):
    tp, W, G = pkg_mod("train_patch"), pkg_mod("weights"), pkg_mod("cfg_gen")
    path = str(tmp_path / "w.weights")
    W.write_weights(path, W.synthesize(cfg, seed=4))
    pc = pkg_mod("patch_config")
    cfgobj = pc.patch_configs["paper_obj"]()

    class _Cfg(type(cfgobj)):
        def __init__(self):
            super().__init__()
            self.cfgfile = cfg
            self.weightfile = path

    pc.patch_configs["_test"] = _Cfg
    tr = tp.PatchTrainer("_test", device=DEV, objective=objective, verbose=False)
    tr.darknet_model.conv_prec = prec
    ref_net = oracle.OracleDarknet(G.cfg_text(cfg), path)
    return tr, ref_net


def _run(cfg, B, P, tmp_path, objective="ce", seed=0):
    sy, ld = pkg_mod("synthetic"), pkg_mod("load_data")
    tr, ref_net = _trainer(cfg, tmp_path, objective)
    S = ref_net.height
    img, lab = sy.frames(B, S, seed=seed), sy.labels(B, seed=seed + 1)
    patch, dr = sy.patch(P, seed=seed + 2), sy.draws(B, P, seed=seed + 3)
    colors = ld.load_printability_colors("builtin:30values")
    pg = patch.to(DEV).requires_grad_(True)
    loss, terms = tr.losses(pg, img.to(DEV), lab.to(DEV), {k: v.to(DEV) for k, v in dr.items()})
    # the oracle runs on the branch decisions (LeakyReLU slopes) the HIP forward took
    br = plan_branches(tr.last_plan)
    ref = oracle.train_step(patch, img, lab, dr, ref_net, colors, objective=objective, branch=br)
    loss.backward()
    return ref, terms, pg.grad.cpu()


def _compare(ref, terms, grad, loss_tol=2e-5, grad_check=True, obj_tol=2e-5):
    assert int(terms["flags"].item()) == 0
    torch.testing.assert_close(terms["patch_center"].cpu(), ref["patch_center"], rtol=0, atol=0)
    cells = terms["cells"].cpu().tolist()
    assert cells == ref["cells"]                                   # bit-exact cell indices
    torch.testing.assert_close(terms["obj"].cpu(), ref["obj"], rtol=0, atol=obj_tol)
    torch.testing.assert_close(terms["cls"].cpu(), ref["cls"], rtol=0, atol=obj_tol)
    for k in ("loss", "nps_loss", "tv_loss", "no_obj_loss", "no_cls_loss", "colorful_loss"):
        a, b = float(terms[k]), float(ref[k])
        assert abs(a - b) <= loss_tol * max(1.0, abs(b)), (k, a, b)
    if grad_check:
        rel = float((grad - ref["grad"]).abs().max() / ref["grad"].abs().max())
        assert rel < 1e-4, rel


def test_step_mini3(tmp_path):
    _compare(*_run("builtin:mini3", 6, 32, tmp_path))


@pytest.mark.parametrize("objective", ["targeted", "untargeted"])
def test_step_mini3_objectives(tmp_path, objective):
    _compare(*_run("builtin:mini3", 4, 32, tmp_path, objective=objective))


# A LeakyReLU decision the HIP forward took differently from the oracle must
# sit within the forward's rounding of zero: |pre-activation| <= TIE_TOL *
# max|pre-activation of the layer|.  Two fp32 evaluations of the 75-layer
# forward (folded vs unfolded BN, different summation orders) differ by up
# to ~5e-5 of a layer's maximum (test_gpu_darknet's forward bound); fp16x3
# operands carry ~22 bits instead of 24.  A kernel that flips a real
# branch misses by O(max).
TIE_TOL = {"fp32": 5e-5, "fp16x3": 1e-4}
# objectness / class probabilities at the loss cells after 75 layers: two fp32
# evaluations agree to the forward's 5e-5 (test_gpu_darknet), sigmoid' <= 1/4
OBJ_TOL_608 = 5e-5


def keyed_draws(seed, step, b0, B, P):
    """(hip draws, oracle draws) of one step exactly as the trainer makes them
    (PatchTransformer.make_draws, the path bench.py times): the HIP side gets
    the six scalars per image and the po_draws key -- no noise tensor, so the
    warp kernels regenerate the noise at each corner they read and the step
    takes the sparse box composite -- and the oracle gets the same scalars
    plus the noise tensor po_draws materialises from that key."""
    sy = pkg_mod("synthetic")
    full = {k: v.cpu() for k, v in sy.draws_device(seed, step, b0, B, P, DEV).items()}
    hip = {k: v for k, v in full.items() if k != "noise"}
    hip["noise_key"] = (seed, step, b0)
    return hip, full


def keyed_noise(dr, key):
    """(hip draws, oracle draws) with ``dr``'s five per-image scalars and the
    noise of po_draws key (seed, step, b0): the HIP side gets the key (the
    keyed sparse path), the oracle the noise tensor po_draws makes from it."""
    B, P = dr["contrast"].numel(), dr["noise"].size(-1)
    _, full = keyed_draws(key[0], key[1], key[2], B, P)
    hip = {k: v for k, v in dr.items() if k != "noise"}
    hip["noise_key"] = tuple(key)
    ref = dict(hip)
    del ref["noise_key"]
    ref["noise"] = full["noise"]
    return hip, ref


def assert_timed_path(tr):
    """The step just run took the path bench.py times: the sparse box-only
    composite (po_warp_box_fwd_keyed / _bwd_keyed) with the first layer reading
    frames + boxes (po_conv_first_*_cmp)."""
    plan = tr.last_plan
    assert tr.last_sparse and plan.sparse_input, "sparse composite not taken"
    assert plan.last_first_op in ("po_conv_first_fwd_cmp", "po_conv_first_pool_fwd_cmp",
                                  "po_conv_first_pool_wino_fwd_cmp"), plan.last_first_op


def yardstick_geometry(tr):
    """The float64 yardstick's placement geometry for trainer ``tr``: with the
    reference geometry (the default) the HIP path samples exactly where the
    fp32 reference samples, so the yardstick is the float64 evaluation at
    those sample points ("fp32in64"); with ADVPATCH_GEOMETRY=f64 it is the
    float64 geometry itself."""
    return "fp32in64" if tr.patch_transformer.geometry == "ref" else "fp32"


def branch_aligned(tr, ref_net, img, lab, patch, dr, objective="ce", hip_dr=None, f64=True):
    """One HIP step and the oracle on the branch decisions it took: the fp32
    oracle (with the tie check) and (``f64``) the float64 yardstick.  Inputs
    on the CPU, draws as CPU tensors (``hip_dr``: the HIP side's draws when
    they differ in form, e.g. keyed_draws).  Returns (terms, hip grad, fp32
    oracle result, errs) with errs = {"hip_o32": north_star's |g_hip -
    g32|/max|g32|, "hip_f64": |g_hip - g64|/max|g64|, "o32_f64": the fp32
    oracle's own distance from the yardstick}."""
    import time
    ld = pkg_mod("load_data")
    colors = ld.load_printability_colors("builtin:30values")
    t0 = time.time()
    say = lambda what: print("  [branch_aligned B=%d] %s (%.1fs)" % (img.size(0), what, time.time() - t0), flush=True)
    pg = patch.to(DEV).requires_grad_(True)
    hd = dr if hip_dr is None else hip_dr
    hd = {k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in hd.items()}
    loss, terms = tr.losses(pg, img.to(DEV), lab.to(DEV), hd, objective=objective)
    br = plan_branches(tr.last_plan)
    loss.backward()
    g = pg.grad.cpu()
    say("HIP step")
    rec = {}
    ref32 = oracle.train_step(patch, img, lab, dr, ref_net, colors, objective=objective, branch=br, record=rec)
    assert_branch_ties_only(br, rec, TIE_TOL[tr.darknet_model.conv_prec])   # differing branches are ties
    del rec
    say("fp32 oracle + tie check")
    g32 = ref32["grad"]
    rel = lambda a, b: float((a.double() - b.double()).abs().max() / b.double().abs().max())
    errs = {"hip_o32": rel(g, g32)}
    if f64:
        g64 = oracle.train_step_f64(patch, img, lab, dr, ref_net, colors, objective=objective, branch=br,
                                    geometry=yardstick_geometry(tr))["grad"]
        errs["hip_f64"], errs["o32_f64"] = rel(g, g64), rel(g32, g64)
        say("float64 oracle")
    return terms, g, ref32, errs


def branch_aligned_608(tr, ref_net, B, seed, objective="ce"):
    """branch_aligned on B seeded 608x608 frames and a 224x224 patch."""
    sy = pkg_mod("synthetic")
    P, S = 224, 608
    img, lab = sy.frames(B, S, seed=seed), sy.labels(B, seed=seed + 1)
    patch, dr = sy.patch(P, seed=seed + 2), sy.draws(B, P, seed=seed + 3)
    return branch_aligned(tr, ref_net, img, lab, patch, dr, objective)


def assert_north_star(errs, tag):
    """north_star's criterion: the HIP patch gradient within 1e-4 (max-abs
    relative) of the fp32 oracle on the aligned branches -- literally, with
    no allowance for the oracle's own error -- and within 1e-4 of the float64
    yardstick."""
    print("%s patch grad: hip vs fp32 oracle %.3g, hip vs float64 %.3g, fp32 oracle vs float64 %.3g" % (
        tag, errs["hip_o32"], errs.get("hip_f64", float("nan")), errs.get("o32_f64", float("nan"))))
    assert errs["hip_o32"] <= 1e-4, errs
    if "hip_f64" in errs:
        assert errs["hip_f64"] <= 1e-4, errs


# The HIP path's own accuracy: its patch gradient against the float64
# evaluation at the same sample points and on the same branches.  The fp32
# oracle carries its own fp32 convolution rounding; this bound is what a
# regression of the HIP arithmetic itself would have to get past.
HIP_F64_TOL = 1e-5


def assert_hip_accuracy(errs, tag):
    print("%s: hip vs float64 %.3g (bound %.0e)" % (tag, errs["hip_f64"], HIP_F64_TOL))
    assert errs["hip_f64"] <= HIP_F64_TOL, errs


@pytest.mark.parametrize("prec", ["fp16x3", "fp32"])
def test_step_yolov3_dota_608(tmp_path, prec):
    """yolov3-dota, two 608x608 frames, 224x224 patch: patch gradient within
    1e-4 (max-abs relative) of the float64 evaluation, branch-aligned with
    ties asserted; the fp32 oracle's own distance is printed beside."""
    tr, ref_net = _trainer("builtin:yolov3-dota", tmp_path, prec=prec)
    terms, g, ref32, errs = branch_aligned_608(tr, ref_net, 2, 40)
    _compare(ref32, terms, g, grad_check=False, obj_tol=OBJ_TOL_608)
    assert_north_star(errs, "yolov3 (%s)" % prec)
    assert_hip_accuracy(errs, "yolov3 (%s)" % prec)


def test_step_yolov3_targeted(tmp_path):
    """BASELINE config 4's per-rank workload: the targeted class objective
    (noCLS_loss_targeted, a batch SUM, train_patch.py:550-577) + NPS + TV on
    yolov3-dota@608, exact fp32 convolutions, with the trainer's keyed draws
    (the sparse box composite the bench times, asserted)."""
    tr, ref_net = _trainer("builtin:yolov3-dota", tmp_path, objective="targeted", prec="fp32")
    sy = pkg_mod("synthetic")
    B, P, S = 3, 224, 608
    img, lab, patch = sy.frames(B, S, seed=140), sy.labels(B, seed=141), sy.patch(P, seed=142)
    # the placement scalars of earlier rounds' draws (seed 143), the noise keyed: the timed path
    hip_dr, dr = keyed_noise(sy.draws(B, P, seed=143), (143, 0, 0))
    terms, g, ref32, errs = branch_aligned(tr, ref_net, img, lab, patch, dr, "targeted", hip_dr=hip_dr)
    assert_timed_path(tr)
    _compare(ref32, terms, g, grad_check=False, obj_tol=OBJ_TOL_608)
    assert_north_star(errs, "yolov3 targeted")
    assert_hip_accuracy(errs, "yolov3 targeted")


def test_step_yolov3_targeted_po_draws(tmp_path):
    """The same workload on the trainer's own draws (po_draws, key (143, 0, 0):
    every scalar and the noise keyed): north_star's literal criterion, the HIP
    gradient within 1e-4 of the fp32 oracle, and the HIP path's own accuracy
    within 1e-5 of the float64 evaluation at the reference's sample points.
    (Round 5 sampled in float64 and measured 2.18e-4 here: the reference's
    fp32 placement rounding, which the reference geometry now reproduces.)"""
    tr, ref_net = _trainer("builtin:yolov3-dota", tmp_path, objective="targeted", prec="fp32")
    sy = pkg_mod("synthetic")
    B, P, S = 3, 224, 608
    img, lab, patch = sy.frames(B, S, seed=140), sy.labels(B, seed=141), sy.patch(P, seed=142)
    hip_dr, dr = keyed_draws(143, 0, 0, B, P)
    terms, g, ref32, errs = branch_aligned(tr, ref_net, img, lab, patch, dr, "targeted", hip_dr=hip_dr)
    assert_timed_path(tr)
    _compare(ref32, terms, g, grad_check=False, obj_tol=OBJ_TOL_608)
    assert_north_star(errs, "yolov3 targeted, po_draws")
    assert_hip_accuracy(errs, "yolov3 targeted, po_draws")


@pytest.mark.parametrize("objective", ["ce", "targeted"])
def test_step_tiny_416(tmp_path, objective):
    """Config 5's network, yolov3-tiny-15 @416 (two heads, 6 anchors: the
    oracle's generalised (nheads, 5+C) loss head), B=4, exact
    fp32: cells bit-exact, loss terms within 2e-5, objectness/class within
    5e-5, the patch gradient branch-aligned (LeakyReLU signs and max-pool
    argmaxes, ties asserted): north_star's literal 1e-4 against the fp32
    oracle and the HIP accuracy bound against float64."""
    sy = pkg_mod("synthetic")
    tr, ref_net = _trainer("builtin:yolov3-tiny-dota", tmp_path, objective=objective, prec="fp32")
    B, P, S = 4, 224, 416
    img, lab = sy.frames(B, S, seed=90), sy.labels(B, seed=91)
    patch, dr = sy.patch(P, seed=92), sy.draws(B, P, seed=93)
    terms, g, ref32, errs = branch_aligned(tr, ref_net, img, lab, patch, dr, objective)
    assert terms["obj"].shape == (B, 6) and terms["cls"].shape == (B, 6, 15)
    _compare(ref32, terms, g, grad_check=False, obj_tol=OBJ_TOL_608)
    assert_north_star(errs, "tiny B=4 %s" % objective)
    assert_hip_accuracy(errs, "tiny B=4 %s" % objective)


def test_two_adam_steps_yolov3(tmp_path):
    """BASELINE config 1: 1 frame, 2 Adam(amsgrad, lr 0.03) steps + clamp
    (train_patch.py:131-136, 327-330), checked in three well-conditioned parts:
    (1) at each step's patch, the HIP gradient within 1e-4 (max-abs relative)
    of the oracle's at that same patch; (2) the optimizer: the oracle's Adam
    replaying the HIP gradients lands on the HIP patch within 1e-6; (3) step
    one against the oracle's own gradient: every element within the spread
    that Adam's first update lr*g/(|g|+eps) maps the two gradients to (it
    moves an element by ~lr*sign(g) whatever |g| is, so a near-zero gradient
    may move either way — and only by that much)."""
    sy, ld = pkg_mod("synthetic"), pkg_mod("load_data")
    tr, ref_net = _trainer("builtin:yolov3-dota", tmp_path)
    img, lab = sy.frames(1, 608, seed=50), sy.labels(1, seed=51)
    patch, dr = sy.patch(224, seed=52), sy.draws(1, 224, seed=53)
    colors = ld.load_printability_colors("builtin:30values")
    pg = patch.to(DEV).requires_grad_(True)
    opt = tr.make_optimizer(pg)
    d = {k: v.to(DEV) for k, v in dr.items()}
    brs, hip_grads, hip_patches = [], [], []
    for _ in range(2):
        hip_patches.append(pg.detach().cpu().clone())
        loss, terms = tr.losses(pg, img.to(DEV), lab.to(DEV), d)
        brs.append(plan_branches(tr.last_plan))
        loss.backward()
        hip_grads.append(pg.grad.detach().cpu().clone())
        opt.step()
        opt.zero_grad()
        pg.data.clamp_(0, 1)
    ref_grads = []
    for k in range(2):                                       # (1)
        g = oracle.train_step(hip_patches[k], img, lab, dr, ref_net, colors, branch=brs[k])["grad"]
        rel = float((hip_grads[k] - g).abs().max() / g.abs().max())
        assert rel <= 1e-4, (k, rel)
        ref_grads.append(g)
    replay = iter(hip_grads)                                  # (2)
    ref = oracle.adam_amsgrad_steps(patch, lambda p: next(replay), 2)
    assert float((pg.detach().cpu() - ref).abs().max()) <= 1e-6
    one = oracle.adam_amsgrad_steps(patch, lambda p: ref_grads[0], 1)      # (3)
    # Adam(amsgrad)'s first update is lr * g / (|g| + eps): the HIP and oracle
    # patches may differ by exactly the difference of that map at their two
    # gradients (clamp is 1-Lipschitz), element by element, and no more
    lr, eps = tr.config.start_learning_rate, 1e-8
    u = lambda g: lr * g / (g.abs() + eps)
    bound = (u(hip_grads[0]) - u(ref_grads[0])).abs() + 1e-6
    diff = (hip_patches[1] - one).abs()
    print("Adam step one: max |HIP - oracle| %.2g; %.3g of the elements have a predicted spread > 1e-5" % (
        float(diff.max()), float((bound > 1e-5).float().mean())))
    assert bool((diff <= bound).all()), float((diff - bound).max())


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg,B,P", [("builtin:mini3", 5, 32), ("builtin:yolov3-tiny-dota", 3, 96),
                                     ("builtin:yolov3-dota", 3, 224)])
def test_windowed_plan_matches_full_maps(tmp_path, cfg, B, P):
    """Receptive-field windows (NetPlan._plan_windows) change which pixels are
    computed, not how: cells bit-exact, the loss terms of the two plans
    within fp32 reassociation, and each plan's patch gradient within
    north_star's 1e-4 of the fp32 oracle run on THAT plan's LeakyReLU /
    max-pool branches (ties asserted).  The two HIP plans are two fp32
    evaluations whose LeakyReLU ties may fall differently (the r03 1.07e-4
    gap between them was one); where their branch decisions agree the oracle
    is the same and the plans must also agree with each other within 1e-4."""
    sy, ld = pkg_mod("synthetic"), pkg_mod("load_data")
    tr, ref_net = _trainer(cfg, tmp_path, prec="fp32")
    S = ref_net.height
    img, lab = sy.frames(B, S, seed=70), sy.labels(B, seed=71)
    patch, dr = sy.patch(P, seed=72), sy.draws(B, P, seed=73)
    colors = ld.load_printability_colors("builtin:30values")
    out = []
    for windows in (False, True):
        tr.darknet_model.window_heads = windows
        pg = patch.to(DEV).requires_grad_(True)
        loss, terms = tr.losses(pg, img.to(DEV), lab.to(DEV), {k: v.to(DEV) for k, v in dr.items()})
        br = plan_branches(tr.last_plan)
        loss.backward()
        assert tr.last_plan.windowed == windows
        if windows:
            assert int(tr.last_plan.win_flags.item()) == 0
        out.append((terms, pg.grad.detach().cpu().clone(), br))
    (t0, g0, br0), (t1, g1, br1) = out
    assert int(t1["flags"].item()) == 0
    assert t0["cells"].tolist() == t1["cells"].tolist()
    for k in ("loss", "no_obj_loss", "no_cls_loss"):
        assert abs(float(t0[k]) - float(t1[k])) <= 1e-5 * max(1.0, abs(float(t0[k]))), (k, float(t0[k]), float(t1[k]))
    torch.testing.assert_close(t1["obj"], t0["obj"], rtol=0, atol=1e-5)

    def same_branches(a, b):
        """b's decisions (windowed: -1 = outside the window, not computed) equal a's where b has one."""
        for i, (kind, v) in b.items():
            u = a[i][1]
            if kind == "leaky" and v.dtype != torch.bool:
                known = v >= 0
                if not torch.equal((u[known] > 0) if u.dtype == torch.bool else (u[known] > 0), v[known] > 0):
                    return False
            elif not torch.equal(u, v):
                return False
        return True

    rel = lambda a, b: float((a.double() - b.double()).abs().max() / b.double().abs().max())
    g32 = {}
    for tag, g, br in (("full", g0, br0), ("windowed", g1, br1)):
        if tag == "windowed" and same_branches(br0, br1):
            g32[tag] = g32["full"]              # same branches: the same oracle evaluation
        else:
            rec = {}
            g32[tag] = oracle.train_step(patch, img, lab, dr, ref_net, colors, branch=br, record=rec)["grad"]
            assert_branch_ties_only(br, rec, TIE_TOL["fp32"])
        print("%s %s plan: hip vs fp32 oracle %.3g" % (cfg, tag, rel(g, g32[tag])))
        assert rel(g, g32[tag]) <= 1e-4, (tag, rel(g, g32[tag]))
    if g32["windowed"] is g32["full"]:
        assert rel(g1, g0) <= 1e-4, rel(g1, g0)


@pytest.mark.parametrize("cfg,B,P", [("builtin:mini3", 4, 32), ("builtin:yolov3-dota", 2, 224)])
def test_sign_bit_masks_match_fp32_masks(tmp_path, cfg, B, P, monkeypatch):
    """The dgrad epilogues' LeakyReLU masks read as sign bits (NetPlan._build_bits)
    select the same slopes as the fp32 activations, and dropping the fp32 copy
    of mask-only activations (NetPlan._drop_mask_only_outputs) changes
    nothing: identical gradients."""
    sy = pkg_mod("synthetic")
    out = []
    monkeypatch.setenv("ADVPATCH_TUNE", "0")          # same tiles (summation order) in both runs
    for bits, drop in (("1", "1"), ("1", "0"), ("0", "1")):
        monkeypatch.setenv("ADVPATCH_MASK_BITS", bits)
        monkeypatch.setenv("ADVPATCH_DROP_MASK_ONLY", drop)
        tr, _ = _trainer(cfg, tmp_path)
        S = tr.darknet_model.height
        img, lab = sy.frames(B, S, seed=80).to(DEV), sy.labels(B, seed=81).to(DEV)
        dr = {k: v.to(DEV) for k, v in sy.draws(B, P, seed=83).items()}
        pg = sy.patch(P, seed=82).to(DEV).requires_grad_(True)
        loss, terms = tr.losses(pg, img, lab, dr)
        loss.backward()
        plan = tr.last_plan
        assert bool(plan.bits) == (bits == "1")
        # activations before a fused shortcut are stored only as sign bits
        assert bool(plan.y_dropped) == (bits == "1" and drop == "1" and bool(plan.fused))
        for i in plan.y_dropped:
            assert plan.leaky_signs(i).shape == (B,) + plan.dims[i] + (plan.shp[i][2],)
        out.append(pg.grad.detach().clone())
    assert torch.equal(out[0], out[1]) and torch.equal(out[0], out[2])


@pytest.mark.parametrize("cfg,B,P", [("builtin:mini3", 4, 32), ("builtin:yolov3-tiny-dota", 3, 96),
                                     ("builtin:yolov3-dota", 2, 224)])
def test_head_tails_on_a_second_stream_change_nothing(tmp_path, cfg, B, P, monkeypatch):
    """The head tails' launches on the second stream (NetPlan._plan_tails)
    keep every accumulation in its order: loss terms, cells and the patch
    gradient bit-identical to the one-stream run."""
    sy = pkg_mod("synthetic")
    out = []
    monkeypatch.setenv("ADVPATCH_TUNE", "0")          # the same tiles (summation orders) in both runs
    for streams in ("1", "0"):
        monkeypatch.setenv("ADVPATCH_STREAMS", streams)
        tr, ref_net = _trainer(cfg, tmp_path, prec="fp32")
        S = ref_net.height
        img, lab = sy.frames(B, S, seed=60).to(DEV), sy.labels(B, seed=61).to(DEV)
        dr = {k: v.to(DEV) for k, v in sy.draws(B, P, seed=63).items()}
        pg = sy.patch(P, seed=62).to(DEV).requires_grad_(True)
        loss, terms = tr.losses(pg, img, lab, dr)
        loss.backward()
        assert bool(tr.last_plan.tails) == (streams == "1")
        out.append((terms, pg.grad.detach().clone()))
    (t1, g1), (t0, g0) = out
    assert torch.equal(g1, g0)
    assert t1["cells"].tolist() == t0["cells"].tolist()
    for k in ("loss", "no_obj_loss", "no_cls_loss", "nps_loss", "tv_loss", "colorful_loss"):
        assert float(t1[k]) == float(t0[k]), k
