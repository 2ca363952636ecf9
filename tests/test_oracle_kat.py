"""Known-answer tests pinning the oracle.  CPU only.

The reference has no tests or golden vectors and may not be executed here
(SURVEY.md §8c), so these analytic answers plus the committed fixtures
(tests/golden/) are what pins the oracle."""
import math

import torch
import torch.nn.functional as F

import oracle
from conftest import pkg_mod


def test_kat1_identity_theta_reproduces_padded_patch():
    # angle 0, scale 1, target (0.5, 0.5) -> theta = identity; grid_sample with
    # it reproduces the padded patch (to sampling-coordinate rounding)
    S, P = 96, 32
    lab = torch.full((1, 4, 5), 1e-6)
    # sel = (max-area row + min-area row)/2 with cols 2,3 giving target_size = P:
    # sqrt((y*S/2)^2 + (w*S/2)^2) = P with y = w  ->  y = sqrt(2)*P/S
    y = math.sqrt(2) * P / S
    lab[0, 0] = torch.tensor([0.0, 0.5, 2 * y - 1e-6, 2 * y - 1e-6, 0.5])
    dr = {"angle": torch.zeros(1), "ux": torch.tensor([0.5]), "uy": torch.tensor([0.5])}
    theta, center, ts = oracle.patch_theta(lab, S, P, dr)
    torch.testing.assert_close(theta[0], torch.tensor([[1., 0., 0.], [0., 1., 0.]]), rtol=0, atol=2e-6)
    assert torch.equal(center, torch.tensor([[48.0, 48.0]]))
    patch = torch.rand(1, 3, P, P, generator=torch.Generator().manual_seed(0))
    padded = F.pad(patch, (32, 32, 32, 32))
    grid = F.affine_grid(torch.eye(2, 3).unsqueeze(0), padded.shape, align_corners=False)
    out = F.grid_sample(padded, grid, align_corners=False)
    # the sampling coordinate is j +- rounding: not bit-exact, within ~1e-5
    torch.testing.assert_close(out, padded, rtol=0, atol=1e-5)


def test_kat2_tv_of_constant_patch():
    P = 50
    tv = oracle.total_variation(torch.full((3, P, P), 0.3))
    assert abs(float(tv) - 2 * (P - 1) / P * 1e-6) < 1e-11


def test_kat3_nps_of_printable_colour_patch():
    colors = pkg_mod("load_data").load_printability_colors("builtin:30values")
    k, P = 7, 40
    patch = colors[k].view(3, 1, 1).expand(3, P, P).clone()
    nps = oracle.nps_score(patch, colors)
    assert abs(float(nps) - math.sqrt(1e-6 + 3e-12) / 3) < 1e-9
    assert abs(float(nps) - 3.3333e-4) < 1e-7


def test_kat4_colour_loss_of_grey_patch():
    assert float(oracle.colorful_loss(torch.full((3, 16, 16), 0.5))) == 0.0


def test_kat5_ce_of_equal_probabilities_is_ln15():
    no_cls = torch.full((4, 9, 15), 0.5)
    assert abs(float(oracle.noCLS_Loss_CE(no_cls, 14)) - math.log(15)) < 1e-6


def test_kat6_obj_loss_of_half_objectness():
    no_obj = torch.full((5, 9), 0.5)
    loss = 4 * (1 - torch.mean(torch.max(no_obj, 1, keepdim=True)[0]))
    assert float(loss) == 2.0


def test_kat7_median_of_constant_and_gradient():
    x = torch.full((1, 3, 12, 12), 0.25, requires_grad=True)
    y = oracle.median_pool7(x)
    assert torch.all(y == 0.25)
    y.sum().backward()
    assert abs(float(x.grad.sum()) - 3 * 144) < 1e-4


def test_kat8_transposed_cell_index():
    # centre (100, 300) at h=19, S=608: ix=3, iy=9, index = 3*19+9 = 66
    assert oracle.cell_indices([19], 608, torch.tensor([[100.0, 300.0]])) == [[66]]


def test_kat9_empty_label_frame_target_size():
    lab = torch.full((1, 252, 5), 1e-6)
    lab[0, 0] = 1.0
    dr = {"angle": torch.zeros(1), "ux": torch.tensor([0.3]), "uy": torch.tensor([0.3])}
    _, _, ts = oracle.patch_theta(lab, 608, 224, dr)
    assert abs(float(ts) - 0.25 * 304 * math.sqrt(2)) < 1e-3
    assert abs(float(ts) - 107.48) < 5e-3
    assert abs(float(ts) / 224 - 0.4798) < 1e-4


def test_position_clamps_q4():
    lab = torch.full((2, 3, 5), 1e-6)
    lab[:, 0] = torch.tensor([1.0, 0.5, 0.5, 0.1, 0.1])
    dr = {"angle": torch.zeros(2), "ux": torch.tensor([0.05, 0.9]), "uy": torch.tensor([0.95, 0.1])}
    _, center, _ = oracle.patch_theta(lab, 100, 20, dr)
    torch.testing.assert_close(center, torch.tensor([[20.0, 80.0], [90.0, 10.0]]))


def test_lab_transform_q2_q3():
    # (max-area row + min-area row)/2; the padding row is the min-area row
    lab = torch.full((1, 5, 5), 1e-6)
    lab[0, 0] = torch.tensor([3.0, 0.2, 0.4, 0.1, 0.1])
    lab[0, 1] = torch.tensor([5.0, 0.6, 0.8, 0.3, 0.2])
    sel = oracle.lab_transform(lab)
    torch.testing.assert_close(sel[0, 0], (lab[0, 1] + 1e-6) / 2)


def test_max_prob_extractor_reads_the_logit_fields():
    """MaxProbExtractor (load_data.py:125-311): bbox_decode rewrites fields 0..3
    only, so the per-image maxima are the maxima of the raw field-4 and
    field-(5+cls) logits over head-major, anchor-major, cell-minor indices."""
    gen = torch.Generator().manual_seed(0)
    heads = [torch.randn(2, 60, s, s, generator=gen) for s in (4, 8)]
    anchors = [[(10, 13), (16, 30), (33, 23)], [(30, 61), (62, 45), (59, 119)]]
    mo, mc, oi, ci = oracle.max_prob_extractor(heads, 7, 15, anchors)
    flat_o = torch.cat([h.view(2, 3, 20, -1)[:, :, 4].reshape(2, -1) for h in heads], 1)
    flat_c = torch.cat([h.view(2, 3, 20, -1)[:, :, 5 + 7].reshape(2, -1) for h in heads], 1)
    assert torch.equal(mo, flat_o.max(1).values) and torch.equal(oi, flat_o.max(1).indices)
    assert torch.equal(mc, flat_c.max(1).values) and torch.equal(ci, flat_c.max(1).indices)
    so, sc, _, _ = oracle.max_prob_extractor(heads, 7, 15, anchors, sigmoid_mode=True)
    torch.testing.assert_close(so, torch.sigmoid(mo), rtol=0, atol=0)
    torch.testing.assert_close(sc, torch.sigmoid(mc), rtol=0, atol=0)


def test_generalised_loss_head_equals_reference_form_at_three_heads():
    """the (nheads, 5+C) head of obj_cls_conf_find / no_obj_reshape /
    no_cls_reshape is, at the reference's 3 heads x (5+15), the literal
    statement of train_patch.py:488-524 (no_obj_reshape3 / no_cls_reshape3)
    bit for bit."""
    gen = torch.Generator().manual_seed(3)
    B = 5
    heads = [torch.randn(B, 60, s, s, generator=gen) for s in (19, 38, 76)]
    center = torch.rand(B, 2, generator=gen) * 608
    obj_l, cls_l = oracle.obj_cls_conf_find(heads, 608, center)
    assert torch.equal(oracle.no_obj_reshape(obj_l), oracle.no_obj_reshape3(obj_l))
    assert torch.equal(oracle.no_cls_reshape(cls_l), oracle.no_cls_reshape3(cls_l))


def test_generalised_loss_head_two_tiny_heads():
    """Config 5 (yolov3-tiny-15, two heads at 13/26 for S=416): anchors are
    k = head*3 + a over 6 anchors, each read at the transposed cell (Q1) of its
    head; a head of C=15 classes reads channels a*20 + 4 .. a*20 + 19."""
    B, S = 3, 416
    heads = [torch.zeros(B, 60, 13, 13), torch.zeros(B, 60, 26, 26)]
    center = torch.tensor([[100.0, 300.0], [5.0, 410.0], [250.0, 17.0]])
    cells = oracle.cell_indices([13, 26], S, center)
    for h, hw in enumerate((13, 26)):
        st = S / hw
        for b in range(B):
            ix, iy = int(center[b, 0] // st), int(center[b, 1] // st)
            assert cells[h][b] == ix * hw + iy
            r, c = divmod(cells[h][b], hw)
            for a in range(3):
                heads[h][b, a * 20 + 4, r, c] = 10.0 * h + a + b / 10.0      # objectness logit
                heads[h][b, a * 20 + 5 + 14, r, c] = -(a + 1.0)              # class-14 logit
    obj_l, cls_l = oracle.obj_cls_conf_find(heads, S, center)
    no_obj, no_cls = oracle.no_obj_reshape(obj_l), oracle.no_cls_reshape(cls_l)
    assert no_obj.shape == (B, 6) and no_cls.shape == (B, 6, 15)
    for b in range(B):
        for h in range(2):
            for a in range(3):
                assert float(no_obj[b, 3 * h + a]) == float(torch.sigmoid(torch.tensor(10.0 * h + a + b / 10.0)))
                assert float(no_cls[b, 3 * h + a, 14]) == float(torch.sigmoid(torch.tensor(-(a + 1.0))))
                assert torch.all(no_cls[b, 3 * h + a, :14] == 0.5)
    # CE of probabilities treated as logits (Q7), target 14, mean over 6 anchors then over B
    want = 0.0
    for b in range(B):
        row = [math.log(14 * math.exp(0.5) + math.exp(float(no_cls[b, k, 14]))) - float(no_cls[b, k, 14])
               for k in range(6)]
        want += sum(row) / 6
    assert abs(float(oracle.noCLS_Loss_CE(no_cls, 14)) - want / B) < 1e-6
