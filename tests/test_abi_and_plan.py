"""CPU tests of the boundary and the host-side plan: the C-ABI library loads
and exports every entry point include/advpatch.h declares; builtin cfgs
reproduce the reference networks; synthetic weights have the reference
.weights layout; the Darknet execution plan is well formed.  No kernel is
launched (no GPU here)."""
import os
import re

import pytest
import torch

from conftest import ROOT, pkg_mod

HEADER = os.path.join(ROOT, "include", "advpatch.h")
REF_CFG = "/root/reference/cfg"


def _lib():
    nat = pkg_mod("_native")
    if not os.path.exists(nat.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return nat, nat.load()


def test_library_exports_every_header_symbol():
    text = open(HEADER).read()
    declared = set(re.findall(r"^\s*(?:int|const char\*)\s+(po_\w+)\s*\(", text, re.M))
    assert len(declared) >= 20
    nat, lib = _lib()
    for name in sorted(declared):
        assert hasattr(lib, name), "libadvpatch_hip.so does not export %s" % name
    assert declared == set(nat.symbols()), declared ^ set(nat.symbols())
    assert lib.po_abi_version() == nat.PO_ABI_VERSION == 30


def test_conv_desc_struct_matches_header():
    text = open(HEADER).read()
    body = text[text.index("typedef struct po_conv_desc"):text.index("} po_conv_desc;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = re.findall(r"(?:int64_t|int|int8_t\*|int32_t\*|float\*|void\*)\s+([^;]+);", body)
    names = []
    for f in fields:
        for part in f.split(","):
            names.append(re.sub(r"\[.*\]", "", part).strip())
    nat = pkg_mod("_native")
    assert names == [f[0] for f in nat.po_conv_desc._fields_]


def test_errors_are_reported_not_silent():
    nat, lib = _lib()
    rc = lib.po_median7_fwd(None, 3, 10, 10, None, None, None)
    assert rc == -1
    assert "null pointer" in nat.last_error()
    with pytest.raises(RuntimeError):
        nat.call("po_median7_fwd", None, 3, 10, 10, None, None, None)


def test_hip_ops_fail_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    mp = pkg_mod("median_pool")
    with pytest.raises(RuntimeError):
        mp.MedianPool2d(7, same=True)(torch.rand(1, 3, 10, 10))


def _layers(text):
    out = []
    for d in pkg_mod("cfg").parse_model_config_text(text):
        t = d["type"]
        if t == "net":
            out.append((t, d["width"], d["height"], d["channels"]))
        elif t == "convolutional":
            out.append((t, int(d["filters"]), int(d["size"]), int(d["stride"]), int(d["batch_normalize"]),
                        d["activation"]))
        elif t == "route":
            out.append((t, tuple(int(x) for x in d["layers"].split(","))))
        elif t == "shortcut":
            out.append((t, int(d["from"])))
        elif t == "upsample":
            out.append((t, int(d["stride"])))
        elif t == "maxpool":
            out.append((t, int(d["size"]), int(d["stride"])))
        elif t == "yolo":
            out.append((t, d["mask"].replace(" ", ""), int(d["classes"])))
    return out


@pytest.mark.skipif(not os.path.isdir(REF_CFG), reason="reference not mounted")
def test_builtin_yolov3_dota_equals_reference_cfg():
    G = pkg_mod("cfg_gen")
    ref = _layers(open(os.path.join(REF_CFG, "yolov3-dota.cfg")).read())
    assert _layers(G.yolov3(15, 608)) == ref


@pytest.mark.skipif(not os.path.isdir(REF_CFG), reason="reference not mounted")
def test_builtin_tiny_equals_reference_cfg_up_to_classes():
    G = pkg_mod("cfg_gen")
    ref = _layers(open(os.path.join(REF_CFG, "yolov3-tiny.cfg")).read())
    mine = _layers(G.yolov3_tiny(80, 416))
    assert mine == ref


def test_conv_macs_match_survey():
    import bench
    dk = pkg_mod("darknet_v3")
    assert bench.conv_macs(dk.Darknet("builtin:yolov3-dota")) == 69_841_000_000 or \
        abs(bench.conv_macs(dk.Darknet("builtin:yolov3-dota")) / 69.841e9 - 1) < 1e-3
    assert abs(bench.conv_macs(dk.Darknet("builtin:yolov3-tiny-dota")) / 2.732e9 - 1) < 2e-3


def test_synthetic_weights_layout_and_parameter_count(tmp_path):
    W, dk = pkg_mod("weights"), pkg_mod("darknet_v3")
    stream = W.synthesize("builtin:yolov3-dota", seed=4)
    assert stream.size == 61_651_732
    path = str(tmp_path / "y.weights")
    W.write_weights(path, stream)
    assert os.path.getsize(path) == 20 + 4 * 61_651_732
    net = dk.Darknet("builtin:yolov3-dota")
    assert net.load_darknet_weights(path) == stream.size
    nparam = sum(p.numel() for p in net.parameters())
    assert nparam == 61_599_124
    # save/load round trip through the reference layout
    p2 = str(tmp_path / "y2.weights")
    net.save_darknet_weights(p2)
    assert open(p2, "rb").read()[20:] == open(path, "rb").read()[20:]


def test_plan_structure_yolov3_on_cpu_buffers():
    W, dk = pkg_mod("weights"), pkg_mod("darknet_v3")
    net = dk.Darknet("builtin:mini3")
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "m.weights")
        W.write_weights(p, W.synthesize("builtin:mini3"))
        net.load_darknet_weights(p)
    plan = net.plan(2, 64, 64, torch.device("cpu"))
    assert plan.heads == [17, 25, 33]
    assert [plan.shp[h] for h in plan.heads] == [(4, 4, 60), (8, 8, 60), (16, 16, 60)]
    assert plan.root[18] == 14 and plan.root[26] == 22           # single-layer routes alias
    assert plan.fused == {4, 8, 12}                               # shortcuts fused into conv epilogues
    names = [o[0] for o in plan.fwd_ops]
    assert names.count("po_conv") + names.count("po_conv_first_fwd") == 22
    # every leaky conv with a gradient gets exactly one masked (final) contribution
    masked = {}
    for name, args, desc in plan.bwd_ops:
        if name == "po_conv" and (args[7] is not None or desc.mbits):
            masked[args[4].value] = masked.get(args[4].value, 0) + 1
    for i, d in enumerate(net.blocks):
        if d["type"] == "convolutional" and plan._leaky(i) and plan.has_grad[i] and i > 0:
            assert plan.ncons[i] >= 1


def test_graft_entry_build_runs():
    """__graft_entry__.build() (the driver's build check): make, import, and the
    library's ABI equals the package's."""
    import __graft_entry__
    __graft_entry__.build()
    nat = pkg_mod("_native")
    assert nat.load().po_abi_version() == nat.PO_ABI_VERSION


@pytest.mark.parametrize("cfg,H,want", [("builtin:yolov3-dota", 128, [([80, 81], 79), ([92, 93], 91)]),
                                        ("builtin:yolov3-tiny-dota", 128, [([14, 15], 13)]),
                                        ("builtin:mini3", 64, [([15, 16], 14), ([23, 24], 22)])])
def test_head_tails(cfg, H, want):
    """NetPlan.tail_chains: the convs that feed a YOLO head and nothing else,
    after the branch point whose other consumer leads on to the next head
    (run on the second stream); the last head's tail is not one of them."""
    W, dk = pkg_mod("weights"), pkg_mod("darknet_v3")
    net = dk.Darknet(cfg)
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "m.weights")
        W.write_weights(p, W.synthesize(cfg))
        net.load_darknet_weights(p)
    plan = net.plan(1, H, H, torch.device("cpu"))
    assert plan.tail_chains() == want
    assert plan.tails == []                   # no second stream off the GPU


def test_sparse_input_plan_flag_on_cpu_buffers():
    """NetPlan.sparse_input: the first layer can read the step's sparse
    composite (po_conv_first_*_cmp) -- a direct 3-channel first conv of at
    most 32 padded channels on a square input whose side is a multiple of 4."""
    W, dk = pkg_mod("weights"), pkg_mod("darknet_v3")
    net = dk.Darknet("builtin:mini3")
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "m.weights")
        W.write_weights(p, W.synthesize("builtin:mini3"))
        net.load_darknet_weights(p)
    sq = net.plan(2, 64, 64, torch.device("cpu"))
    assert sq.first_direct and sq.cp[0] <= 32 and sq.sparse_input
    assert not net.plan(2, 64, 96, torch.device("cpu")).sparse_input          # not square


def test_warp_form_selection_and_sparse_ok(monkeypatch):
    """PatchTransformer.warp_form (ADVPATCH_WARP: box / pre / frame, anything
    else refused) and sparse_ok: the sparse composite needs keyed noise, the
    box form and a side that is a multiple of 4."""
    ld = pkg_mod("load_data")
    pt = ld.PatchTransformer()
    assert pt.warp_form == "box" and pt.keyed_noise
    assert pt.sparse_ok(608) and pt.sparse_ok(416) and not pt.sparse_ok(97)
    assert not pt.sparse_ok(608, {"noise": torch.zeros(1)})                   # a noise tensor: not keyed
    assert pt.sparse_ok(608, {"noise_key": (1, 2, 3)})
    pt.warp_form = "pre"
    assert not pt.sparse_ok(608)
    monkeypatch.setenv("ADVPATCH_WARP", "frame")
    assert ld.PatchTransformer().warp_form == "frame"
    monkeypatch.setenv("ADVPATCH_WARP", "sideways")
    with pytest.raises(ValueError):
        ld.PatchTransformer()


def test_wino6_matrices_and_fragment_order():
    """F(4x4,3x3) (tile 71): A^T [(G g G^T) * (B^T d B)] A is the 3x3
    correlation of the 6x6 patch (float64), with G = darknet_v3._WINO6_G and
    the B^T / A^T the kernel's bt6 / at6 implement; wino6_transform stores
    U[xi][16 kc + 8 (l >> 5) + s][32 nb + (l & 31)] at [nb][kc][xi][s >> 2][l][s & 3]."""
    import torch
    dk = pkg_mod("darknet_v3")
    G = torch.tensor(dk._WINO6_G, dtype=torch.float64)
    BT = torch.tensor(dk.WINO6_BT, dtype=torch.float64)
    AT = torch.tensor(dk.WINO6_AT, dtype=torch.float64)
    gen = torch.Generator().manual_seed(0)
    for _ in range(5):
        d = torch.randn(6, 6, generator=gen, dtype=torch.float64)
        g = torch.randn(3, 3, generator=gen, dtype=torch.float64)
        ref = torch.stack([torch.stack([(d[i:i + 3, j:j + 3] * g).sum() for j in range(4)]) for i in range(4)])
        out = AT @ ((G @ g @ G.T) * (BT @ d @ BT.T)) @ AT.T
        assert float((out - ref).abs().max()) < 1e-12
    N, C = 64, 32
    w = torch.randn(N, 9, C, generator=gen)
    offs = [(kh - 1, kw - 1) for kh in range(3) for kw in range(3)]
    frag = dk.wino6_transform(w, offs).reshape(N // 32, C // 16, 36, 2, 64, 4)
    g = torch.zeros(N, C, 3, 3, dtype=torch.float64)
    for t, (dh, dw) in enumerate(offs):
        g[:, :, dh + 1, dw + 1] = w[:, t, :].double()
    U = torch.einsum("xa,ncab,yb->xycn", G, g, G).reshape(36, C, N).float()
    for nb, kc, xi, l, s in ((1, 0, 35, 63, 7), (0, 1, 7, 5, 0), (1, 1, 20, 40, 5)):
        assert frag[nb, kc, xi, s >> 2, l, s & 3] == U[xi, 16 * kc + 8 * (l >> 5) + s, 32 * nb + (l & 31)]
