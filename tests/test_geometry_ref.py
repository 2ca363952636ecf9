"""The reference's fp32 placement arithmetic, pinned against the installed
PyTorch-CPU bit for bit (oracle/geometry_ref.py restates it; the HIP kernels'
reference-geometry form, csrc/warp_geom.h, implements the same sequence).

load_data.py:726-749 builds theta from sin/cos/scale and samples the padded
patch with F.affine_grid + F.grid_sample (align_corners=False).  Those ops
are PyTorch's (ATen linspace / affine_grid / MKL sgemm / the vectorised CPU
grid sampler), so their exact roundings are measured here, not assumed: a
torch whose kernels round differently fails these tests before any GPU
parity test can be misread.  The same checks run in the GPU suite
(``test_geometry_restatement_on_this_host``) because the oracle runs on the
GPU box's CPU there."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle
from oracle import draws_ref
from oracle import geometry_ref as G
from conftest import pkg_mod


def _fma_exact(a, b, c):
    from fractions import Fraction
    ex = Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))
    x = np.float32(float(ex))
    best = x
    for nb in (np.nextafter(x, np.float32(np.inf)), np.nextafter(x, np.float32(-np.inf))):
        if abs(Fraction(float(nb)) - ex) < abs(Fraction(float(best)) - ex):
            best = nb
    return best


def test_fma32_is_correctly_rounded():
    rng = np.random.default_rng(0)
    a = rng.standard_normal(4000).astype(np.float32)
    b = rng.standard_normal(4000).astype(np.float32)
    c = (rng.standard_normal(4000) * 10.0 ** rng.integers(-8, 3, 4000)).astype(np.float32)
    r = G.fma32(a, b, c)
    for i in range(0, 4000, 7):
        assert r[i] == _fma_exact(a[i], b[i], c[i]), i


def _placements(B, S, P, seed):
    """theta [B,2,3] of the trainer's own draws (po_draws' lattice angles,
    the synthetic labels) through the oracle's literal fp32 ops."""
    sy = pkg_mod("synthetic")
    d = {k: torch.from_numpy(v) for k, v in draws_ref.draws(3, seed, 0, B, P).items()}
    lab = sy.labels(B, seed=seed + 1)
    th, _, ts = oracle.patch_theta(lab, S, P, d)
    return th, ts, d, lab


def check_linspace():
    for S in list(range(2, 70)) + [208, 224, 304, 416, 608, 1024]:
        assert np.array_equal(G.linspace32(S), torch.linspace(-1, 1, S).numpy()), S


def test_base_division_by_reciprocal_is_exact():
    """The HIP kernels' base coordinate (reciprocal + one Markstein step,
    warp_geom.h ref_base) equals affine_grid's correctly rounded division on
    every axis length up to 2048 and on a spread of lengths up to 32768 (the
    build container's C check covered all 32767 lengths)."""
    sizes = list(range(2, 2049)) + list(range(2049, 32769, 397)) + [4096, 8192, 16384, 32767, 32768]
    for S in sizes:
        assert np.array_equal(G.base32_markstein(S), G.base32(S)), S


def check_theta(B=64, S=608, P=224):
    th, ts, d, lab = _placements(B, S, P, 5)
    sel = oracle.lab_transform(lab)
    h2 = (sel[:, 0, 2] * S).mul(0.5)
    h3 = (sel[:, 0, 3] * S).mul(0.5)
    sc = (torch.sqrt(h2 ** 2 + h3 ** 2) / P).numpy()
    tx = ((-torch.max(d["ux"], torch.tensor(0.2)) + 0.5) * 2).numpy()
    ty = ((-torch.min(d["uy"], torch.tensor(0.8)) + 0.5) * 2).numpy()
    mine = G.theta32(torch.sin(d["angle"]).numpy(), torch.cos(d["angle"]).numpy(), sc, tx, ty)
    assert np.array_equal(mine, th.numpy())


def check_affine_grid():
    """The host's sgemm follows one of the two restated K = 3 orders exactly,
    on every shape, and the trainer's own probe (load_data.reference_bmm_form,
    which picks the HIP geometry) names the same one."""
    form = G.host_bmm_form()
    print("host sgemm form:", form)
    assert form in G.BMM_FORMS
    for S, P in ((608, 224), (416, 224), (96, 32)):
        th, _, _, _ = _placements(4, S, P, S)
        g = F.affine_grid(th, (4, 3, S, S), align_corners=False).numpy()
        assert np.array_equal(G.affine_grid32(th.numpy(), S, S, form), g), S
    th = torch.randn(3, 2, 3, generator=torch.Generator().manual_seed(1)) * 3
    g = F.affine_grid(th, (3, 1, 50, 70), align_corners=False).numpy()
    assert np.array_equal(G.affine_grid32(th.numpy(), 50, 70, form), g)
    ld = pkg_mod("load_data")
    assert ld.reference_bmm_form() == form
    assert ld.GEOMETRIES["ref"] == 1 + G.BMM_FORMS.index(form)


def check_grid_sample():
    for S, P in ((608, 224), (416, 224)):
        th, _, _, _ = _placements(3, S, P, S + 1)
        grid = F.affine_grid(th, (3, 3, S, S), align_corners=False)
        img = torch.rand(3, 3, S, S, generator=torch.Generator().manual_seed(S))
        img[:, :, :S // 3] = 0.0                       # exact zeros, as the padded patch has
        out = F.grid_sample(img, grid, align_corners=False).numpy()
        assert np.array_equal(G.grid_sample32(img.numpy(), grid.numpy()), out), S


def check_sqrt_period():
    """torch.sqrt on this host (MKL VML) is a function of one period: for
    every normal positive x = 4^k m (m in [1, 4)), sqrt(x) = 2^k sqrt(m) bit
    for bit -- what load_data.sqrt_period_table and po_patch_params' lookup
    rely on.  Checked over 2^20 random floats spread across 2^-60 .. 2^60."""
    g = np.random.default_rng(3)
    bits = g.integers(0, 1 << 23, 1 << 20).astype(np.uint32) | ((g.integers(67, 187, 1 << 20).astype(np.uint32)) << 23)
    x = bits.view(np.float32)
    got = torch.sqrt(torch.from_numpy(x)).numpy()
    ue = ((bits >> 23) & 0xFF).astype(np.int64) - 127
    k = np.floor_divide(ue, 2)
    mbits = (((ue - 2 * k) << 23) | (bits & 0x7FFFFF)).astype(np.uint32) + np.uint32(0x3F800000)
    period = torch.sqrt(torch.from_numpy(mbits.view(np.float32))).numpy()
    want = np.ldexp(period.astype(np.float64), k).astype(np.float32)
    assert np.array_equal(got, want), int(np.count_nonzero(got != want))
    cr = np.sqrt(x.astype(np.float64)).astype(np.float32)
    print("torch.sqrt vs correctly rounded: %.2f %% differ" % (100.0 * np.mean(got != cr)))


def test_sqrt_is_periodic_in_powers_of_4():
    check_sqrt_period()


def test_linspace_restatement():
    check_linspace()


def test_theta_restatement():
    check_theta()


def test_affine_grid_restatement():
    check_affine_grid()


def test_grid_sample_restatement():
    check_grid_sample()


def test_lattice_angles_match_po_draws_restatement():
    """sy.draws and load_data.sincos_lattice_table index po_draws' angle lattice."""
    d = draws_ref.draws(7, 3, 0, 256, 8)
    k = np.rint((d["angle"].astype(np.float64) + np.float64(np.float32(math.pi))) /
                np.float64(np.float32(2.0) * np.float32(math.pi)) * 2.0 ** 24).astype(np.int64)
    assert np.array_equal(G.lattice_angles(k), d["angle"])
    sy = pkg_mod("synthetic")
    a = sy.draws(64, 8, seed=3)["angle"].numpy()
    k = np.rint((a.astype(np.float64) + np.float64(np.float32(math.pi))) /
                np.float64(np.float32(2.0) * np.float32(math.pi)) * 2.0 ** 24).astype(np.int64)
    assert np.array_equal(G.lattice_angles(k), a)


def test_sin_cos_are_position_independent():
    """torch.sin / torch.cos of an angle do not depend on the tensor it sits
    in (MKL VML on any length): the trainer's table of the whole lattice gives
    the oracle's values for a batch of B angles."""
    a = torch.from_numpy(G.lattice_angles(np.arange(0, 1 << 24, 4099)))
    big_s, big_c = torch.sin(a), torch.cos(a)
    for n in (1, 3, 16, 64, 256):
        for off in (0, 5, 333):
            sl = a[off:off + n].clone()
            assert torch.equal(torch.sin(sl), big_s[off:off + n])
            assert torch.equal(torch.cos(sl), big_c[off:off + n])
    cr = torch.sin(a.double()).float()
    print("torch.sin vs correctly rounded: %.2f %% of lattice samples differ" %
          (100.0 * float((cr != big_s).float().mean())))


@pytest.mark.gpu
def test_geometry_restatement_on_this_host():
    """The same pins in the GPU suite: the parity tests' oracle runs on this
    host's CPU, whose MKL code path may differ from the build container's."""
    check_linspace()
    check_theta()
    check_affine_grid()
    check_grid_sample()
    check_sqrt_period()
    test_sin_cos_are_position_independent()
