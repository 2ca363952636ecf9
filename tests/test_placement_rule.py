"""CPU checks of the test-time placement oracle (SURVEY.md §8f row 4,
reference load_data.py:1322-1430): the closed form the HIP kernels implement
(free cells = non-border cells whose first covering box is the last one the
reference's early-exit loop sums, oracle.placement_ref.free_cells_rule) gives
exactly the zeros of the literal inter_axis_cal, across sparse and crowded
scenes, every semi_edge regime (0 -> '-0:' slices cover everything, beyond S/2
the border covers everything), single-label scenes and boxes whose int()
bounds go negative (Python slices wrap or empty)."""
import itertools

import numpy as np
import pytest
import torch

from oracle import placement_ref as pr


def _labels(n, seed, wmax):
    g = np.random.Generator(np.random.PCG64(seed))
    lab = np.zeros((1, n, 7), dtype=np.float32)
    lab[0, :, 0] = g.uniform(-0.05, 1.05, n)
    lab[0, :, 1] = g.uniform(-0.05, 1.05, n)
    lab[0, :, 2] = g.uniform(0.01, wmax, n)
    lab[0, :, 3] = g.uniform(0.01, wmax, n)
    lab[0, :, 4:6] = g.uniform(0, 1, (n, 2))
    lab[0, :, 6] = g.integers(0, 15, n)
    return torch.from_numpy(lab)


CASES = list(itertools.product([1, 2, 5, 30], [0.1, 0.5, 1.2], [0.0, 0.5, 3.5, 11.0, 40.0]))


@pytest.mark.parametrize("n,wmax,semi", CASES)
def test_free_cells_rule_matches_inter_axis_cal(n, wmax, semi):
    S = 64
    for seed in range(3):
        lab = _labels(n, seed * 101 + n, wmax)
        semi_t = torch.tensor(semi, dtype=torch.float32)
        want = pr.inter_axis_cal(lab, semi_t, S) == 0
        got = pr.free_cells_rule(lab, semi_t, S)
        assert torch.equal(got, want), (n, wmax, semi, seed, int(got.sum()), int(want.sum()))


def test_equal_areas_keep_label_order():
    """Equal areas: the stable order (first row first) decides which box the
    early exit drops."""
    lab = torch.zeros(1, 3, 7)
    lab[0, :, 2:4] = 0.3
    lab[0, :, 0] = torch.tensor([0.2, 0.5, 0.8])
    lab[0, :, 1] = 0.5
    semi = torch.tensor(2.0)
    assert torch.equal(pr.free_cells_rule(lab, semi, 48), pr.inter_axis_cal(lab, semi, 48) == 0)


def _boxes(rows):
    lab = torch.zeros(1, len(rows), 7)
    for i, (x, y, w, h) in enumerate(rows):
        lab[0, i, :4] = torch.tensor([x, y, w, h])
    return lab


@pytest.mark.parametrize("rows,semi,regime", [
    ([(0.5, 0.5, 0.9, 0.9)], 2.0, "M=0"),                                      # one box covers the interior
    ([(0.5, 0.5, 0.95, 0.95), (0.5, 0.5, 0.96, 0.96), (0.2, 0.2, 0.97, 0.97)], 2.0, "M=0"),
    ([(0.25, 0.25, 0.6, 0.6), (0.75, 0.75, 0.62, 0.62), (0.25, 0.75, 0.64, 0.64), (0.75, 0.25, 0.66, 0.66),
      (0.5, 0.5, 0.1, 0.1), (0.5, 0.5, 0.9, 0.9), (0.4, 0.4, 0.95, 0.95)], 1.5, "early"),   # filled before the last
    ([(0.1, 0.1, 0.1, 0.1), (0.9, 0.9, 0.1, 0.1)], 4.0, "M=n"),
    ([(0.5, 0.5, 0.2, 0.2), (0.5, 0.5, 0.9, 0.9)], 3.0, "M=n-1"),             # the last box fills the rest
    ([(0.02, 0.03, 0.3, 0.3)], 0.4, "M=-1"),                                  # int(semi) = 0: '-0:' covers all
    ([(0.02, 0.03, 0.3, 0.3), (0.5, 0.5, 0.1, 0.1)], 0.4, "M=-1"),
])
def test_placement_regimes(rows, semi, regime):
    S = 48
    lab = _boxes(rows)
    st = torch.tensor(semi)
    free, M = pr.free_cells_rule(lab, st, S, return_m=True)
    n = len(rows)
    got = "M=0" if M == 0 else "M=-1" if M == -1 else "M=n" if M == n else "M=n-1" if M == n - 1 else "early"
    assert got == regime, (M, n)
    assert torch.equal(free, pr.inter_axis_cal(lab, st, S) == 0)
