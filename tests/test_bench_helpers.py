"""bench.py's reporting helpers (CPU): ULP distance and the ULP histogram the
N>1 bench line carries for the re-associated client-sharded sum."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_ulp_hist_counts_every_element():
    g = torch.Generator().manual_seed(0)
    a = torch.randn(10000, generator=g)
    b = a.clone()
    # step b away from a by 0..40 ULP, in both directions and across zero
    steps = torch.randint(0, 41, (10000,), generator=g)
    bi = b.view(torch.int32)
    bi += torch.where(b >= 0, steps, -steps).to(torch.int32)
    h = bench.ulp_hist(a, b)
    assert sum(h.values()) == a.numel()
    assert h["0"] == int((steps == 0).sum())
    assert h["17+"] == int((steps >= 17).sum())
    assert bench.ulp_dist(a, b) == int(steps.max())


def test_ulp_across_signed_zero():
    a = torch.tensor([0.0, -0.0, 1.0e-45])
    b = torch.tensor([-0.0, 0.0, -1.0e-45])
    h = bench.ulp_hist(a, b)
    assert h["0"] == 2 and h["2"] == 1
