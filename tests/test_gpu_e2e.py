"""Reference-shaped round loops (examples/fedavg_loop.py) on the GPU: local
SGD with momentum (and the FedProx term), then the drop-in aggregation,
bit-exact against the reference arithmetic every round."""
import os
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(ROOT, "examples"))


@pytest.mark.parametrize("mu", [0.0, 0.01])
def test_round_loop_bit_exact(mu):
    from fedavg_loop import run
    log = run(rounds=3, clients=5, steps=3, mu=mu, check=True)
    assert all(e["bit_exact_vs_reference"] for e in log), log
