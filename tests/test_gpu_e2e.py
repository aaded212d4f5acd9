"""Reference-shaped round loops (examples/fedavg_loop.py) on the GPU: local
SGD with momentum (and the FedProx term), then the drop-in aggregation,
bit-exact against the reference arithmetic every round."""
import os
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(ROOT, "examples"))


def _check(snap, global_model, client_models):
    import torch
    from oracle.torch_mirror import arithmetic_core
    ref = arithmetic_core(snap)
    ok = True
    for k, v in global_model.state_dict().items():
        want = v.detach().cpu().clone()
        want.copy_(ref[k])  # load_state_dict's copy_ into the key's dtype
        ok &= torch.equal(v.cpu(), want)
        for m in client_models:
            ok &= torch.equal(m.state_dict()[k], v)
    return {"bit_exact_vs_reference": bool(ok)}


@pytest.mark.parametrize("mu", [0.0, 0.01])
def test_round_loop_bit_exact(mu):
    from fedavg_loop import run
    log = run(rounds=3, clients=5, steps=3, mu=mu, check=_check)
    assert all(e["bit_exact_vs_reference"] for e in log), log


def test_stale_graph_fails_like_load_state_dict():
    """After the round (kernel writes behind autograd's back) a graph that
    saved a client's pre-round weights fails in backward, as it does after
    the reference's load_state_dict broadcast."""
    import torch
    from feddct_amd.aggregate import server_aggregate
    dev = torch.device("cuda", 0)

    def mk():
        return torch.nn.Sequential(torch.nn.Linear(8, 4), torch.nn.BatchNorm1d(4)).to(dev)
    g, clients = mk(), [mk() for _ in range(3)]
    server_aggregate(g, clients)  # binds the arenas
    w = clients[1][0].weight
    y = (w * w).sum()
    server_aggregate(g, clients)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        y.backward()
    (clients[1][0].weight ** 2).sum().backward()  # a fresh graph is fine
