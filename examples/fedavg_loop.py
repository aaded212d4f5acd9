#!/usr/bin/env python3
"""A FedAvg / FedProx round loop shaped like the reference's
(train_fedavg.py:367-410, train_fedprox.py:373-416) with the engine dropped
in.  Small CNN, synthetic CIFAR-shaped data, everything on the GPU.

    python examples/fedavg_loop.py [--rounds 3] [--clients 4] [--mu 0.01]

Each round: every client slot trains locally (SGD, optional FedProx term),
then ``server_aggregate(global_model, client_models)`` replaces the
reference's loop of state_dict() / stack / mean / load_state_dict.
(tests/test_gpu_e2e.py runs this loop with a per-round bit-exactness check
against the reference arithmetic.)
"""
from __future__ import annotations

import argparse
import copy
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from feddct_amd.fedavg import server_aggregate  # noqa: E402
from feddct_amd.prox import proximal_term  # noqa: E402


class SmallNet(nn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 3, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(32)
        self.conv2 = nn.Conv2d(32, 64, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(64)
        self.fc = nn.Linear(64, num_classes)

    def forward(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        x = F.max_pool2d(x, 2)
        x = F.relu(self.bn2(self.conv2(x)))
        x = F.adaptive_avg_pool2d(x, 1).flatten(1)
        return self.fc(x)


def run(rounds=3, clients=4, steps=5, mu=0.0, check=None, seed=0, device="cuda"):
    """``check(snapshot, global_model, client_models) -> dict`` (optional) is
    called after every aggregation with the clients' pre-round CPU states."""
    torch.manual_seed(seed)
    dev = torch.device(device)
    global_model = SmallNet().to(dev)
    client_models = [copy.deepcopy(global_model) for _ in range(clients)]
    opts = [torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9) for m in client_models]
    data = [(torch.randn(steps, 16, 3, 32, 32, device=dev),
             torch.randint(0, 10, (steps, 16), device=dev)) for _ in range(clients)]
    log = []
    for r in range(rounds):
        t0 = time.perf_counter()
        for m, opt, (xs, ys) in zip(client_models, opts, data):
            m.train()
            for x, y in zip(xs, ys):
                opt.zero_grad()
                loss = F.cross_entropy(m(x), y)
                if mu > 0:  # train_fedprox.py:113-116
                    loss = loss + (mu / 2) * proximal_term(m, global_model, flat_grads=True)
                loss.backward()
                opt.step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        snap = [{k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
                for m in client_models] if check else None
        server_aggregate(global_model, client_models)          # train_fedavg.py:408
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        entry = {"round": r, "train_s": round(t1 - t0, 4), "aggregate_ms": round((t2 - t1) * 1e3, 3)}
        if check:
            entry.update(check(snap, global_model, client_models))
        log.append(entry)
    return log


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--clients", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--mu", type=float, default=0.0)
    a = ap.parse_args()
    for e in run(a.rounds, a.clients, a.steps, a.mu):
        print(e)


if __name__ == "__main__":
    main()
