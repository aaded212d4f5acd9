"""ORACLE / CPU BASELINE — test and bench infrastructure only.

A restatement, on CPU torch, of the reference's aggregation loop exactly as
it runs in train_fedavg.py:138-149 (== train_fedprox.py:143-154):

* for every key of the global state_dict, rebuild every client's
  ``state_dict()`` and ``torch.stack([...float()], 0).mean(0)`` (the K·N
  rebuild pattern is part of the reference's cost);
* ``load_state_dict`` the result into the global model;
* ``load_state_dict`` the global state into every client (the broadcast).

bench.py times this on the GPU box's host cores as the ``cpu_baseline``
(kind "port": the reference's Python cannot travel to the box), next to the
arithmetic-only ``stack+mean`` core.
"""
from __future__ import annotations

import time

import torch


def reference_loop(global_model, client_models):
    g = global_model.state_dict()
    for k in g.keys():
        g[k] = torch.stack([client_models[i].state_dict()[k].float()
                            for i in range(len(client_models))], 0).mean(0)
    global_model.load_state_dict(g)
    for m in client_models:
        m.load_state_dict(global_model.state_dict())


def arithmetic_core(client_states):
    """Only the ``stack(...).mean(0)`` expression, per key (no rebuilds)."""
    keys = list(client_states[0].keys())
    return {k: torch.stack([s[k].float() for s in client_states], 0).mean(0) for k in keys}


def time_call(fn, reps: int, budget_s: float):
    """Median wall time of ``fn()`` over up to ``reps`` runs within budget."""
    ts = []
    t_end = time.perf_counter() + budget_s
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
        if time.perf_counter() > t_end:
            break
    ts.sort()
    return ts[len(ts) // 2], len(ts)
