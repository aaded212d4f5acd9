"""feddct_amd — MI355X-native server-side parameter aggregation.

Drop-in replacement for the reference's ``server_aggregate`` (FedAvg /
FedProx / FedDCT / SplitFed rounds).  See DESIGN.md and INTEGRATION.md.

    from feddct_amd.fedavg import server_aggregate     # train_fedavg.py:138
    from feddct_amd.feddct import server_aggregate     # train_feddct.py:34

Importing the package does not load the HIP library; the first aggregation
(or ``feddct_amd._lib``) does, and fails loudly if it is missing.
"""
__version__ = "0.1.0"


def server_aggregate(global_model, client_models):
    from .aggregate import server_aggregate as _sa
    return _sa(global_model, client_models)


def set_summation_order(order: str, strict: bool = False) -> None:
    """"torch_cpu" (default) or "torch_gpu" (torch-ROCm's GPU mean on this
    device, not the published NVIDIA runs' order): see
    aggregate.set_summation_order."""
    from .aggregate import set_summation_order as _s
    _s(order, strict)
