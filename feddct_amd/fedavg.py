"""``server_aggregate`` with the signature of the reference's train_fedavg.py:138."""
from .aggregate import server_aggregate  # noqa: F401  (global_model, client_models)
