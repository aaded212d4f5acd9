"""``server_aggregate`` with the signature of the reference's train_fedprox.py:143."""
from .aggregate import server_aggregate  # noqa: F401  (global_model, client_models)
