"""``server_aggregate`` with the signature of train_splitfed.py:34-56."""
from .aggregate import server_aggregate_split


def server_aggregate(global_model_client, global_model_server, models_client, models_server):
    server_aggregate_split(global_model_client, global_model_server, models_client,
                           models_server)
