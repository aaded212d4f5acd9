"""``server_aggregate`` with the signature of train_feddct.py:34-56."""
from .aggregate import server_aggregate_split


def server_aggregate(global_model_main_client, global_model_proxy_clients,
                     models_main_client, models_proxy_clients):
    server_aggregate_split(global_model_main_client, global_model_proxy_clients,
                           models_main_client, models_proxy_clients)
