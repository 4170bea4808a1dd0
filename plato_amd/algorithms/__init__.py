"""Algorithm-side plugin surface (plato/algorithms/fedavg.py counterpart)."""

from .fedavg import FedAvgAlgorithmMixin, FedAsyncAlgorithmMixin  # noqa: F401
