"""plato_amd — MI355X-native server-side aggregation engine for Plato.

The FedAvg weighted reduction of Plato's server (plato/servers/fedavg.py,
plato/algorithms/fedavg.py) as hand-written HIP kernels for gfx950, reached
through the C ABI in include/plato_agg.h and plugged in behind Plato's own
server/algorithm hooks (plato_amd.servers, plato_amd.algorithms).
"""

__version__ = "0.1.0"
