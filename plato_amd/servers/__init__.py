"""Server-side plugin surface: GPU-backed aggregation hooks for Plato servers."""

from .fedavg import DeltasAggregationMixin, FusedAggregationMixin, make_server  # noqa: F401
from .ingest import WireIngestMixin  # noqa: F401
