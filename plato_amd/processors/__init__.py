"""Server inbound processors whose decoding runs natively.

* ``qsgd``: QSGD payloads stay coded to HBM, decoded in the FedAvg kernel.
* ``zstd``: model_compress payloads decompressed and parsed natively into pinned arenas.
"""

from .qsgd import QsgdPayload  # noqa: F401
