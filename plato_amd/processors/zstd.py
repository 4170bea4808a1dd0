"""zstd-compressed payloads (Plato's model_compress / model_decompress pair), ingested natively.

A client with the ``model_compress`` outbound processor sends
``zstd.compress(pickle.dumps(state_dict), level)``
(plato/processors/model_compress.py:25); the server's ``model_decompress``
inbound processor undoes it with ``pickle.loads(zstd.decompress(data))``
(plato/processors/model_decompress.py:24).

:class:`Processor` is the drop-in for the server side.  The frames are
decompressed by libplato_ingest (the system ``libzstd.so.1``, bound at first
use) into one host buffer, and the pickle inside is parsed natively
(:func:`plato_amd.ingest.loads`, nothing executed) straight into a pinned arena
laid out like the server's model, so the aggregation hooks stage it to HBM
without a per-tensor pack.  A decompressed payload that is not a dict of
tensors goes to ``pickle.loads``, as the reference's processor would.
"""

from __future__ import annotations

import logging
import pickle

import torch

from .. import ingest
from ..arena import ArenaLayout


class Processor:
    """Drop-in for ``plato.processors.model_decompress.Processor`` (same arguments).

    Register it in plato/processors/registry.py under ``model_decompress``
    (or list it in ``server.inbound_processors``).  The server builds its
    processors with ``trainer=self.trainer`` (plato/servers/fedavg.py:88-90);
    the trainer's model defines the arena layout.  ``pin=True`` puts the arena
    in pinned memory for an asynchronous H2D copy.
    """

    def __init__(self, client_id=None, server_id=None, trainer=None, pin: bool = True, layout=None, **kwargs):
        self.client_id = client_id
        self.server_id = server_id
        self.trainer = trainer
        self.pin = pin
        self._layout = layout

    def _arena_layout(self):
        model = getattr(self.trainer, "model", None)
        if model is None:
            return self._layout
        layout = ArenaLayout.from_state_dict(model.state_dict())
        if self._layout is None or self._layout.signature != layout.signature:
            self._layout = layout
        return self._layout

    def process(self, data):
        raw = ingest.zstd_decompress(data)
        try:
            output = ingest.loads(raw, layout=self._arena_layout(), pin=self.pin and torch.cuda.is_available())
        except (ingest.IngestError, KeyError, ValueError):
            output = pickle.loads(raw.tobytes())
        if self.client_id is None:
            logging.info("[Server #%s] Decompressed received model parameters.", self.server_id)
        else:
            logging.info("[Client #%s] Decompressed received model parameters.", self.client_id)
        return output


class CompressProcessor:
    """``model_compress`` (model_compress.py:17-32) on the same libzstd, for clients and tests."""

    def __init__(self, compression_level=1, client_id=None, server_id=None, **kwargs):
        self.compression_level = compression_level
        self.client_id = client_id
        self.server_id = server_id

    def process(self, data) -> bytes:
        return ingest.zstd_compress(pickle.dumps(data), self.compression_level)
