"""Server-side payload ingestion hook: native parsing of arriving payload bytes.

The reference joins a client's socket.io chunks and calls ``pickle.loads``
on them (plato/servers/base.py:817-831).  :class:`WireIngestMixin` overrides
that one method so the bytes are parsed by libplato_ingest.so directly into a
pinned arena laid out like the engine's (baseline key order).  The result is a
real ``OrderedDict`` of CPU tensors (an :class:`~plato_amd.ingest.ArenaStateDict`),
so every later step of the reference — inbound processors, ``weights_received``,
size accounting, ``self.updates`` — sees what ``pickle.loads`` would have
produced, and the aggregation hook stages it to HBM without packing.

Payloads that are not a plain dict of tensors (algorithms that send extra
objects) are handed to ``pickle.loads`` exactly as the reference does.
"""

from __future__ import annotations

import pickle

from .. import ingest
from ..arena import ArenaLayout


class WireIngestMixin:
    #: pin the per-payload arenas (async H2D); False keeps them pageable
    ingest_pinned = True
    #: copy each payload to HBM as soon as it arrives (the aggregation hook then
    #: adopts it); payloads must not be modified in place after arrival
    stage_on_arrival = False

    def _ingest_layout(self):
        try:
            baseline = self.algorithm.extract_weights()
            layout = ArenaLayout.from_state_dict(baseline)
        except (AttributeError, TypeError):
            return None
        cached = getattr(self, "_plato_amd_ingest_layout", None)
        if cached is not None and cached.signature == layout.signature:
            return cached
        self._plato_amd_ingest_layout = layout
        return layout

    def ingest_payload(self, payload):
        """Native ``pickle.loads`` of one payload (falls back for non-tensor payloads).

        ``payload`` is the payload's bytes, or the list of its transport chunks
        (joined natively, in parallel, instead of ``b"".join``).
        """
        data = ingest.join(payload) if isinstance(payload, (list, tuple)) else payload
        try:
            return ingest.loads(data, layout=self._ingest_layout(), pin=self.ingest_pinned)
        except (ingest.IngestError, KeyError, ValueError):
            return pickle.loads(data)

    async def _client_payload_arrived(self, sid, client_id):
        """plato/servers/base.py:817-831 with the join and the unpickle done natively."""
        assert len(self.client_chunks[sid]) > 0 and client_id in self.training_clients

        _data = self.ingest_payload(self.client_chunks[sid])
        self.client_chunks[sid] = []
        if self.stage_on_arrival and isinstance(_data, ingest.ArenaStateDict):
            layout = self._ingest_layout()
            if layout is not None:
                self.aggregation_engine().prestage(_data, layout)

        if self.client_payload[sid] is None:
            self.client_payload[sid] = _data
        elif isinstance(self.client_payload[sid], list):
            self.client_payload[sid].append(_data)
        else:
            self.client_payload[sid] = [self.client_payload[sid]]
            self.client_payload[sid].append(_data)
