"""Server-side payload ingestion hook: native parsing of arriving payload bytes.

The reference joins a client's socket.io chunks and calls ``pickle.loads``
on them (plato/servers/base.py:817-831), or, under comm_simulation (the
default), ``pickle.load``s the file the client wrote (:775-811).
:class:`WireIngestMixin` overrides those methods so the bytes are parsed by
libplato_ingest.so directly into a pinned arena laid out like the engine's
(baseline key order), and sizes payloads by the bytes they arrived as instead
of re-pickling them (:794-796, :839-846).  The result is a
real ``OrderedDict`` of CPU tensors (an :class:`~plato_amd.ingest.ArenaStateDict`),
so every later step of the reference — inbound processors, ``weights_received``,
size accounting, ``self.updates`` — sees what ``pickle.loads`` would have
produced, and the aggregation hook stages it to HBM without packing.

Payloads that are not a plain dict of tensors (algorithms that send extra
objects) are handed to ``pickle.loads`` exactly as the reference does.
"""

from __future__ import annotations

import logging
import os
import pickle
import sys

from .. import ingest
from ..arena import ArenaLayout, payload_codec


class WireIngestMixin:
    #: pin the per-payload arenas (async H2D); False keeps them pageable
    ingest_pinned = True
    #: copy each payload to HBM as soon as it arrives (the aggregation hook then
    #: adopts it); payloads must not be modified in place after arrival
    stage_on_arrival = False
    #: size payloads by their wire bytes instead of re-pickling them (see _wire_payload_size)
    wire_size_accounting = True

    def _ingest_layout(self):
        try:
            baseline = self.algorithm.extract_weights()
            layout = ArenaLayout.from_state_dict(baseline, align=getattr(self, "arena_alignment", None))
        except (AttributeError, TypeError):
            return None
        cached = getattr(self, "_plato_amd_ingest_layout", None)
        if cached is not None and cached.signature == layout.signature:
            return cached
        self._plato_amd_ingest_layout = layout
        return layout

    def _arrival_baseline(self):
        """The current model, for engines that stage arrivals as deltas (``arena_deltas``), else None.

        It is the baseline of the round the arriving payload joins, unless the model changes before
        that round aggregates; the round then sees a different key and stages the payload again.
        """
        if not getattr(self, "arena_deltas", False):
            return None
        try:
            return self.algorithm.extract_weights()
        except (AttributeError, TypeError):
            return None

    def ingest_payload(self, payload):
        """Native ``pickle.loads`` of one payload (falls back for non-tensor payloads).

        ``payload`` is the payload's bytes, or the list of its transport chunks
        (joined natively, in parallel, instead of ``b"".join``).
        """
        return self._ingest(payload)[0]

    def _ingest(self, payload):
        """(data, wire length if parsed natively else None)."""
        data = ingest.join(payload) if isinstance(payload, (list, tuple)) else payload
        try:
            return ingest.loads(data, layout=self._ingest_layout(), pin=self.ingest_pinned), len(data)
        except (ingest.IngestError, KeyError, ValueError):
            return pickle.loads(data), None

    def _load_payload_file(self, path):
        """(payload, file length if parsed natively else None) of a comm_simulation file."""
        try:
            return ingest.load_file(path, layout=self._ingest_layout(), pin=self.ingest_pinned), os.path.getsize(path)
        except (ingest.IngestError, KeyError, ValueError):
            with open(path, "rb") as payload_file:
                return pickle.load(payload_file), None

    async def _client_report_arrived(self, sid, client_id, report):
        """plato/servers/base.py:775-811 with the payload file parsed natively and sized by its length.

        ``comm_simulation`` (the default, clients/base.py:92-96) hands payloads
        over as files the clients ``pickle.dump`` (clients/base.py:372-386); the
        reference ``pickle.load``s one and re-pickles it to size it (:791-796).
        """
        if not self.comm_simulation:
            await super()._client_report_arrived(sid, client_id, report)
            return
        from plato.config import Config

        self.reports[sid] = pickle.loads(report)
        self.client_payload[sid] = None
        self.client_chunks[sid] = []

        model_name = Config().trainer.model_name if hasattr(Config().trainer, "model_name") else "custom"
        model_name = model_name.replace("/", "_")
        checkpoint_path = Config().params["checkpoint_path"]
        payload, file_len = self._load_payload_file(f"{checkpoint_path}/{model_name}_client_{client_id}.pth")
        self.client_payload[sid] = payload
        if self.stage_on_arrival and isinstance(payload, ingest.ArenaStateDict):
            layout = self._ingest_layout()
            if layout is not None:
                self.round_engine(payload_codec(payload)).prestage(payload, layout, self._arrival_baseline())

        if self.wire_size_accounting and file_len is not None:
            payload_size = (file_len + sys.getsizeof(b"")) / 1024**2
        else:
            payload_size = sys.getsizeof(pickle.dumps(payload)) / 1024**2
        logging.info(
            "[%s] Received %.2f MB of payload data from client #%d (simulated).",
            self,
            payload_size,
            client_id,
        )
        self.comm_overhead += payload_size
        self.uplink_comm_time[client_id] = payload_size / (self.uplink_bandwidth / 8)

        await self.process_client_info(client_id, sid)

    async def _client_payload_arrived(self, sid, client_id):
        """plato/servers/base.py:817-831 with the join and the unpickle done natively."""
        assert len(self.client_chunks[sid]) > 0 and client_id in self.training_clients

        _data, wire_len = self._ingest(self.client_chunks[sid])
        self.client_chunks[sid] = []
        sizes = self.__dict__.setdefault("_plato_amd_wire_sizes", {})
        if self.client_payload[sid] is None:
            sizes[sid] = []
        if sizes.get(sid) is not None:
            # the bytes this part arrived as, for the size accounting below
            sizes[sid].append(wire_len)
        if self.stage_on_arrival and isinstance(_data, ingest.ArenaStateDict):
            layout = self._ingest_layout()
            if layout is not None:
                self.round_engine(payload_codec(_data)).prestage(_data, layout, self._arrival_baseline())

        if self.client_payload[sid] is None:
            self.client_payload[sid] = _data
        elif isinstance(self.client_payload[sid], list):
            self.client_payload[sid].append(_data)
        else:
            self.client_payload[sid] = [self.client_payload[sid]]
            self.client_payload[sid].append(_data)

    def _wire_payload_size(self, sid):
        """``Σ sys.getsizeof(pickle.dumps(part))`` of a payload, from the bytes it arrived as.

        The reference re-pickles every payload only to measure it
        (servers/base.py:839-846), ~45-130 ms per ResNet-18 payload.  A dict of
        tensors re-pickles to its wire length up to the decimal length of each
        storage's address, which pickle writes as the storage key (so the
        reference's own figure moves by a byte per tensor with where the
        allocator placed it); None when a part was not a native-ingested dict.
        """
        parts = self.__dict__.get("_plato_amd_wire_sizes", {}).pop(sid, None)
        payload = self.client_payload[sid]
        count = len(payload) if isinstance(payload, list) else 1
        if not self.wire_size_accounting or not parts or None in parts or len(parts) != count:
            return None
        return sum(n + sys.getsizeof(b"") for n in parts)

    async def _client_payload_done(self, sid, client_id, s3_key=None):
        """plato/servers/base.py:833-857 with the payload sized by its wire bytes, not re-pickled."""
        payload_size = self._wire_payload_size(sid) if s3_key is None else None
        if payload_size is None:
            await super()._client_payload_done(sid, client_id, s3_key)
            return
        logging.info(
            "[%s] Received %.2f MB of payload data from client #%d.",
            self,
            payload_size / 1024**2,
            client_id,
        )
        self.comm_overhead += payload_size / 1024**2
        await self.process_client_info(client_id, sid)
