"""QSGD payloads kept coded until the aggregation kernel decodes them.

Plato's server decodes QSGD uploads with the ``model_dequantize_qsgd`` inbound
processor (plato/processors/model_dequantize_qsgd.py:24-60): for every entry,
a big-endian header (``!f max_v``, ``!I numel``, ``!h ndim``, ``ndim x !h``)
and one byte per element (bit 7 sign, bits 0-6 ``|zeta|``), decoded in a
Python loop into an int64 tensor and multiplied out in fp32.  That loop is
the server's per-payload cost (seconds for ResNet-18).

:class:`Processor` is the drop-in replacement: it only parses the headers and
gathers the code bytes into one contiguous (optionally pinned) buffer, and
returns a :class:`QsgdPayload`.  The aggregation hooks recognise it
(``plato_codec == "qsgd"``), stage one byte per element to HBM and run
``plato_agg_fedavg_qsgd``, which decodes in registers exactly as the reference
does (``fp32(fp32(fp32(zeta) * max_v) / (level - 1))``) before the FedAvg chain.
"""

from __future__ import annotations

import struct
from collections import OrderedDict

import numpy as np
import torch


class QsgdPayload(OrderedDict):
    """A QSGD-coded state_dict: name -> 1-D ``torch.uint8`` code bytes (views of one buffer).

    ``max_v[name]`` is the entry's fp32 scale, ``shapes[name]`` the tensor
    shape, ``level`` the quantization level the client used.
    """

    plato_codec = "qsgd"

    def __init__(self, *args, max_v=None, shapes=None, level: int = 64, **kwargs):
        super().__init__(*args, **kwargs)
        self.max_v = dict(max_v or {})
        self.shapes = dict(shapes or {})
        self.level = int(level)

    def max_v_array(self, names) -> np.ndarray:
        return np.asarray([self.max_v[n] for n in names], dtype=np.float32)


def parse_layer(blob) -> tuple[float, tuple, int, int]:
    """Header of one entry (model_dequantize_qsgd.py:38-47): (max_v, shape, code offset, numel)."""
    mv = memoryview(blob)
    if len(mv) < 10:
        raise ValueError("QSGD layer shorter than its header")
    max_v = struct.unpack("!f", mv[0:4])[0]
    numel = struct.unpack("!I", mv[4:8])[0]
    ndim = struct.unpack("!h", mv[8:10])[0]
    if ndim < 0 or len(mv) < 10 + 2 * ndim:
        raise ValueError("bad QSGD header")
    shape = tuple(struct.unpack("!h", mv[10 + 2 * i:12 + 2 * i])[0] for i in range(ndim))
    count = 1
    for d in shape:
        count *= d
    start = 10 + 2 * ndim
    if count != numel or len(mv) < start + numel:
        raise ValueError(f"QSGD layer: numel {numel} does not match shape {shape} / payload length")
    return max_v, shape, start, numel


class Processor:
    """Drop-in for ``plato.processors.model_dequantize_qsgd.Processor`` (same arguments).

    Register it in plato/processors/registry.py under ``model_dequantize_qsgd``
    (or list it in ``server.inbound_processors``).  ``pin=True`` puts the code
    buffer in pinned memory for an asynchronous H2D copy.
    """

    def __init__(self, quantization_level=64, client_id=None, server_id=None, pin: bool = True, **kwargs):
        self.quantization_level = quantization_level
        self.client_id = client_id
        self.server_id = server_id
        self.pin = pin

    def process(self, data) -> QsgdPayload:
        headers = []
        total = 0
        for name, blob in data.items():
            max_v, shape, start, n = parse_layer(blob)
            headers.append((name, max_v, shape, start, n))
            total += n
        buf = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=self.pin and torch.cuda.is_available())
        host = buf.numpy()
        out = QsgdPayload(level=self.quantization_level)
        pos = 0
        for (name, max_v, shape, start, n), blob in zip(headers, data.values()):
            host[pos:pos + n] = np.frombuffer(blob, dtype=np.uint8, count=n, offset=start)
            out[name] = buf[pos:pos + n]
            out.max_v[name] = max_v
            out.shapes[name] = shape
            pos += n
        return out
