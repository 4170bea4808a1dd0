"""zstd-compressed payloads (model_compress / model_decompress) through libplato_ingest, on the CPU.

The reference's server runs ``pickle.loads(zstd.decompress(data))``
(plato/processors/model_decompress.py:24) on what clients' model_compress sent,
``zstd.compress(pickle.dumps(state_dict), level)`` (model_compress.py:25).
The python ``zstd`` package is not installed here (parity for this codec is
pinned by the zstd frame format, not by reference fixtures): frames are
cross-checked against an independent zstd implementation, pyarrow's bundled
libzstd, in both directions, and the decompressed payload must equal
``pickle.loads`` of the original bytes.
"""

import pickle
from collections import OrderedDict

import numpy as np
import pytest
import torch

from plato_amd import ingest, workloads
from plato_amd.arena import ArenaLayout

pytestmark = pytest.mark.skipif(
    not (ingest.os.path.exists(ingest.LIB_PATH) and ingest.zstd_available()),
    reason="libplato_ingest.so not built or libzstd.so.1 absent")

pa = pytest.importorskip("pyarrow")


def _state_dict(spec, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = OrderedDict()
    for name, shape, region in spec:
        out[name] = torch.randn(shape, generator=g) if region == "f32" else torch.randint(0, 10**6, shape, generator=g)
    return out


def _same(a, b):
    assert list(a) == list(b)
    for k in a:
        assert a[k].dtype == b[k].dtype and torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("level", [1, 3, 19])
def test_round_trip_and_cross_implementation(level):
    raw = pickle.dumps(_state_dict(workloads.lenet5(), level))
    frame = ingest.zstd_compress(raw, level)
    assert ingest.zstd_decompress(frame).tobytes() == raw
    # our frame decodes with pyarrow's zstd, and pyarrow's with ours
    assert pa.decompress(frame, decompressed_size=len(raw), codec="zstd", asbytes=True) == raw
    theirs = pa.compress(raw, codec="zstd", asbytes=True)
    assert ingest.zstd_decompress(theirs).tobytes() == raw


def test_streamed_frame_without_content_size():
    raw = pickle.dumps(_state_dict(workloads.lenet5(), 5)) * 9  # > the initial 4x guess
    sink = pa.BufferOutputStream()
    with pa.CompressedOutputStream(sink, "zstd") as out:
        for i in range(0, len(raw), 4096):
            out.write(raw[i:i + 4096])
    frame = sink.getvalue().to_pybytes()
    lib = ingest.lib()
    buf = np.frombuffer(frame, dtype=np.uint8)
    size = lib.plato_ingest_zstd_content_size(buf.ctypes.data, buf.size)
    assert size in (len(raw), ingest.EUNKNOWNSIZE)
    assert ingest.zstd_decompress(frame).tobytes() == raw


def test_concatenated_frames():
    a, b = b"x" * 1000, pickle.dumps(list(range(100)))
    frames = ingest.zstd_compress(a, 1) + ingest.zstd_compress(b, 1)
    assert ingest.zstd_decompress(frames).tobytes() == a + b


def test_corrupt_and_truncated_frames_raise():
    raw = pickle.dumps(_state_dict(workloads.lenet5(), 2))
    frame = bytearray(ingest.zstd_compress(raw, 3))
    for cut in (0, 4, 12, len(frame) // 2, len(frame) - 1):
        with pytest.raises(ingest.IngestError):
            ingest.zstd_decompress(bytes(frame[:cut]))
    with pytest.raises(ingest.IngestError):
        ingest.zstd_decompress(b"not a zstd frame at all")
    rng = np.random.default_rng(0)
    for _ in range(50):  # byte flips: an error or some bytes, never a crash
        bad = bytearray(frame)
        bad[int(rng.integers(0, len(bad)))] ^= 1 << int(rng.integers(0, 8))
        try:
            ingest.zstd_decompress(bytes(bad))
        except ingest.IngestError:
            pass


def test_destination_capacity_is_enforced():
    raw = b"abc" * 5000
    frame = np.frombuffer(ingest.zstd_compress(raw, 1), dtype=np.uint8)
    out = np.empty(100, dtype=np.uint8)
    lib = ingest.lib()
    assert lib.plato_ingest_zstd_decompress(frame.ctypes.data, frame.size, out.ctypes.data, out.size) \
        == ingest.ECAPACITY


def test_processor_matches_reference_decompress_then_pickle_loads():
    from plato_amd.processors import zstd as zp

    sd = _state_dict(workloads.resnet(18), 7)
    data = zp.CompressProcessor(compression_level=1).process(sd)   # the client's model_compress
    layout = ArenaLayout.from_state_dict(sd)

    class Trainer:
        class model:
            @staticmethod
            def state_dict():
                return sd

    got = zp.Processor(server_id=0, trainer=Trainer, pin=False).process(data)
    _same(got, pickle.loads(ingest.zstd_decompress(data).tobytes()))
    _same(got, sd)
    assert isinstance(got, ingest.ArenaStateDict) and got.layout_signature == layout.signature
    # without a trainer: a plain OrderedDict of tensors
    _same(zp.Processor(server_id=0).process(data), sd)


def test_processor_falls_back_for_non_tensor_payloads():
    from plato_amd.processors import zstd as zp

    payload = {"weights": [1, 2, 3], "note": "features"}
    data = zp.CompressProcessor(compression_level=2).process(payload)
    assert zp.Processor(server_id=0).process(data) == payload
