"""Native payload ingestion (libplato_ingest.so) vs pickle.loads, on the CPU.

The reference server turns payload bytes back into a state_dict with
pickle.loads (plato/servers/base.py:822).  The native parser must produce the
same keys, dtypes, shapes and values, land them in the engine's arena layout,
and refuse (never execute) anything that is not a pickled dict of tensors.
"""

import io
import os
import pickle
import random
import subprocess
import sys
import time
from collections import OrderedDict

import numpy as np
import pytest
import torch

from plato_amd import ingest, workloads
from plato_amd.arena import ArenaLayout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(not os.path.exists(ingest.LIB_PATH), reason="libplato_ingest.so not built")


def state_dict(spec, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = OrderedDict()
    for name, shape, region in spec:
        if region == "f32":
            out[name] = torch.randn(shape, generator=g)
        else:
            out[name] = torch.randint(0, 10**6, shape, generator=g)
    return out


def assert_same(a, b):
    assert list(a.keys()) == list(b.keys())
    for k in a:
        assert a[k].dtype == b[k].dtype, k
        assert tuple(a[k].shape) == tuple(b[k].shape), k
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("proto", [3, 4, 5])
def test_matches_pickle_loads_resnet18(proto):
    sd = state_dict(workloads.resnet(18), 1)
    data = pickle.dumps(sd, protocol=proto)
    assert_same(ingest.loads(data), pickle.loads(data))


def test_protocol2_is_refused_cleanly():
    """Protocol 2 has no bytes opcode (storage blobs become _codecs.encode calls): refused."""
    with pytest.raises(ingest.IngestError, match="_codecs"):
        ingest.loads(pickle.dumps(state_dict(workloads.lenet5()), protocol=2))


def test_arena_layout_matches_pack():
    spec = workloads.resnet(18)
    sd = state_dict(spec, 2)
    layout = ArenaLayout.from_shapes(spec)
    got = ingest.loads(pickle.dumps(sd), layout=layout)
    assert isinstance(got, ingest.ArenaStateDict) and got.layout_signature == layout.signature
    f = torch.empty(layout.row_f32)
    i = torch.empty(layout.row_i64, dtype=torch.int64)
    layout.pack(sd, f, i)
    assert torch.equal(got.arena_f32[: layout.n_f32], f[: layout.n_f32])
    assert torch.equal(got.arena_i64[: layout.n_i64], i[: layout.n_i64])
    assert_same(got, sd)
    # and it pickles back like the plain dict the reference sizes (servers/base.py:839-846)
    assert_same(pickle.loads(pickle.dumps(got)), sd)


def test_odd_tensors():
    base = torch.arange(24, dtype=torch.float32).reshape(4, 6)
    sd = OrderedDict()
    sd["tied_a"] = base
    sd["tied_b"] = base                      # shared storage (tied weights)
    sd["transposed"] = base.t()              # non-contiguous
    sd["slice"] = base[1:3, 2:5]             # storage offset + strides
    sd["scalar_i64"] = torch.tensor(7)
    sd["empty"] = torch.empty(0, 3)
    sd["half"] = torch.randn(5).half()
    sd["bf16"] = torch.randn(5).bfloat16()
    sd["f64"] = torch.randn(3, dtype=torch.float64)
    sd["bool"] = torch.tensor([True, False, True])
    sd["u8"] = torch.arange(7, dtype=torch.uint8)
    sd["i32"] = torch.arange(-3, 3, dtype=torch.int32)
    data = pickle.dumps(sd)
    assert_same(ingest.loads(data), pickle.loads(data))
    plain = dict(sd)
    assert_same(ingest.loads(pickle.dumps(plain)), plain)


def test_layout_mismatch_is_rejected():
    layout = ArenaLayout.from_shapes(workloads.lenet5())
    sd = state_dict(workloads.lenet5())
    sd["fc5.bias"] = torch.zeros(11)
    with pytest.raises(ValueError):
        ingest.loads(pickle.dumps(sd), layout=layout)
    del sd["fc5.bias"]
    with pytest.raises(KeyError):
        ingest.loads(pickle.dumps(sd), layout=layout)


class Evil:
    def __reduce__(self):
        return (os.system, ("touch /tmp/plato_ingest_pwned",))


def test_never_executes_and_rejects_foreign_objects():
    if os.path.exists("/tmp/plato_ingest_pwned"):
        os.remove("/tmp/plato_ingest_pwned")
    for obj in [OrderedDict(a=Evil()), Evil(), [torch.zeros(2)], OrderedDict(a=[1, 2]), {"a": 1.5},
                OrderedDict(a=torch.zeros(2), b="x")]:
        with pytest.raises(ingest.IngestError):
            ingest.loads(pickle.dumps(obj))
    assert not os.path.exists("/tmp/plato_ingest_pwned")


class _StridedTensor:
    """Pickles as _rebuild_tensor_v2(storage, offset, size, stride, ...) with chosen geometry."""

    def __init__(self, storage, offset, size, stride):
        self.args = (storage, offset, size, stride, False, OrderedDict())

    def __reduce__(self):
        return (torch._utils._rebuild_tensor_v2, self.args)


def _hostile_geometry_payloads():
    big = 2**63 - 1
    u8 = torch.zeros(2, dtype=torch.uint8)._typed_storage()
    f32 = torch.zeros(16)._typed_storage()
    yield _StridedTensor(u8, 0, (2, 2, 2), (big, big, 3))     # extents wrap to 1
    yield _StridedTensor(u8, 0, (2,), (big,))                # one huge stride
    yield _StridedTensor(f32, 2**62, (1,), (1,))             # offset far outside
    yield _StridedTensor(f32, 15, (2,), (1,))                # one past the end
    yield _StridedTensor(f32, 1, (2, 2), (2**62, 2**62))     # 2*2^62 wraps to 0 in a 64-bit sum
    yield _StridedTensor(f32, 0, (4, 5), (5, 1))             # 20 > 16 elements


@pytest.mark.parametrize("case", range(6))
def test_hostile_strides_and_offsets_are_rejected(case):
    """Geometry that would read outside the storage (wrapping extents included) is a format error."""
    obj = list(_hostile_geometry_payloads())[case]
    data = pickle.dumps(OrderedDict(w=obj), protocol=4)
    with pytest.raises(ingest.IngestError, match="outside its storage"):
        ingest.loads(data)


def test_legal_strided_tensor_still_loads():
    base = torch.arange(24, dtype=torch.float32)
    data = pickle.dumps(OrderedDict(w=_StridedTensor(base._typed_storage(), 2, (3, 4), (1, 5))), protocol=4)
    got = ingest.loads(data)
    assert torch.equal(got["w"], base.as_strided((3, 4), (1, 5), 2))


def test_deep_nesting_is_refused_without_recursion():
    """200k nested 1-tuples: parsed into a pool and refused (not a dict), no stack overflow."""
    code = r"""
import sys
sys.path.insert(0, sys.argv[1])
from plato_amd import ingest
for body in (b")" + b"\x85" * 200000, b"]" + b"\x94" + b"h\x00a" * 100000):
    try:
        ingest.loads(b"\x80\x04" + body + b".")
    except ingest.IngestError:
        pass
    else:
        raise SystemExit("accepted")
print("OK")
"""
    proc = subprocess.run([sys.executable, "-c", code, ROOT], capture_output=True, text=True, timeout=300)
    assert proc.returncode == 0 and "OK" in proc.stdout, proc.stderr[-2000:]


def test_mutating_an_arena_payload_detaches_its_arena():
    spec = workloads.lenet5(10)
    layout = ArenaLayout.from_shapes(spec)
    sd = state_dict(spec, 3)
    got = ingest.loads(pickle.dumps(sd), layout=layout)
    assert got.layout_signature == layout.signature and got.arena_f32 is not None
    key = next(iter(got))
    got[key] = torch.zeros_like(got[key])
    assert got.layout_signature is None and got.arena_f32 is None
    for mutate in (lambda d: d.pop(key), lambda d: d.update({key: d[key]}), lambda d: d.clear(),
                   lambda d: d.popitem()):
        fresh = ingest.loads(pickle.dumps(sd), layout=layout)
        mutate(fresh)
        assert fresh.layout_signature is None


def test_truncation_and_corruption_fuzz():
    """Every prefix and random byte flips: error or a result, never a crash (subprocess)."""
    code = r'''
import pickle, random, sys
from collections import OrderedDict
import torch
sys.path.insert(0, sys.argv[1])
from plato_amd import ingest
sd = OrderedDict(w=torch.randn(3, 4), b=torch.arange(5), n=torch.tensor(3))
data = pickle.dumps(sd)
ok = err = 0
for cut in range(len(data)):
    try:
        ingest.loads(data[:cut]); ok += 1
    except (ingest.IngestError, KeyError, ValueError):
        err += 1
rnd = random.Random(0)
for _ in range(3000):
    b = bytearray(data)
    for _ in range(rnd.randint(1, 4)):
        b[rnd.randrange(len(b))] = rnd.randrange(256)
    try:
        ingest.loads(bytes(b)); ok += 1
    except (ingest.IngestError, KeyError, ValueError, RuntimeError, OverflowError):
        err += 1
print("OK", ok, err)
'''
    proc = subprocess.run([sys.executable, "-c", code, ROOT], capture_output=True, text=True, timeout=300)
    assert proc.returncode == 0 and "OK" in proc.stdout, proc.stderr[-2000:]


def test_faster_than_pickle_loads():
    sd = state_dict(workloads.resnet(18), 3)
    layout = ArenaLayout.from_shapes(workloads.resnet(18))
    data = pickle.dumps(sd)
    ingest.loads(data, layout=layout)
    t0 = time.perf_counter()
    for _ in range(5):
        pickle.loads(data)
    t_pickle = (time.perf_counter() - t0) / 5
    t0 = time.perf_counter()
    for _ in range(5):
        ingest.loads(data, layout=layout)
    t_native = (time.perf_counter() - t0) / 5
    print(f"pickle.loads {t_pickle * 1e3:.1f} ms, native {t_native * 1e3:.1f} ms")
    assert t_native < t_pickle


def test_join_matches_bytes_join_and_chunked_path_is_faster():
    """Native join of 1 MiB transport chunks == b"".join; chunked ingest beats join + pickle.loads."""
    sd = state_dict(workloads.resnet(18), 4)
    layout = ArenaLayout.from_shapes(workloads.resnet(18))
    data = pickle.dumps(sd)
    chunks = [data[i:i + 2**20] for i in range(0, len(data), 2**20)]
    assert ingest.join(chunks).tobytes() == data
    assert ingest.join([]).size == 0 and ingest.join([b"", b"ab", b""]).tobytes() == b"ab"
    assert_same(ingest.loads_chunks(chunks, layout=layout), sd)
    ingest.loads_chunks(chunks, layout=layout)
    t0 = time.perf_counter()
    for _ in range(3):
        pickle.loads(b"".join(chunks))
    t_ref = (time.perf_counter() - t0) / 3
    t0 = time.perf_counter()
    for _ in range(3):
        ingest.loads_chunks(chunks, layout=layout)
    t_native = (time.perf_counter() - t0) / 3
    print(f"join + pickle.loads {t_ref * 1e3:.1f} ms, native join + parse + gather {t_native * 1e3:.1f} ms")
    assert t_native < t_ref


def test_wire_ingest_mixin_replaces_pickle_loads():
    """The overridden _client_payload_arrived (servers/base.py:817-831) yields the same payload."""
    import asyncio

    from plato_amd.servers import WireIngestMixin

    spec = workloads.resnet(18)
    base = state_dict(spec, 5)
    client = state_dict(spec, 6)
    data = pickle.dumps(client)

    class Algo:
        def extract_weights(self):
            return base

    class S(WireIngestMixin):
        ingest_pinned = False

        def __init__(self):
            self.algorithm = Algo()
            self.client_chunks = {"sid": [data[i:i + 2**20] for i in range(0, len(data), 2**20)]}
            self.client_payload = {"sid": None}
            self.training_clients = {3: 1}

    s = S()
    asyncio.run(s._client_payload_arrived("sid", 3))
    got = s.client_payload["sid"]
    assert isinstance(got, ingest.ArenaStateDict)
    assert_same(got, client)
    # a non-state-dict payload goes through pickle.loads like the reference
    s.client_chunks["sid"] = [pickle.dumps(["features", 1, 2])]
    s.client_payload["sid"] = None
    asyncio.run(s._client_payload_arrived("sid", 3))
    assert s.client_payload["sid"] == ["features", 1, 2]


def test_repickled_payload_is_payload_sized():
    """Arena-backed tensors re-pickle their own bytes only (servers/base.py:839-846 sizes payloads so).

    pickle writes each storage's address as its key, so sizes move by a byte
    per tensor with where the allocator put the storage; nothing else differs.
    """
    spec = workloads.resnet(18)
    sd = state_dict(spec, 7)
    data = pickle.dumps(sd)
    ref = len(pickle.dumps(pickle.loads(data)))
    slack = 2 * len(sd) + 64
    for got in (ingest.loads(data, layout=ArenaLayout.from_shapes(spec)), ingest.loads(data)):
        n = len(pickle.dumps(got))
        assert abs(n - ref) <= slack, (n, ref)
        assert_same(pickle.loads(pickle.dumps(got)), sd)
        # the storages are slices of the arena (no copy) and keep it alive
        first = next(iter(got.values()))
        assert first.untyped_storage().nbytes() == first.numel() * first.element_size()


def test_wire_size_accounting_matches_repickling():
    """_client_payload_done (servers/base.py:833-857): same log, comm_overhead and hand-off, no re-pickle."""
    import asyncio

    from plato_amd.servers import WireIngestMixin

    spec = workloads.lenet5()
    base = state_dict(spec, 8)
    parts = [pickle.dumps(state_dict(spec, 9)), pickle.dumps(state_dict(spec, 10))]

    class Algo:
        def extract_weights(self):
            return base

    class Reference:  # the reference's sizing, as the mixin's fallback
        async def _client_payload_done(self, sid, client_id, s3_key=None):
            payload = self.client_payload[sid]
            items = payload if isinstance(payload, list) else [payload]
            self.comm_overhead += sum(sys.getsizeof(pickle.dumps(p)) for p in items) / 1024**2
            await self.process_client_info(client_id, sid)

    class S(WireIngestMixin, Reference):
        ingest_pinned = False

        def __init__(self, wire):
            self.wire_size_accounting = wire
            self.algorithm = Algo()
            self.client_chunks = {"sid": []}
            self.client_payload = {"sid": None}
            self.training_clients = {3: 1}
            self.comm_overhead = 0.0
            self.handed = []

        async def process_client_info(self, client_id, sid):
            self.handed.append((client_id, sid))

        async def receive(self, payload_parts):
            for p in payload_parts:
                self.client_chunks["sid"] = [p[i:i + 4096] for i in range(0, len(p), 4096)]
                await self._client_payload_arrived("sid", 3)
            await self._client_payload_done("sid", 3)

    for n_parts in (1, 2):
        fast, slow = S(True), S(False)
        asyncio.run(fast.receive(parts[:n_parts]))
        asyncio.run(slow.receive(parts[:n_parts]))
        assert fast.handed == slow.handed == [(3, "sid")]
        n_tensors = n_parts * len(spec)
        assert abs(fast.comm_overhead - slow.comm_overhead) * 1024**2 <= 2 * n_tensors + 64
        assert fast.comm_overhead * 1024**2 == sum(len(p) + sys.getsizeof(b"") for p in parts[:n_parts])
    # a part that pickle.loads had to take is sized the reference's way (a list payload is
    # taken as its parts there, servers/base.py:840-842)
    s = S(True)
    asyncio.run(s.receive([pickle.dumps(["features", 1, 2])]))
    assert s.comm_overhead * 1024**2 == sum(sys.getsizeof(pickle.dumps(x)) for x in ["features", 1, 2])


def test_load_file_matches_pickle_load(tmp_path):
    """comm_simulation payload files (clients/base.py:372-386 -> servers/base.py:791-792)."""
    spec = workloads.resnet(18)
    sd = state_dict(spec, 11)
    path = tmp_path / "resnet_18_client_1.pth"
    with open(path, "wb") as f:
        pickle.dump(sd, f)
    assert ingest.read_file(str(path)).tobytes() == path.read_bytes()
    for threads in (1, 0):
        assert_same(ingest.load_file(str(path), layout=ArenaLayout.from_shapes(spec), threads=threads), sd)
    assert_same(ingest.load_file(str(path)), sd)
    small = tmp_path / "small.pth"  # smaller than the scratch buffer left by the first load
    with open(small, "wb") as f:
        pickle.dump(state_dict(workloads.lenet5(), 12), f)
    assert_same(ingest.load_file(str(small)), pickle.load(open(small, "rb")))
    empty = tmp_path / "empty.pth"
    empty.write_bytes(b"")
    assert ingest.read_file(str(empty)).size == 0
    with pytest.raises(ingest.IngestError):
        ingest.load_file(str(empty))
    with pytest.raises(FileNotFoundError):
        ingest.load_file(str(tmp_path / "missing.pth"))
    # pickle.load from the file: ~90 ms per ResNet-18 payload here; native read + parse + gather
    ingest.load_file(str(path), layout=ArenaLayout.from_shapes(spec))
    t0 = time.perf_counter()
    for _ in range(3):
        with open(path, "rb") as f:
            pickle.load(f)
    t_ref = (time.perf_counter() - t0) / 3
    t0 = time.perf_counter()
    for _ in range(3):
        ingest.load_file(str(path), layout=ArenaLayout.from_shapes(spec))
    t_native = (time.perf_counter() - t0) / 3
    print(f"pickle.load {t_ref * 1e3:.1f} ms, native load_file {t_native * 1e3:.1f} ms")
    assert t_native < t_ref
