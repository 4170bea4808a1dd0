"""GPU parity of the flattened-model reductions (plato_amd/csrc/flat.hip) vs oracle/reductions.c.

The oracle is pinned to numpy / torch on the CPU (tests/test_reductions.py)
and to the reference's fixtures; here the device kernels must equal it bit
for bit on ragged sizes (every tail case of the 64- and 32-element blocks, the
cascade's partial groups, one- and two-pass thread splits).
"""

import numpy as np
import pytest
import torch

from oracle import reductions as R
from plato_amd import _lib

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SIZES = [1, 5, 31, 32, 33, 63, 64, 65, 95, 96, 100, 127, 129, 4095, 4096, 4097, 8191, 32767, 32768, 32769,
         100003, 262144 + 37]


def _rows(vecs):
    """[len, stride] device buffer (64-float aligned rows) and its row pointer table."""
    n = max(v.size for v in vecs)
    stride = max(64, -(-n // 64) * 64)
    buf = torch.zeros((len(vecs), stride), dtype=torch.float32, device=DEV)
    for r, v in enumerate(vecs):
        buf[r, : v.size] = torch.from_numpy(v)
    ptrs = torch.tensor([buf.data_ptr() + r * stride * 4 for r in range(len(vecs))], dtype=torch.int64, device=DEV)
    return buf, ptrs


@pytest.mark.parametrize("n", SIZES)
def test_sdot_pairs_equal_openblas_order(n):
    rng = np.random.default_rng(n)
    xs = [rng.standard_normal(n).astype(np.float32) for _ in range(3)]
    ys = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(3)]
    bx, px = _rows(xs)
    by, py = _rows(ys)
    out_xy = torch.full((3,), float("nan"), device=DEV)
    out_yy = torch.full((3,), float("nan"), device=DEV)
    _lib.call("plato_agg_sdot_pairs", px.data_ptr(), py.data_ptr(), 3, n, out_xy.data_ptr(), out_yy.data_ptr(),
              torch.cuda.current_stream().cuda_stream)
    got_xy, got_yy = out_xy.cpu().numpy(), out_yy.cpu().numpy()
    for j in range(3):
        assert got_xy[j].tobytes() == R.sdot(xs[j], ys[j]).tobytes(), (n, j)
        assert got_yy[j].tobytes() == R.sdot(ys[j], ys[j]).tobytes(), (n, j)


@pytest.mark.parametrize("n,npairs", [(n, 9) for n in SIZES + [(1 << 20) + 37]] +
                         [(n, 128) for n in SIZES if n <= 100003])
def test_sdot_shared_equals_openblas_order(n, npairs):
    """The split-chain shared-x kernel (every variant, the size-picked default) == OpenBLAS order: 9 pairs
    (ragged pair groups) and 128 (FedAdp's ResNet-18 round), with and without x.x as the virtual pair
    (x, x) after the last one (FedAdp's g.g)."""
    rng = np.random.default_rng(n + 7)
    x = rng.standard_normal(n).astype(np.float32)
    ys = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(npairs)]
    bx, _ = _rows([x])
    by, py = _rows(ys)
    k = len(ys)
    ws = torch.empty(_lib.lib().plato_agg_sdot_shared_workspace(k, 1) // 4, dtype=torch.float32, device=DEV)
    h = torch.cuda.current_stream().cuda_stream
    want_xy = [R.sdot(x, y).tobytes() for y in ys] + [R.sdot(x, x).tobytes()]
    want_yy = [R.sdot(y, y).tobytes() for y in ys] + [R.sdot(x, x).tobytes()]
    for variant in [None] + list(range(_lib.tune().plato_agg_tune_num_sdot_shared_variants())):
        for with_xx in (0, 1):
            out_xy = torch.full((k + 1,), float("nan"), device=DEV)
            out_yy = torch.full((k + 1,), float("nan"), device=DEV)
            if variant is None:
                _lib.call("plato_agg_sdot_shared", bx.data_ptr(), py.data_ptr(), k, n, with_xx, ws.data_ptr(),
                          out_xy.data_ptr(), out_yy.data_ptr(), h)
            else:
                _lib.tune_call("plato_agg_tune_sdot_shared", variant, bx.data_ptr(), py.data_ptr(), k, n, with_xx,
                          ws.data_ptr(), out_xy.data_ptr(), out_yy.data_ptr(), h)
            got_xy, got_yy = out_xy.cpu().numpy(), out_yy.cpu().numpy()
            for j in range(k + with_xx):
                assert got_xy[j].tobytes() == want_xy[j], (n, variant, with_xx, j)
                assert got_yy[j].tobytes() == want_yy[j], (n, variant, with_xx, j)
            if not with_xx:
                assert np.isnan(got_xy[k]) and np.isnan(got_yy[k])


@pytest.mark.parametrize("n", SIZES + [1 << 20, (1 << 20) + 3])
def test_norms_and_cosine_sum_equal_torch_order(n):
    rng = np.random.default_rng(n + 1)
    a = (rng.standard_normal(n) * 1e-2).astype(np.float32)
    bs = [(rng.standard_normal(n) * 3e-2).astype(np.float32) + a for _ in range(2)]
    buf, ptrs = _rows([a] + bs)
    chunk = torch.from_numpy(np.asarray([[0, 0, n, 0]], dtype=np.uint32).view(np.int32)).to(DEV)
    norms = torch.empty(3, dtype=torch.float32, device=DEV)
    h = torch.cuda.current_stream().cuda_stream
    _lib.call("plato_agg_entry_norms_f32", ptrs.data_ptr(), None, 3, None, None, chunk.data_ptr(), 1, None, 0, 1,
              n, 0, norms.data_ptr(), h)
    got_n = norms.cpu().numpy()
    for j, v in enumerate([a] + bs):
        assert got_n[j].tobytes() == R.torch_norm(v).tobytes(), (n, j)
    for threads in (1, 3, 8, 16, 64):
        ws = torch.empty(_lib.lib().plato_agg_torch_cosine_workspace(2, threads) // 4 + 1, device=DEV)
        out = torch.full((2,), float("nan"), device=DEV)
        _lib.call("plato_agg_torch_cosine_sum", buf.data_ptr(), ptrs.data_ptr() + 8, 2, n, norms.data_ptr(),
                  norms.data_ptr() + 4, 1e-8, threads, ws.data_ptr(), out.data_ptr(), h)
        got = out.cpu().numpy()
        for j in range(2):
            assert got[j].tobytes() == R.torch_cosine(a, bs[j], threads).tobytes(), (n, threads, j)


@pytest.mark.parametrize("n", [1000, (1 << 20) + 3])
def test_scaled_cosine_equals_torch_order(n):
    """plato_agg_scale_by_norm + every form of the scaled cascade cosine sum (Port's path), ragged chunkings."""
    rng = np.random.default_rng(n + 7)
    a = (rng.standard_normal(n) * 1e-2).astype(np.float32)
    bs = [(rng.standard_normal(n) * 3e-2).astype(np.float32) + a for _ in range(3)]
    buf, ptrs = _rows([a] + bs)
    chunk = torch.from_numpy(np.asarray([[0, 0, n, 0]], dtype=np.uint32).view(np.int32)).to(DEV)
    norms = torch.empty(4, dtype=torch.float32, device=DEV)
    h = torch.cuda.current_stream().cuda_stream
    _lib.call("plato_agg_entry_norms_f32", ptrs.data_ptr(), None, 4, None, None, chunk.data_ptr(), 1, None, 0, 1,
              n, 0, norms.data_ptr(), h)
    scaled = torch.empty(n, device=DEV)
    _lib.call("plato_agg_scale_by_norm", buf.data_ptr(), n, norms.data_ptr(), 1e-8, scaled.data_ptr(), h)
    for threads in (1, 5, 16):
        want = [R.torch_cosine(a, b, threads).tobytes() for b in bs]
        ws = torch.empty(_lib.lib().plato_agg_torch_cosine_workspace(3, threads) // 4 + 1, device=DEV)
        for v in [None] + list(range(_lib.tune().plato_agg_tune_num_cosine_variants())):
            out = torch.full((3,), float("nan"), device=DEV)
            args = (scaled.data_ptr(), ptrs.data_ptr() + 8, 3, n, norms.data_ptr() + 4, 1e-8, threads, ws.data_ptr(),
                    out.data_ptr(), h)
            if v is None:
                _lib.call("plato_agg_torch_cosine_sum_scaled", *args)
            else:
                _lib.tune_call("plato_agg_tune_torch_cosine_sum_scaled", v, *args)
            got = out.cpu().numpy()
            assert [got[j].tobytes() for j in range(3)] == want, (n, threads, v)


def test_cosine_of_a_zero_vector_uses_eps():
    n = 1000
    a = np.zeros(n, np.float32)
    b = np.random.default_rng(0).standard_normal(n).astype(np.float32)
    buf, ptrs = _rows([a, b])
    chunk = torch.from_numpy(np.asarray([[0, 0, n, 0]], dtype=np.uint32).view(np.int32)).to(DEV)
    norms = torch.empty(2, dtype=torch.float32, device=DEV)
    h = torch.cuda.current_stream().cuda_stream
    _lib.call("plato_agg_entry_norms_f32", ptrs.data_ptr(), None, 2, None, None, chunk.data_ptr(), 1, None, 0, 1,
              n, 0, norms.data_ptr(), h)
    ws = torch.empty(64, device=DEV)
    out = torch.empty(1, device=DEV)
    _lib.call("plato_agg_torch_cosine_sum", buf.data_ptr(), ptrs.data_ptr() + 8, 1, n, norms.data_ptr(),
              norms.data_ptr() + 4, 1e-8, 8, ws.data_ptr(), out.data_ptr(), h)
    assert out.item() == float(R.torch_cosine(a, b, 8)) == 0.0


@pytest.mark.parametrize("k", [1, 2, 3, 11])
def test_np_sumsq_variants_agree_bitwise(k):
    """Every np_sumsq kernel (the default's two clients per workgroup, three and four with ragged last
    groups, the one-client half-staged form, round-3 whole-chunk form, round-2 client-major form; not the
    timing probes) equals the product default, which the test below pins to numpy."""
    from plato_amd.arena import ArenaLayout
    from plato_amd.engine import FedAvgEngine

    spec = [("a", (7,), "f32"), ("b", (8192,), "f32"), ("n", (1,), "i64"), ("c", (8193,), "f32"),
            ("d", (70001,), "f32"), ("e", (129,), "f32")]
    layout = ArenaLayout.from_shapes(spec)
    rng = np.random.default_rng(k)
    bf = rng.standard_normal(layout.n_f32).astype(np.float32)
    bi = rng.integers(0, 100, layout.n_i64)
    eng = FedAvgEngine(DEV)
    base = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    rnd = eng.begin(base, k)
    rnd.put_baseline(base)
    for c in range(k):
        xf = (bf + rng.standard_normal(layout.n_f32).astype(np.float32) * 1e-2).astype(np.float32)
        rnd.put_client(c, layout.unpack(torch.from_numpy(xf), torch.from_numpy(bi)))
    want = rnd.np_sumsq(range(k))
    pieces, first, entry_of, n_chunks = rnd.layout._cache[("np_sumsq_pieces", str(eng.device))]
    tf = torch.from_numpy(np.asarray([rnd._pf[i] for i in range(k)], dtype=np.int64)).to(DEV)
    ws = torch.empty(max(1, eng.lib.plato_agg_np_sumsq_workspace(k, n_chunks) // 4), dtype=torch.float32, device=DEV)
    for v in [v for v in range(_lib.tune().plato_agg_tune_num_np_sumsq_variants()) if v not in (2, 3)]:  # probes
        out = torch.full((k, int(entry_of.size)), float("nan"), device=DEV)
        ws.fill_(float("nan"))  # a variant that leaves a chunk sum unwritten must not inherit the previous one's
        _lib.tune_call("plato_agg_tune_np_sumsq", v, tf.data_ptr(), k, rnd._base.f32.data_ptr(), pieces.data_ptr(),
                       first.data_ptr(), int(entry_of.size), n_chunks, ws.data_ptr(), out.data_ptr(),
                       torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert out.cpu().numpy().tobytes() == want[:, entry_of].tobytes(), v
    # delta arenas (null baseline): the default's kernels on the rows turned into x - b in place
    h = torch.cuda.current_stream().cuda_stream
    for c in range(k):
        _lib.call("plato_agg_compute_deltas", rnd._pf[c], rnd._pi[c], rnd._base.f32.data_ptr(),
                  rnd._base.i64.data_ptr(), rnd._pf[c], rnd._pi[c], layout.n_f32, layout.n_i64, h)
    for v in (None, 0, 6, 14):
        out = torch.full((k, int(entry_of.size)), float("nan"), device=DEV)
        ws.fill_(float("nan"))
        args = (tf.data_ptr(), k, None, pieces.data_ptr(), first.data_ptr(), int(entry_of.size), n_chunks,
                ws.data_ptr(), out.data_ptr(), h)
        if v is None:
            _lib.call("plato_agg_np_sumsq", *args)
        else:
            _lib.tune_call("plato_agg_tune_np_sumsq", v, *args)
        torch.cuda.synchronize()
        assert out.cpu().numpy().tobytes() == want[:, entry_of].tobytes(), ("deltas", v)
    with pytest.raises(ValueError, match="null baseline"):
        _lib.tune_call("plato_agg_tune_np_sumsq", 5, tf.data_ptr(), k, None, pieces.data_ptr(), first.data_ptr(),
                       int(entry_of.size), n_chunks, ws.data_ptr(), out.data_ptr(), h)


def test_np_sumsq_equals_numpy_order():
    from oracle import fedavg_oracle as ref
    from plato_amd.arena import ArenaLayout
    from plato_amd.engine import FedAvgEngine

    spec = [("conv.a", (7,), "f32"), ("conv.b", (129,), "f32"), ("n", (2,), "i64"), ("conv.c", (8192,), "f32"),
            ("conv.d", (8193,), "f32"), ("fc", (100003,), "f32"), ("conv.e", (512, 256, 3, 3), "f32"),
            ("s64", (64,), "f32"), ("s1000", (1000,), "f32"), ("s16377", (16377,), "f32"), ("s8191", (8191,), "f32")]
    layout = ArenaLayout.from_shapes(spec)
    rng = np.random.default_rng(4)
    bf = rng.standard_normal(layout.n_f32).astype(np.float32)
    bi = rng.integers(0, 100, layout.n_i64)
    xs = [((rng.standard_normal(layout.n_f32) * 1e-2).astype(np.float32) + bf, bi + 1) for _ in range(3)]
    eng = FedAvgEngine(DEV)
    rnd = eng.begin(layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi)), 3)
    rnd.put_baseline(layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi)))
    for c, (xf, xi) in enumerate(xs):
        rnd.put_client(c, layout.unpack(torch.from_numpy(xf), torch.from_numpy(xi)))
    got = rnd.np_sumsq(range(3))
    for c, (xf, _) in enumerate(xs):
        for e_i, e in enumerate(layout.entries):
            if e.region != "f32":
                assert got[c, e_i] == 0
                continue
            d = np.subtract(xf[e.offset:e.offset + e.numel], bf[e.offset:e.offset + e.numel], dtype=np.float32)
            assert got[c, e_i].tobytes() == np.sum(np.square(d.reshape(e.shape))).tobytes(), (c, e.name)
            assert got[c, e_i].tobytes() == R.np_sum(np.square(d)).tobytes()


@pytest.mark.parametrize("mode", [_lib.PLATO_AGG_FLAT_DELTA, _lib.PLATO_AGG_FLAT_CAST_DIFF, _lib.PLATO_AGG_FLAT_RAW])
@pytest.mark.parametrize("k", [1, 8, 11])
def test_flatten_modes_match_numpy(mode, k):
    """plato_agg_flatten: segments in a permuted order (fp32 and int64 entries, ragged sizes, every
    source/flat alignment), -1/lr on some segments, client groups of 8 with a ragged last group
    (the baseline is read once per group): equal to the numpy restatement of torch.cat / FedAdp's
    process_grad element by element."""
    rng = np.random.default_rng(100 * mode + k)
    sizes = [("a", 5, "f32"), ("n0", 1, "i64"), ("b", 4099, "f32"), ("c", 37, "f32"), ("n1", 3, "i64"),
             ("d", 70001, "f32"), ("e", 2, "f32")]
    off = {"f32": 0, "i64": 0}
    ents = []
    for name, n, reg in sizes:
        ents.append((name, n, reg, off[reg]))
        off[reg] += n
    n_f, n_i = off["f32"], off["i64"]
    lr = np.float32(0.0137)
    bf = rng.standard_normal(n_f).astype(np.float32)
    bi = rng.integers(-2**40, 2**40, n_i)
    xf = [bf + rng.standard_normal(n_f).astype(np.float32) * 0.1 for _ in range(k)]
    xi = [bi + rng.integers(-5, 5, n_i) for _ in range(k)]
    xi_raw = [rng.standard_normal(n_i).astype(np.float32) for _ in range(k)]  # RAW: fp32 values
    order = list(rng.permutation(len(ents)))
    rows, flat, want = [], 0, [[] for _ in range(k)]
    for j, idx in enumerate(order):
        name, n, reg, so = ents[idx]
        neg = j % 2 == 1
        rows.append([flat, so, n, (0 if reg == "f32" else 1) | ((1 if neg else 0) << 32)])
        flat += n
        for c in range(k):
            if reg == "f32":
                x = xf[c][so:so + n]
                v = x if mode == _lib.PLATO_AGG_FLAT_RAW else np.subtract(x, bf[so:so + n], dtype=np.float32)
                if neg:
                    v = np.divide(-v, lr, dtype=np.float32)
            elif mode == _lib.PLATO_AGG_FLAT_RAW:
                v = xi_raw[c][so:so + n]
                if neg:
                    v = np.divide(-v, lr, dtype=np.float32)
            elif mode == _lib.PLATO_AGG_FLAT_CAST_DIFF:
                v = np.subtract(xi[c][so:so + n].astype(np.float32), bi[so:so + n].astype(np.float32),
                                dtype=np.float32)
                if neg:
                    v = np.divide(-v, lr, dtype=np.float32)
            else:
                d = (xi[c][so:so + n] - bi[so:so + n]).astype(np.int64)
                v = np.divide((-d).astype(np.float32), lr, dtype=np.float32) if neg else d.astype(np.float32)
            want[c].append(np.asarray(v, dtype=np.float32))
    segs = torch.from_numpy(np.asarray(rows, dtype=np.uint64).view(np.int64)).to(DEV)
    stride = -(-flat // 64) * 64
    out = torch.full((k, stride), float("nan"), device=DEV)
    src_f = [torch.from_numpy(v).to(DEV) for v in xf]
    src_i = [torch.from_numpy(v).to(DEV) for v in (xi_raw if mode == _lib.PLATO_AGG_FLAT_RAW else xi)]
    ptrs = torch.tensor([t.data_ptr() for t in src_f] + [t.data_ptr() for t in src_i] +
                        [out.data_ptr() + r * stride * 4 for r in range(k)], dtype=torch.int64, device=DEV)
    b_f, b_i = torch.from_numpy(bf).to(DEV), torch.from_numpy(bi).to(DEV)
    _lib.call("plato_agg_flatten", mode, ptrs.data_ptr(), ptrs.data_ptr() + 8 * k, k, b_f.data_ptr(), b_i.data_ptr(),
              segs.data_ptr(), len(rows), flat, float(lr), ptrs.data_ptr() + 16 * k,
              torch.cuda.current_stream().cuda_stream)
    got = out.cpu().numpy()[:, :flat]
    for c in range(k):
        assert got[c].tobytes() == np.concatenate(want[c]).tobytes(), c
