"""GPU parity at BASELINE.json's full configuration sizes (size-independent properties).

The reference-generated fixtures cover C1, C2 (K=128), C4 (K=256) and a
ResNet-50/200 K=8 stand-in for C3 (tests/golden/).  At the full sizes of C3
(ResNet-50/200 x 1,024 clients, 98 GB of payloads on one MI355X) and C5
(ViT-L and GPT-2-medium shapes x 32 clients, 41-55 GB) the CPU oracle cannot
replay the whole job in seconds, so each test checks two properties that do
not depend on size:

* per-element exactness on a sample: the oracle's sequential fp32 chain
  (oracle/fedavg_oracle.py) over the K clients of 8,192 randomly chosen fp32
  elements and every int64 entry, bit for bit;
* kernel-variant invariance on the whole arena: the XCD-ordered and
  persistent variants produce the default variant's bits for every element.
"""

import zlib

import numpy as np
import pytest
import torch

from oracle import fedavg_oracle as ref
from plato_amd import synthetic, workloads
from plato_amd import weights as W
from plato_amd.arena import ArenaLayout
from plato_amd.engine import ClientSlab, DeviceArena, FedAvgEngine, fp32_weights
from plato_amd.synthetic import fill_baseline, fill_clients

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
SAMPLE = 8192

CONFIGS = {
    "C3_resnet50_200_k1024": (lambda: workloads.resnet(50, 200), 1024, "fedavg"),
    "C4_resnet18_k256_port": (lambda: workloads.resnet(18, 10), 256, "port"),
    "C5_vit_large_k32": (workloads.vit_large, 32, "fedavg"),
    "C5_gpt2_medium_k32": (workloads.gpt2_medium, 32, "fedavg"),
}


@pytest.fixture(scope="module")
def engine():
    return FedAvgEngine(DEV)


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_full_size_sampled_exact_and_variant_invariant(engine, name):
    spec, k, mode = CONFIGS[name]
    layout = ArenaLayout.from_shapes(spec())
    seed = 17
    base = DeviceArena(layout, DEV)
    slab = ClientSlab(layout, k, DEV)
    fill_baseline(base, seed)
    fill_clients(slab, base, seed, k)
    ns = synthetic.num_samples(k, seed)
    if mode == "port":
        weights = W.port(ns, synthetic.staleness(k, seed), similarity_weight=1, staleness_weight=3)
    else:
        weights = W.fedavg(ns)
    w = torch.from_numpy(fp32_weights(weights)).to(DEV)
    pf, pi = slab.row_pointers(range(k))
    tf, ti = torch.from_numpy(pf).to(DEV), torch.from_numpy(pi).to(DEV)
    outs = []
    for variant in (None, 6, 5):  # default, XCD-contiguous, persistent
        out_f = torch.full((layout.row_f32,), float("nan"), device=DEV)
        out_i = torch.full((layout.row_i64,), float("nan"), device=DEV)
        engine.variant = variant
        engine.launch_fedavg(layout, tf, ti, w, None, k, base.f32, base.i64, out_f, out_i)
        outs.append((out_f, out_i))
    engine.variant = None
    torch.cuda.synchronize()
    n_f, n_i = layout.n_f32, layout.n_i64
    for out_f, out_i in outs[1:]:
        assert torch.equal(out_f[:n_f].view(torch.int32), outs[0][0][:n_f].view(torch.int32))
        assert torch.equal(out_i[:n_i].view(torch.int32), outs[0][1][:n_i].view(torch.int32))

    rng = np.random.default_rng(zlib.crc32(name.encode()))
    idx = np.unique(np.concatenate([rng.integers(0, n_f, SAMPLE), [0, n_f - 1]]))
    idx_t = torch.from_numpy(idx).to(DEV)
    bf = base.f32[:n_f].index_select(0, idx_t).cpu().numpy()
    xf = slab.f32[:, :n_f].index_select(1, idx_t).cpu().numpy()
    bi = base.i64[:n_i].cpu().numpy()
    xi = slab.i64[:, :n_i].cpu().numpy()
    exp_f, exp_i = ref.fedavg_numpy(bf, bi, list(xf), list(xi), weights)
    got_f = outs[0][0][:n_f].index_select(0, idx_t).cpu().numpy()
    got_i = outs[0][1][:n_i].cpu().numpy()
    assert got_f.tobytes() == exp_f.tobytes()
    assert got_i.tobytes() == exp_i.tobytes()
    del slab, base, outs
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k", [128, 256])
def test_shared_baseline_kernels_match_one_client_forms_at_full_size(engine, k):
    """FedAtt norms and Polaris sums on K ResNet-18 clients: the product kernels (two clients per
    workgroup sharing the baseline loads; FedAtt from K = 96) equal, bit for bit on every (client, entry),
    the one-client forms that the small-size tests pin to the oracle (tuning variants 8 / 6)."""
    from plato_amd import _lib

    layout = ArenaLayout.from_shapes(workloads.resnet(18, 10))
    base = DeviceArena(layout, DEV)
    slab = ClientSlab(layout, k, DEV)
    fill_baseline(base, 23)
    fill_clients(slab, base, 23, k)
    pf, pi = slab.row_pointers(range(k))
    tf = torch.from_numpy(pf).to(DEV)
    ti = torch.from_numpy(pi).to(DEV)
    h = torch.cuda.current_stream(DEV).cuda_stream
    n_e = len(layout.entries)
    ef, ei = engine._norm_tables(layout)
    norm_args = (tf.data_ptr(), ti.data_ptr(), k, base.f32.data_ptr(), base.i64.data_ptr(), ef.data_ptr(), ef.shape[0],
                 ei.data_ptr(), ei.shape[0], n_e, layout.n_f32, layout.n_i64)
    prod = torch.full((k * n_e,), float("nan"), device=DEV)
    one = torch.full((k * n_e,), float("nan"), device=DEV)
    _lib.call("plato_agg_entry_norms_f32", *norm_args, prod.data_ptr(), h)
    _lib.tune_call("plato_agg_tune_entry_norms", 8, *norm_args, one.data_ptr(), h)
    torch.cuda.synchronize()
    assert not torch.isnan(prod).any()
    assert prod.cpu().numpy().tobytes() == one.cpu().numpy().tobytes()

    rows, first, n_chunks = [], [], 0
    for idx, e in enumerate(layout.entries):
        if e.region == "f32" and e.numel:
            rows.append((idx, e.offset, e.offset + e.numel, 0))
            first.append(n_chunks)
            n_chunks += -(-e.numel // 8192)
    pieces = torch.from_numpy(np.asarray(rows, dtype=np.uint32).view(np.int32).copy()).to(DEV)
    firsts = torch.from_numpy(np.asarray(first, dtype=np.uint32).view(np.int32)).to(DEV)
    ws = torch.empty(max(1, engine.lib.plato_agg_np_sumsq_workspace(k, n_chunks) // 4), device=DEV)
    sq_args = (tf.data_ptr(), k, base.f32.data_ptr(), pieces.data_ptr(), firsts.data_ptr(), len(rows), n_chunks,
               ws.data_ptr())
    sq_prod = torch.full((k, len(rows)), float("nan"), device=DEV)
    sq_one = torch.full((k, len(rows)), float("nan"), device=DEV)
    _lib.call("plato_agg_np_sumsq", *sq_args, sq_prod.data_ptr(), h)
    ws.fill_(float("nan"))
    _lib.tune_call("plato_agg_tune_np_sumsq", 6, *sq_args, sq_one.data_ptr(), h)
    torch.cuda.synchronize()
    assert not torch.isnan(sq_prod).any()
    assert sq_prod.cpu().numpy().tobytes() == sq_one.cpu().numpy().tobytes()
