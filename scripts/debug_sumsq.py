"""Which (client, entry) sums of an np_sumsq variant differ from the default, on ResNet-18 (debug aid)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from plato_amd import _lib, workloads  # noqa: E402
from plato_amd.arena import ArenaLayout  # noqa: E402
from plato_amd.engine import FedAvgEngine  # noqa: E402
from plato_amd.synthetic import fill_baseline, fill_clients  # noqa: E402

v = int(sys.argv[1]) if len(sys.argv) > 1 else 6
dev = torch.device("cuda", 0)
lay = ArenaLayout.from_shapes(workloads.resnet(18, 10))
eng = FedAvgEngine(dev)
from plato_amd.engine import DeviceArena  # noqa: E402
base = DeviceArena(lay, dev)
fill_baseline(base, 0)
baseline = lay.unpack(base.f32[: lay.n_f32].cpu(), base.i64[: lay.n_i64].cpu())
for k in (3, 16, 128):
    r = eng.begin(baseline, k)
    r.put_baseline(baseline)
    torch.cuda.synchronize(dev)
    fill_clients(r.slab, r.engine._base, 0, k)
    for s in range(k):
        pf, pi = r.slab.row_pointers([s])
        r._pf[s], r._pi[s] = int(pf[0]), int(pi[0])
        r.staged[s] = True
    torch.cuda.synchronize(dev)
    want = r.np_sumsq(range(k))
    pieces, first, entry_of, n_chunks = r.layout._cache[("np_sumsq_pieces", str(dev))]
    tf = torch.from_numpy(np.asarray([r._pf[i] for i in range(k)], dtype=np.int64)).to(dev)
    ws = torch.zeros(max(1, eng.lib.plato_agg_np_sumsq_workspace(k, n_chunks) // 4), device=dev)
    out = torch.full((k, int(entry_of.size)), float("nan"), device=dev)
    _lib.tune_call("plato_agg_tune_np_sumsq", v, tf.data_ptr(), k, r._base.f32.data_ptr(), pieces.data_ptr(),
                   first.data_ptr(), int(entry_of.size), n_chunks, ws.data_ptr(), out.data_ptr(),
                   torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    cs = ws[: k * n_chunks].view(k, n_chunks).cpu().numpy()
    off = (k * n_chunks * 4 + 15) // 16 * 16 // 8
    tab = ws.view(torch.int64)[off: off + 2 * n_chunks].view(n_chunks, 2).cpu().numpy()
    full = [c for c in range(n_chunks) if tab[c, 1] == 8192][:5]
    print(json.dumps({"K": k, "tab_head": tab[:8].tolist(), "full_chunks": full,
                      "chunk_sums_full_k0": [float(cs[0, c]) for c in full],
                      "n_full": int((tab[:, 1] == 8192).sum())}), flush=True)
    got = out.cpu().numpy()
    exp = want[:, entry_of]
    bad = got.view(np.uint32) != exp.view(np.uint32)
    rel = np.abs(got - exp) / np.maximum(np.abs(exp), 1e-30)
    print(json.dumps({"variant": v, "K": k, "n_chunks": int(n_chunks), "mismatch_frac": float(bad.mean()),
                      "bad_clients": sorted(set(np.nonzero(bad)[0].tolist()))[:20],
                      "bad_pieces": sorted(set(np.nonzero(bad)[1].tolist()))[:20],
                      "max_rel": float(np.nanmax(rel)) if bad.any() else 0.0, "nan": int(np.isnan(got).sum())}),
          flush=True)
    del r
