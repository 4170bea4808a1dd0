"""Host-side timing of native ingestion on the GPU box: parse + gather of a pickled ResNet-18 payload
into a pinned arena, by thread count, against a plain 16-thread copy of the same bytes."""
import json
import os
import pickle
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from plato_amd import ingest, workloads  # noqa: E402
from plato_amd.arena import ArenaLayout  # noqa: E402

layout = ArenaLayout.from_shapes(workloads.resnet(18, 10))
sd = layout.unpack(torch.randn(layout.n_f32), torch.zeros(layout.n_i64, dtype=torch.int64))
data = pickle.dumps(type(sd)((n, t.clone()) for n, t in sd.items()))
keep = []
for th in (0, 1, 4, 8, 16):
    ts = []
    for r in range(12):
        t0 = time.perf_counter()
        out = ingest.loads(data, layout=layout, pin=True, threads=th)
        ts.append(time.perf_counter() - t0)
        keep.append(out)
        if len(keep) > 4:
            keep.pop(0)
    print(json.dumps({"threads": th, "ms_median": round(statistics.median(ts[2:]) * 1e3, 3),
                      "ms_min": round(min(ts) * 1e3, 3), "GBps": round(len(data) / statistics.median(ts[2:]) / 1e9, 1)}),
          flush=True)
# the parse alone and a pinned-to-pinned torch copy of the arena bytes
t0 = time.perf_counter()
for _ in range(10):
    infos = ingest.parse(data) if hasattr(ingest, "parse") else None
print(json.dumps({"parse_only_ms": round((time.perf_counter() - t0) * 100, 3) if infos is not None else None}))
src = torch.frombuffer(bytearray(data), dtype=torch.uint8)
dst = torch.empty(len(data), dtype=torch.uint8, pin_memory=True)
dst.copy_(src)
t0 = time.perf_counter()
for _ in range(10):
    dst.copy_(src)
print(json.dumps({"torch_copy_ms": round((time.perf_counter() - t0) * 100, 3), "threads": torch.get_num_threads()}))
