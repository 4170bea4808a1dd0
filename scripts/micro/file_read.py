"""Host microbenchmark: where the comm_simulation payload-file time goes (no GPU work).

Writes one pickled ResNet-18 state_dict to a temp file and times pickle.load,
the native parallel read at several thread counts, and parse + gather out of
a mapped file, so DESIGN.md can say what bounds plato_amd.ingest.load_file.
"""
import os
import pickle
import statistics
import sys
import tempfile
import time
from collections import OrderedDict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from plato_amd import ingest, workloads  # noqa: E402
from plato_amd.arena import ArenaLayout  # noqa: E402


def tm(fn, n=7):
    fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3


spec = workloads.resnet(18)
layout = ArenaLayout.from_shapes(spec)
g = torch.Generator().manual_seed(0)
sd = OrderedDict((n, torch.randn(s, generator=g) if r == "f32" else torch.randint(0, 9, s, generator=g))
                 for n, s, r in spec)
pin = torch.cuda.is_available()
with tempfile.NamedTemporaryFile(suffix=".pth", dir=os.environ.get("TMPDIR", "/tmp")) as f:
    pickle.dump(sd, f)
    f.flush()
    path = f.name
    buf = np.empty(os.path.getsize(path) + 4096, dtype=np.uint8)
    buf[:] = 0
    print(f"file {os.path.getsize(path)} B in {os.path.dirname(path)}, pinned arenas: {pin}")
    print(f"pickle.load                    {tm(lambda: pickle.load(open(path, 'rb'))):8.2f} ms")
    for t in (1, 2, 4, 8, 16):
        print(f"read_file threads={t:<2}           {tm(lambda: ingest.read_file(path, out=buf, threads=t)):8.2f} ms")
    data = ingest.read_file(path, out=buf)
    print(f"loads (parse+gather) from RAM   {tm(lambda: ingest.loads(data, layout=layout, pin=pin)):8.2f} ms")
    print(f"loads from np.memmap            "
          f"{tm(lambda: ingest.loads(np.memmap(path, dtype=np.uint8, mode='r'), layout=layout, pin=pin)):8.2f} ms")
    print(f"load_file                       {tm(lambda: ingest.load_file(path, layout=layout, pin=pin)):8.2f} ms")
