"""ASan/UBSan build of the ingestion parser driven by a native fuzzer (host code only)."""

import os
import pickle
import shutil
import subprocess
from collections import OrderedDict

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_parser_under_address_and_ub_sanitizers(tmp_path):
    exe = tmp_path / "fuzz_ingest"
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-pthread", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "native", "fuzz_ingest.cpp"),
           os.path.join(ROOT, "plato_amd", "csrc", "ingest.cpp"), "-o", str(exe)]
    build = subprocess.run(cmd, capture_output=True, text=True)
    if build.returncode != 0:
        pytest.skip("sanitizer toolchain unavailable: " + build.stderr[-300:])
    samples = []
    sd = OrderedDict(w=torch.randn(3, 4), b=torch.arange(5), n=torch.tensor(3), h=torch.randn(2).half())
    sd["t"] = sd["w"].t()
    for proto in (3, 4, 5):
        path = tmp_path / f"sd{proto}.pkl"
        path.write_bytes(pickle.dumps(sd, protocol=proto))
        samples.append(str(path))
    # crafted geometry that reads outside its storage (wrapping extents), and deep nesting
    from tests.test_ingest import _hostile_geometry_payloads

    for i, obj in enumerate(_hostile_geometry_payloads()):
        path = tmp_path / f"hostile{i}.pkl"
        path.write_bytes(pickle.dumps(OrderedDict(w=obj), protocol=4))
        samples.append(str(path))
    deep = tmp_path / "deep.pkl"
    deep.write_bytes(b"\x80\x04)" + b"\x85" * 20000 + b".")
    samples.append(str(deep))
    run = subprocess.run([str(exe), *samples], capture_output=True, text=True, timeout=600,
                         env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
    assert run.returncode == 0 and "FUZZ_OK" in run.stdout, run.stderr[-3000:]
