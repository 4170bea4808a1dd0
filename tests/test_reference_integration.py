"""The product's aggregate_weights hook inside the real reference server (CPU wiring test).

Runs only where TL-System/plato is present (this build container); see
tests/ref_integration.py.  Numerics of the same hook on the GPU are covered by
tests/test_golden_gpu.py::test_server_hooks_match_reference.
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE = os.environ.get("PLATO_REFERENCE", "/root/reference")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REFERENCE, "plato")), reason="reference not present")
def test_hook_dispatch_in_reference_process_reports(tmp_path):
    out = tmp_path / "calls.json"
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "ref_integration.py"), str(out)],
                          capture_output=True, text=True, timeout=600,
                          env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4"))
    assert proc.returncode == 0, proc.stderr[-3000:]
    calls = json.loads(out.read_text())
    assert calls["hook"] == 1                 # _process_reports took the aggregate_weights branch
    assert calls["load"] == 1                 # ... and loaded what the hook returned
    assert calls["load_dtypes"] == ["torch.float32"]  # update_weights' dtypes (int keys as fp32)
    assert calls["cb_received"] == 1 and calls["cb_aggregated"] == 1
    assert calls["model_matches_reference_chain"]
    assert calls["total_samples"]
    for mode in ("socket", "simulated"):  # WireIngestMixin in the reference's arrival paths
        ing = calls["ingest"][mode]
        assert ing["payload_matches"] and ing["arena_backed"], mode
        got, exp = ing["comm_overhead_bytes"]
        assert abs(got - exp) <= 2 * 2 * 122 + 64, mode  # storage-key digits only (see test_ingest.py)
    # the other callers of the hooks, in the reference's own code paths:
    # fedavg_cs._process_reports, RLServer.aggregate_deltas (mixin), HE _fedavg_hybrid (mixin),
    # and _process_clients' async simulated-wall-time ordering -> the reference's fixtures
    assert calls["more"] == {"cross_silo": True, "rl": True, "he": True, "async_order": True, "async_model": True}
