"""Hook plumbing on the CPU (no GPU): where the hooks run and what they release.

The engine is a test double; the device numerics of the same hooks are covered
by tests/test_server_loop_gpu.py and tests/test_golden_gpu.py.
"""

import asyncio
import threading
import types

import pytest

from plato_amd.servers.fedavg import FusedAggregationMixin


class _Round:
    def __init__(self, log):
        self.log = log
        self.timings = {}

    def put_baseline(self, b):
        self.log.append(("baseline", threading.current_thread().name))

    def adopt(self, slot, p):
        return False

    def put_client(self, slot, p):
        self.log.append(("client", threading.current_thread().name))

    def launch(self, weights, scales=None):
        self.log.append(("launch", weights))

    def wait(self):
        self.log.append(("wait", threading.current_thread().name))

    def result(self):
        return {"w": 1}

    def algorithmic_bytes(self):
        return 0


class _Engine:
    def __init__(self):
        self.log = []
        self.released = 0

    def begin(self, template, k, codec="native"):
        return _Round(self.log)

    def release_arrivals(self):
        self.released += 1


def _server(weights_fn):
    class Server(FusedAggregationMixin):
        def aggregation_weights(self, updates):
            return weights_fn(self, updates)

    s = Server()
    s._plato_amd_engine = _Engine()
    return s


UPDATES = [types.SimpleNamespace(report=types.SimpleNamespace(num_samples=n)) for n in (1, 3)]
PAYLOADS = [{"w": 0}, {"w": 1}]


def test_weights_and_staging_run_off_the_event_loop():
    seen = {}

    def weights(server, updates):
        seen["thread"] = threading.current_thread().name
        seen["round"] = server._plato_amd_round is not None
        return [0.25, 0.75], None

    s = _server(weights)
    out = asyncio.run(s.aggregate_weights(UPDATES, {"w": 0}, PAYLOADS))
    assert out == {"w": 1}
    assert seen["thread"].startswith("plato-amd-stage") and seen["round"]
    assert all(t.startswith("plato-amd-stage") for kind, t in s._plato_amd_engine.log
               if kind in ("baseline", "client", "wait"))
    assert s._plato_amd_round is None
    assert s._plato_amd_engine.released == 1


@pytest.mark.parametrize("where", ["weights", "launch"])
def test_arrivals_are_released_when_the_round_fails(where):
    class Boom(RuntimeError):
        pass

    def weights(server, updates):
        if where == "weights":
            raise Boom("no lr")
        return [0.5, 0.5], None

    s = _server(weights)
    if where == "launch":
        def bad_launch(self, weights, scales=None):
            raise Boom("launch failed")

        _Round.launch, saved = bad_launch, _Round.launch
    try:
        with pytest.raises(Boom):
            asyncio.run(s.aggregate_weights(UPDATES, {"w": 0}, PAYLOADS))
    finally:
        if where == "launch":
            _Round.launch = saved
    assert s._plato_amd_engine.released == 1
    assert s._plato_amd_round is None
