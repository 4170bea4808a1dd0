"""Multi-rank paths: bucket plan, gloo world_size-2 runs of the sharding logic."""

import json
import os
import socket
import subprocess
import sys

import pytest

from plato_amd.distributed import BucketPlan, EntryPlan, client_shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(mode, world, tmp_path, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_worker.py"), mode, str(tmp_path)]
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    proc = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    return [json.load(open(os.path.join(tmp_path, f"rank{r}.json"))) for r in range(world)]


@pytest.mark.parametrize("n_f32,world", [(61706, 1), (61706, 2), (61706, 3), (11183562, 8), (10, 8), (0, 2)])
def test_bucket_plan_covers_arena_once(n_f32, world):
    plan = BucketPlan.make(n_f32, 20, world)
    assert plan.per % 64 == 0
    seen = 0
    for r in range(world):
        lo, hi = plan.f32_range(r)
        assert lo == min(seen, n_f32) and hi - lo <= plan.per
        seen = hi
    assert seen == n_f32
    assert plan.i64_range(0) == (0, 20) and all(plan.i64_range(r) == (0, 0) for r in range(1, world))
    assert sum(plan.bucket_bytes(r, 5) for r in range(world)) == 7 * (n_f32 * 4 + 20 * 8)


@pytest.mark.parametrize("world", [1, 2, 3, 8, 13])
@pytest.mark.parametrize("model", ["lenet5", "resnet18", "tiny"])
def test_entry_plan_partitions_whole_entries(model, world):
    """Entry-aligned shards: contiguous, every entry once, in order, balanced by elements."""
    from plato_amd.arena import ArenaLayout
    from tests import golden_cases as G

    spec = [("a", (3,), "f32"), ("n", (), "i64"), ("b", (5000,), "f32")] if model == "tiny" else G.model_spec(model)
    layout = ArenaLayout.from_shapes(spec)
    plan = EntryPlan.for_layout(layout, world)
    assert plan.world == world
    n = len(layout.entries)
    assert plan.groups[0][0] == 0 and plan.groups[-1][1] == n
    for (a, b), (c, d) in zip(plan.groups, plan.groups[1:]):
        assert a <= b == c <= d
    names = [x for g in range(world) for x in plan.names(layout, g)]
    assert names == layout.keys()
    if n >= world:
        assert all(b > a for a, b in plan.groups)  # every shard holds at least one entry
    sizes = [sum(e.numel for e in layout.entries[a:b]) for a, b in plan.groups]
    biggest = max(e.numel for e in layout.entries)
    # no shard exceeds its share by more than one entry (the cut is at the nearest entry boundary)
    assert max(sizes) <= sum(sizes) / world + biggest


def test_client_shard_partition():
    shards = [client_shard(10, 3, r) for r in range(3)]
    assert sorted(sum(shards, [])) == list(range(10))


def test_gloo_bucket_sharding_bit_exact(tmp_path):
    outs = _run("cpu-bucket", 2, tmp_path)
    assert all(o["bit_exact"] for o in outs)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_piece_sharding_bit_exact(tmp_path, world):
    """The strong-scaling bench's layout: round-robin pieces, one all-gather per piece."""
    outs = _run("cpu-pieces", world, tmp_path)
    assert all(o["bit_exact"] for o in outs)


@pytest.mark.parametrize("world,pieces", [(2, 4), (8, 4)])
def test_piece_layouts_count_their_bytes(world, pieces):
    """bench.py's per-rank piece layouts (entry-less arenas) count every element as model data, so a
    rank's algorithmic bytes sum to the job's (the N > 1 roofline's numerator)."""
    from plato_amd import workloads
    from plato_amd.arena import ArenaLayout
    from plato_amd.distributed import PiecePlan

    full = ArenaLayout.from_shapes(workloads.resnet(18, 10))
    plan = PiecePlan.for_layout(full, world, pieces)
    k = 128
    total = 0
    for r in range(world):
        lays = [ArenaLayout([], plan.piece_elements(r, p), full.n_i64 if (p == 0 and r == 0) else 0)
                for p in range(pieces)]
        got = sum(lay.algorithmic_bytes(k) for lay in lays)
        assert got > 0
        total += got
    assert total == full.algorithmic_bytes(k)


@pytest.mark.parametrize("n_f32,world,pieces", [(61706, 2, 4), (11183562, 8, 4), (100, 8, 3), (0, 2, 2)])
def test_piece_plan_covers_arena_once(n_f32, world, pieces):
    from plato_amd.distributed import PiecePlan

    plan = PiecePlan.make(n_f32, 20, world, pieces)
    L = plan.length
    assert L % 64 == 0
    covered = []
    for p in range(pieces):
        for r in range(world):
            lo, hi = plan.piece_range(r, p)
            assert hi - lo <= L
            # in the assembled arena the piece sits where the all-gather of group p puts rank r
            if hi > lo:
                assert plan.gather_offset(p) + r * L == lo
            covered.append((lo, hi))
    covered.sort()
    pos = 0
    for lo, hi in covered:
        if hi > lo:
            assert lo == pos
            pos = hi
    assert pos == n_f32


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_gloo_bench_strong_job_parity(tmp_path, world):
    """bench.py's N > 1 job is ONE FedAvg job: each rank's pieces are slices of the same global inputs, and
    the parity fields the bench reports (compare_windows, ranks_agree) say bit-exact against the whole job."""
    outs = _run("cpu-bench-strong", world, tmp_path)
    assert all(o["ranks_agree"] for o in outs)
    r0 = outs[0]
    assert r0["parity"] == "bit-exact vs 1-GPU kernel" and r0["mismatched_elements"] == 0, r0
    assert r0["whole_job_bit_exact"] and r0["windows"] >= 3  # the windowed check covers the model in pieces


def test_gloo_bench_strong_job_parity_catches_a_flipped_bit(tmp_path):
    outs = _run("cpu-bench-strong-corrupt", 2, tmp_path)
    r0 = outs[0]
    assert r0["parity"] == "MISMATCH vs 1-GPU kernel" and r0["mismatched_elements"] == 1, r0
    assert not r0["whole_job_bit_exact"]


def test_gloo_client_sharding_normwise(tmp_path):
    outs = _run("cpu-client", 2, tmp_path)
    for o in outs:
        assert o["normwise"] <= 1e-6, o


@pytest.mark.gpu
def test_two_ranks_bucket_aggregator_on_gpu(tmp_path):
    outs = _run("gpu-bucket", 2, tmp_path)
    for o in outs:
        assert o["f32_match"] and o["i64_match"], o


@pytest.mark.gpu
def test_rccl_collectives_one_rank_per_gpu(tmp_path):
    """The driver's multi-GPU runs use RCCL; on a one-GPU box this is world size 1."""
    import torch

    outs = _run("gpu-rccl", min(torch.cuda.device_count(), 8), tmp_path)
    for o in outs:
        assert o["f32_match"] and o["i64_match"] and o["reduce_scatter_on_gpu"], o
        assert o["normwise"] <= 1e-6, o


def _bench_lines(args, env_extra, timeout):
    env = dict(os.environ, OMP_NUM_THREADS="2", PLATO_BENCH_BACKEND="gloo", **env_extra)
    env.pop("WORLD_SIZE", None)
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=timeout)
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    lines = [ln for ln in proc.stdout.splitlines() if ln.strip()]
    return lines, proc.stderr


def test_bench_self_launches_its_ranks():
    """``python bench.py --gpus 2`` from a plain invocation spawns torch.distributed.run itself (before any GPU
    call) and forwards rank 0's single JSON line: the launcher plumbing, with gloo and no GPU work."""
    lines, err = _bench_lines(["--gpus", "2", "--probe-launch"], {}, 300)
    assert len(lines) == 1, (lines, err[-2000:])
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["requested"] == 2 and out["rank_sum"] == 1.0
    assert "launching 2 ranks" in err


def _bench_fails(args, limit):
    import time

    env = dict(os.environ, OMP_NUM_THREADS="2", PLATO_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    t0 = time.monotonic()
    proc = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=limit)
    return proc, time.monotonic() - t0


def test_bench_collective_timeout_names_rank_and_collective():
    """A rank that never joins: the waiting rank's collective fails after --dist-timeout, naming itself and the
    collective, and ``python bench.py --gpus 2`` exits non-zero well before any outer limit."""
    proc, took = _bench_fails(["--gpus", "2", "--probe-launch", "--probe-stall-rank", "1", "--dist-timeout", "8",
                               "--launch-timeout", "240"], 280)
    assert proc.returncode not in (0, 124), proc.stderr[-3000:]
    assert "rank 0: collective 'all_reduce(rank_sum)' failed" in proc.stderr, proc.stderr[-3000:]
    assert took < 200
    assert not [ln for ln in proc.stdout.splitlines() if ln.strip()]  # no result line


def test_bench_launch_timeout_kills_the_tree_and_reports_phases():
    """The self-launcher's wall-clock limit: the rank tree is killed, each rank's last phase is printed
    (the stalled rank and the collective the other one waits in), exit code 124."""
    proc, took = _bench_fails(["--gpus", "2", "--probe-launch", "--probe-stall-rank", "1", "--dist-timeout", "600",
                               "--launch-timeout", "45"], 200)
    assert proc.returncode == 124, proc.stderr[-3000:]
    err = proc.stderr
    assert "TIMEOUT" in err and "rank 1: stalling before all_reduce" in err, err[-3000:]
    assert "rank 0: all_reduce(rank_sum)" in err, err[-3000:]
    assert took < 120


@pytest.mark.gpu
def test_bench_self_launch_two_ranks_on_gpu():
    """The N > 1 bench from a plain ``python bench.py --gpus 2`` on the one-GPU box (gloo rehearsal: the ranks share
    the GPU): one parsed line with n_gpus == 2 and the per-rank algorithmic bytes counted."""
    lines, err = _bench_lines(["--gpus", "2", "--steps", "3", "--warmup", "1"], {}, 600)
    assert len(lines) == 1, (lines, err[-2000:])
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0
    cfg = out["config"]
    assert cfg["algorithmic_bytes_per_step_per_gpu"] > 0 and cfg["pieces_per_rank"] >= 1
    assert out["roofline"]["frac"] > 0
    # one FedAvg job: the gathered model is the one-GPU kernel's on the same inputs, bit for bit
    assert out["parity"] == "bit-exact vs 1-GPU kernel", out.get("parity_detail")
    assert out["parity_detail"]["ranks_hold_identical_models"]
    assert out["parity_detail"]["elements_checked"] == 11183562 + 20
    # the server's in-process multi-GPU path (MultiDeviceEngine over 2 devices, repeated on one GPU)
    ed = out["engine_devices"]
    assert ed["status"] == "ok" and ed["engine_devices"] == 2, ed
    assert ed["parity"].startswith("bit-exact vs 1-GPU engine"), ed
    assert ed["parity_detail"]["gathered_copies_checked"] == 2
