"""Worker for the multi-process tests (launched by torch.distributed.run).

Modes:
  cpu-bench-strong
               gloo, CPU: bench.py's N > 1 job (pieces filled as slices of one global
               job, PieceExchange send/gather/assemble) with the oracle as the
               per-piece compute; bench's parity fields must say bit-exact
               (-corrupt: one flipped bit on the last rank must say MISMATCH).
  cpu-bucket   gloo, CPU: bucket sharding with the oracle as the per-bucket
               compute (the sequential-K kernel is elementwise, so each
               bucket's result is the oracle on that slice); gathered model
               must equal the single-process oracle bit for bit.
  cpu-pieces   gloo, CPU: bucket sharding in round-robin pieces (PiecePlan, the
               strong-scaling bench's layout), one all-gather per piece; the
               assembled model must equal the single-process oracle bit for bit.
  cpu-client   gloo, CPU: client sharding + reduce_scatter + all_gather;
               max|new - new_seq| / max|new_seq| <= 1e-6.
  gpu-bucket   gloo, every rank on cuda:0: BucketAggregator (HIP kernel) per
               rank, gathered model must equal the reference fixture digest.
  gpu-rccl     nccl (= RCCL), one rank per GPU: gpu-bucket's all-gather on
               device tensors, and the client-sharded reduce-scatter of HIP
               deltas-kernel partials (normwise <= 1e-6).
"""

import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import fedavg_oracle as ref  # noqa: E402
from oracle import synth  # noqa: E402
from plato_amd import workloads  # noqa: E402
from plato_amd.arena import ArenaLayout  # noqa: E402
from plato_amd.distributed import (BucketPlan, PiecePlan, client_shard, gather_buckets,  # noqa: E402
                                   reduce_scatter_partials)


def inputs(spec, k, seed):
    layout = ArenaLayout.from_shapes(spec)
    bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, seed)
    xs = [synth.client_arena(bf, bi, seed, c) for c in range(k)]
    return layout, bf, bi, [x[0] for x in xs], [x[1] for x in xs]


def cpu_pieces(rank, world, out):
    layout, bf, bi, xs_f, xs_i = inputs(workloads.lenet5(), 6, 23)
    w = ref.fedavg_weights(synth.num_samples(6, 23))
    plan = PiecePlan.make(layout.n_f32, layout.n_i64, world, 3)
    L = plan.length
    local = torch.zeros(plan.pieces * L, dtype=torch.float32)
    for p in range(plan.pieces):
        lo, hi = plan.piece_range(rank, p)
        got, _ = ref.fedavg_numpy(bf[lo:hi], bi[:0], [x[lo:hi] for x in xs_f], [x[:0] for x in xs_i], w)
        local[p * L: p * L + (hi - lo)] = torch.from_numpy(got)
    full = torch.empty(world * plan.pieces * L, dtype=torch.float32)
    for p in range(plan.pieces):
        plan.gather_piece(p, local[p * L:], full)
    exp, _ = ref.fedavg_numpy(bf, bi, xs_f, xs_i, w)
    out["bit_exact"] = full[: layout.n_f32].numpy().tobytes() == exp.tobytes()
    out["pieces"], out["length"] = plan.pieces, L


def cpu_bench_strong(rank, world, out, corrupt=False):
    """bench.py's N > 1 job and its parity fields, with the oracle in the kernel's place.

    Every rank generates ITS pieces as slices of the one global job (the counter generator from the
    pieces' global offsets, as plato_agg_fill_synth_*_at does on the GPU), lays its results out in
    the send buffer of PieceExchange, all-gathers piece by piece, and reads the model back with
    PieceExchange.assemble; then bench.ranks_agree and, on rank 0, bench.compare_windows against the
    whole job regenerated window by window.  ``corrupt``: rank world-1 flips one bit of its last piece.
    """
    import bench

    layout = ArenaLayout.from_shapes(workloads.lenet5())
    k, seed, pieces = 5, 31, 3
    w = ref.fedavg_weights(synth.num_samples(k, seed))
    plan = PiecePlan.for_layout(layout, world, pieces)
    xchg = plan.exchange(layout.n_i64)

    def job_slice(lo, n, ni):
        b = synth.synth_f32(n, seed, 0, synth.BASE_SCALE, start=lo)
        xs = [synth.synth_f32(n, seed, c + 1, synth.CLIENT_SCALE, add=b, start=lo) for c in range(k)]
        bi = synth.synth_i64(ni, seed, 0, synth.I64_BASE_MOD)
        xi = [synth.synth_i64(ni, seed, c + 1, synth.I64_CLIENT_MOD, add=bi) for c in range(k)]
        f, i = ref.fedavg_numpy(b, bi, xs, xi, w)
        return torch.from_numpy(f), torch.from_numpy(i)

    send = torch.zeros(xchg.send_numel, dtype=torch.float32)
    for p in range(pieces):
        lo, hi = plan.piece_range(rank, p)
        ni = layout.n_i64 if (rank == 0 and p == 0) else 0
        f, i = job_slice(lo, hi - lo, ni)
        send[xchg.soff[p]: xchg.soff[p] + (hi - lo)] = f
        if ni:
            send[xchg.int64_offset(): xchg.int64_offset() + ni] = i
    if corrupt and rank == world - 1:
        lo, hi = plan.piece_range(rank, pieces - 1)
        if hi > lo:
            send[xchg.soff[pieces - 1]: xchg.soff[pieces - 1] + 1].view(torch.int32).bitwise_xor_(1)
    gathered = torch.empty(xchg.gathered_numel, dtype=torch.float32)
    for p in range(pieces):
        dist.all_gather_into_tensor(xchg.gather_slice(gathered, p), xchg.send_slice(send, p))
    got_f, got_i = xchg.assemble(gathered)
    out["ranks_agree"] = bench.ranks_agree(bench.bits_digest(got_f, got_i), world)
    if rank == 0:
        res = bench.compare_windows(layout.n_f32, layout.n_i64, 20000, job_slice, got_f, got_i)
        out.update(res)
        exp_f, exp_i = job_slice(0, layout.n_f32, layout.n_i64)
        out["whole_job_bit_exact"] = (got_f.numpy().tobytes() == exp_f.numpy().tobytes()
                                      and got_i.numpy().tobytes() == exp_i.numpy().tobytes())


def cpu_bucket(rank, world, out):
    layout, bf, bi, xs_f, xs_i = inputs(workloads.lenet5(), 6, 21)
    ns = synth.num_samples(6, 21)
    w = ref.fedavg_weights(ns)
    plan = BucketPlan.for_layout(layout, world)
    lo, hi = plan.f32_range(rank)
    bucket = np.zeros(plan.per, dtype=np.float32)
    got_f, _ = ref.fedavg_numpy(bf[lo:hi], bi[:0], [x[lo:hi] for x in xs_f], [x[:0] for x in xs_i], w)
    bucket[: hi - lo] = got_f
    full, _ = gather_buckets(plan, torch.from_numpy(bucket), None)
    exp_f, _ = ref.fedavg_numpy(bf, bi, xs_f, xs_i, w)
    out["bit_exact"] = full.numpy().tobytes() == exp_f.tobytes()


def cpu_client(rank, world, out):
    layout, bf, bi, xs_f, xs_i = inputs(workloads.resnet(18), 8, 22)
    ns = synth.num_samples(8, 22)
    w = ref.fedavg_weights(ns)
    plan = BucketPlan.for_layout(layout, world)
    mine = client_shard(8, world, rank)
    deltas = [np.subtract(xs_f[c], bf, dtype=np.float32) for c in mine]
    partial, _ = ref.deltas_numpy(deltas, [xs_i[c][:0] for c in mine], [w[c] for c in mine])
    bucket_sum = reduce_scatter_partials(plan, torch.from_numpy(partial))
    lo, hi = plan.f32_range(rank)
    bucket = torch.zeros(plan.per)
    bucket[: hi - lo] = torch.from_numpy(bf[lo:hi]) + bucket_sum[: hi - lo]
    full, _ = gather_buckets(plan, bucket, torch.from_numpy(bi.astype(np.float32)))
    exp_f, _ = ref.fedavg_numpy(bf, bi, xs_f, xs_i, w)
    # tolerance mode: normwise relative error of the new weights (north star:
    # "within 1e-6 relative on fp32 sums"); per element it is not bit-exact.
    diff = np.abs(full.numpy().astype(np.float64) - exp_f)
    out["normwise"] = float(np.max(diff) / np.max(np.abs(exp_f)))
    out["bit_exact"] = full.numpy().tobytes() == exp_f.tobytes()


def gpu_bucket(rank, world, out):
    from plato_amd.distributed import BucketAggregator
    from tests import golden_cases as G

    case = next(c for c in G.load_cases() if c["recipe"]["name"] == "resnet18_k16")
    recipe, exp = case["recipe"], case["expected"]
    layout, bf, bi, xs_f, xs_i = inputs(workloads.resnet(18), recipe["k"], recipe["seed"])
    agg = BucketAggregator(layout, recipe["k"], world, rank, device="cuda:0")
    agg.stage_baseline(torch.from_numpy(bf), torch.from_numpy(bi))
    for c in range(recipe["k"]):
        agg.stage_client(c, torch.from_numpy(xs_f[c]), torch.from_numpy(xs_i[c]))
    from plato_amd import weights as W

    agg.launch(W.fedavg(recipe["num_samples"]))
    torch.cuda.synchronize()
    full, ints = agg.gather()
    out["f32_match"] = G.sha(G.canon(full.cpu().numpy())) == exp["updated_f32_sha256"]
    out["i64_match"] = G.sha(G.canon(ints.cpu().numpy())) == exp["updated_i64f_sha256"]


def gpu_rccl(rank, world, out):
    """RCCL (backend "nccl") on GPU tensors: the bucket all-gather + int64 broadcast
    (gpu_bucket) and the client-sharded reduce-scatter of HIP-kernel partials."""
    gpu_bucket(rank, world, out)
    from plato_amd import weights as W
    from plato_amd.engine import FedAvgEngine

    layout, bf, bi, xs_f, xs_i = inputs(workloads.resnet(18), 8, 22)
    w = W.fedavg(synth.num_samples(8, 22))
    plan = BucketPlan.for_layout(layout, world)
    mine = client_shard(8, world, rank)
    eng = FedAvgEngine(f"cuda:{rank % torch.cuda.device_count()}")
    deltas = [layout.unpack(torch.from_numpy(np.subtract(xs_f[c], bf, dtype=np.float32)),
                            torch.from_numpy(xs_i[c] - bi)) for c in mine]
    part = eng.aggregate_deltas(deltas, [w[c] for c in mine])   # HIP deltas-mode kernel
    flat = torch.cat([part[e.name].reshape(-1) for e in layout.entries if e.region == "f32"]).to(eng.device)
    bucket_sum = reduce_scatter_partials(plan, flat)             # RCCL reduce-scatter
    out["reduce_scatter_on_gpu"] = bucket_sum.is_cuda
    lo, hi = plan.f32_range(rank)
    bucket = torch.zeros(plan.per, device=eng.device)
    bucket[: hi - lo] = torch.from_numpy(bf[lo:hi]).to(eng.device) + bucket_sum[: hi - lo]
    full, _ = gather_buckets(plan, bucket, torch.from_numpy(bi.astype(np.float32)).to(eng.device))
    exp_f, _ = ref.fedavg_numpy(bf, bi, xs_f, xs_i, w)
    diff = np.abs(full.cpu().numpy().astype(np.float64) - exp_f)
    out["normwise"] = float(np.max(diff) / np.max(np.abs(exp_f)))


def main():
    mode, out_dir = sys.argv[1], sys.argv[2]
    if mode == "gpu-rccl":  # one process per GPU over RCCL
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    out = {"rank": rank, "world": world}
    {"cpu-bench-strong": cpu_bench_strong,
     "cpu-bench-strong-corrupt": lambda r, wd, o: cpu_bench_strong(r, wd, o, corrupt=True),
     "cpu-bucket": cpu_bucket, "cpu-pieces": cpu_pieces, "cpu-client": cpu_client, "gpu-bucket": gpu_bucket,
     "gpu-rccl": gpu_rccl}[mode](rank, world, out)
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
