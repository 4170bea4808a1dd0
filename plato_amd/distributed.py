"""Multi-GPU aggregation on one node: one process per GPU over RCCL (xGMI).

Two modes:

* **Parameter-bucket sharding (default, bit-exact).**  The flat fp32 arena
  is cut into ``world`` contiguous, 256-byte-aligned buckets; rank r receives
  bucket r of every client update and runs the same sequential-K kernel on it.
  Every output element still sums its clients in ``self.updates`` order, so the
  result is bit-identical to the one-GPU / CPU-reference result.  The data path
  needs no collective; the new model is assembled only when it must live on
  every GPU (``gather_buckets``: one RCCL all-gather of the P·4-byte result).
  The int64 counters (20 scalars for ResNet-18) ride with rank 0's bucket.

* **Client sharding + RCCL reduce-scatter (tolerance mode).**  When payloads
  land client-sharded (client j on GPU j mod N), each rank forms the weighted
  partial sum of its clients' deltas, ``reduce_scatter`` sums the partials by
  bucket and ``all_gather`` assembles the model.  The K-sum is reordered, so it
  is NOT bit-exact (per-element relative error up to ~1e-3,
  normwise ~5e-7); tests gate it on ``max|Δ| / max|new| <= 1e-6``.

Collectives go through ``torch.distributed`` (backend "nccl" = RCCL on ROCm;
"gloo" for the CPU tests); the per-bucket arithmetic is the HIP kernel.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence

import numpy as np
import torch
import torch.distributed as dist

from .arena import ROW_ALIGN, ArenaLayout


@dataclass(frozen=True)
class BucketPlan:
    """Contiguous fp32 buckets, one per rank; int64 entries on rank 0."""

    n_f32: int
    n_i64: int
    world: int
    per: int  # padded bucket length (elements), a multiple of ROW_ALIGN

    @classmethod
    def make(cls, n_f32: int, n_i64: int, world: int) -> "BucketPlan":
        if world < 1:
            raise ValueError("world must be >= 1")
        per = -(-max(n_f32, 1) // world)
        per = -(-per // ROW_ALIGN) * ROW_ALIGN
        return cls(n_f32, n_i64, world, per)

    @classmethod
    def for_layout(cls, layout: ArenaLayout, world: int) -> "BucketPlan":
        return cls.make(layout.n_f32, layout.n_i64, world)

    def f32_range(self, rank: int) -> tuple[int, int]:
        lo = min(rank * self.per, self.n_f32)
        hi = min(lo + self.per, self.n_f32)
        return lo, hi

    def i64_range(self, rank: int) -> tuple[int, int]:
        return (0, self.n_i64) if rank == 0 else (0, 0)

    def bucket_bytes(self, rank: int, k: int) -> int:
        """Algorithmic HBM bytes of rank's launch: (K+2) x its bucket."""
        lo, hi = self.f32_range(rank)
        a, b = self.i64_range(rank)
        return (k + 2) * ((hi - lo) * 4 + (b - a) * 8)


@dataclass(frozen=True)
class EntryPlan:
    """Entry-aligned sharding: shard g holds whole entries ``[groups[g][0], groups[g][1])`` (layout order).

    The per-entry reductions of the variant servers — FedAtt's per-(entry,
    client) norms and attentive sum (fedatt_algorithm.py:23-69), Polaris'
    per-layer squared sums (polaris_server.py:68-100), QSGD's per-entry scales
    (model_dequantize_qsgd.py:34-60) — read one entry at a time, so cutting the
    model between entries keeps every value on one GPU and bit-identical to
    the one-GPU result.  Groups are contiguous and chosen to minimise the
    largest group's element count (fp32 and int64 elements alike; a small
    dynamic program over the entry boundaries); every shard holds at least one
    entry unless there are more shards than entries.
    """

    groups: tuple  # ((lo, hi), ...) entry index ranges, one per shard

    @classmethod
    def make(cls, sizes: Sequence[int], world: int) -> "EntryPlan":
        if world < 1:
            raise ValueError("world must be >= 1")
        n = len(sizes)
        prefix = np.concatenate([[0], np.cumsum(np.asarray(sizes, dtype=np.float64))])
        empty_ok = n < world  # more shards than entries: some stay empty
        # dp[j]: the smallest possible largest shard when the first j entries fill g shards
        inf = float("inf")
        dp = np.full(n + 1, inf)
        dp[0] = 0.0
        back = []
        for g in range(1, world + 1):
            new = np.full(n + 1, inf)
            arg = np.zeros(n + 1, dtype=np.int64)
            for j in range(n + 1):
                hi = j if empty_ok else j - 1  # the last shard takes entries [i, j)
                if hi < 0:
                    continue
                cost = np.maximum(dp[: hi + 1], prefix[j] - prefix[: hi + 1])
                i = int(np.argmin(cost))
                new[j], arg[j] = cost[i], i
            back.append(arg)
            dp = new
        cuts = [n]
        for g in range(world - 1, 0, -1):
            cuts.append(int(back[g][cuts[-1]]))
        cuts.append(0)
        cuts.reverse()
        return cls(tuple((cuts[r], cuts[r + 1]) for r in range(world)))

    @classmethod
    def for_layout(cls, layout: ArenaLayout, world: int) -> "EntryPlan":
        return cls.make([e.numel for e in layout.entries], world)

    @property
    def world(self) -> int:
        return len(self.groups)

    def names(self, layout: ArenaLayout, shard: int) -> list[str]:
        lo, hi = self.groups[shard]
        return [e.name for e in layout.entries[lo:hi]]


@dataclass(frozen=True)
class PiecePlan:
    """Bucket sharding in round-robin pieces, for an assembly that overlaps the kernels.

    The arena is cut into ``world * pieces`` equal 256-byte-aligned pieces
    (:class:`BucketPlan` over that many virtual buckets); piece ``j`` belongs to
    rank ``j % world``.  Rank r keeps its pieces back to back in a local arena
    (piece p at ``p * length``).  The p-th pieces of all ranks are contiguous
    in the model, so one all-gather per p lands them in place, and the
    all-gather of piece p can run while the kernels of pieces p+1.. run.  The
    int64 entries ride with piece 0 of rank 0.
    """

    buckets: BucketPlan
    world: int
    pieces: int

    @classmethod
    def make(cls, n_f32: int, n_i64: int, world: int, pieces: int) -> "PiecePlan":
        if pieces < 1:
            raise ValueError("pieces must be >= 1")
        return cls(BucketPlan.make(n_f32, n_i64, world * pieces), world, pieces)

    @classmethod
    def for_layout(cls, layout: ArenaLayout, world: int, pieces: int) -> "PiecePlan":
        return cls.make(layout.n_f32, layout.n_i64, world, pieces)

    @property
    def length(self) -> int:
        """Padded piece length (elements)."""
        return self.buckets.per

    def piece_range(self, rank: int, p: int) -> tuple[int, int]:
        """Model element range of rank's piece p (may be short or empty at the end)."""
        return self.buckets.f32_range(p * self.world + rank)

    def piece_elements(self, rank: int, p: int) -> int:
        lo, hi = self.piece_range(rank, p)
        return hi - lo

    def gather_offset(self, p: int) -> int:
        """Where the all-gather of the p-th pieces starts in the assembled arena."""
        return p * self.world * self.length

    def exchange(self, n_i64: int) -> "PieceExchange":
        """The send / gather buffer layout of a rank whose piece 0 carries the int64 results (bench.py, N > 1)."""
        return PieceExchange.make(self, n_i64)

    def gather_piece(self, p: int, piece: torch.Tensor, full: torch.Tensor, group=None, async_op: bool = False):
        """All-gather rank pieces p (``length`` elements each) into ``full`` (``world*pieces*length``)."""
        n = self.world * self.length
        dst = full[self.gather_offset(p): self.gather_offset(p) + n]
        return dist.all_gather_into_tensor(dst, piece[: self.length], group=group, async_op=async_op)


@dataclass(frozen=True)
class PieceExchange:
    """Where a rank's pieces sit in its send buffer and in the all-gathered buffer.

    Send buffer of every rank: ``[piece 0 | int64 results, ipad floats | piece 1 | ... ]`` (the
    int64 results are meaningful on rank 0 only).  The all-gather of the p-th pieces of all ranks
    (``slen[p]`` floats each) lands at ``goff[p]``, ranks in model order, so the gathered buffer
    holds the model once the ``pieces`` all-gathers are done; :meth:`assemble` reads it back in
    model order (fp32 arena, fp32 values of the int64 entries).
    """

    plan: PiecePlan
    n_i64: int
    ipad: int
    soff: tuple
    slen: tuple
    goff: tuple

    @classmethod
    def make(cls, plan: PiecePlan, n_i64: int) -> "PieceExchange":
        L, world, pieces = plan.length, plan.world, plan.pieces
        ipad = -(-max(n_i64, 1) // ROW_ALIGN) * ROW_ALIGN
        soff = (0,) + tuple(L + ipad + (p - 1) * L for p in range(1, pieces))
        slen = (L + ipad,) + (L,) * (pieces - 1)
        goff = (0,) + tuple(world * (L + ipad) + (p - 1) * world * L for p in range(1, pieces))
        return cls(plan, n_i64, ipad, soff, slen, goff)

    @property
    def send_numel(self) -> int:
        return self.plan.pieces * self.plan.length + self.ipad

    @property
    def gathered_numel(self) -> int:
        return self.plan.world * self.send_numel

    def int64_offset(self) -> int:
        """Offset of the int64 results in a send buffer (and in the gathered one: rank 0 comes first)."""
        return self.plan.length

    def send_slice(self, send: torch.Tensor, p: int) -> torch.Tensor:
        return send[self.soff[p]: self.soff[p] + self.slen[p]]

    def gather_slice(self, gathered: torch.Tensor, p: int) -> torch.Tensor:
        return gathered[self.goff[p]: self.goff[p] + self.plan.world * self.slen[p]]

    def assemble(self, gathered: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """(fp32 arena [n_f32], int64-entry results [n_i64]) of the model, from the gathered buffer."""
        plan = self.plan
        n_f32 = plan.buckets.n_f32
        full = torch.empty(n_f32, dtype=gathered.dtype, device=gathered.device)
        for p in range(plan.pieces):
            for r in range(plan.world):
                lo, hi = plan.piece_range(r, p)
                if hi > lo:
                    src = self.goff[p] + r * self.slen[p]
                    full[lo:hi] = gathered[src: src + hi - lo]
        i0 = self.int64_offset()
        return full, gathered[i0: i0 + self.n_i64].clone()


def gather_buckets(plan: BucketPlan, bucket_f32: torch.Tensor, bucket_i64f: torch.Tensor | None,
                   group=None) -> tuple[torch.Tensor, torch.Tensor]:
    """Assemble the full result on every rank: all-gather of equal padded buckets.

    ``bucket_f32`` has ``plan.per`` elements (this rank's range, zero padded);
    ``bucket_i64f`` holds the int64 entries' fp32 results on rank 0 (ignored
    elsewhere).  Returns (full fp32 arena [n_f32], int64-entry results [n_i64]).
    """
    if bucket_f32.numel() != plan.per:
        raise ValueError(f"bucket has {bucket_f32.numel()} elements, plan says {plan.per}")
    dev = bucket_f32.device
    # gloo (CPU tests, or several ranks sharing one GPU) moves host tensors.
    host = dist.get_backend(group) == "gloo"
    src = bucket_f32.contiguous().cpu() if host else bucket_f32.contiguous()
    full = torch.empty(plan.per * plan.world, dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(full, src, group=group)
    ints = torch.empty(plan.n_i64, dtype=torch.float32, device=src.device)
    if plan.n_i64:
        if dist.get_rank(group) == 0:
            ints.copy_(bucket_i64f[: plan.n_i64])
        dist.broadcast(ints, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return full[: plan.n_f32].to(dev), ints.to(dev)


def reduce_scatter_partials(plan: BucketPlan, partial_f32: torch.Tensor, group=None) -> torch.Tensor:
    """Client-sharded mode: sum every rank's full-arena partial, keep this rank's bucket."""
    dev = partial_f32.device
    host = dist.get_backend(group) == "gloo"
    padded = torch.zeros(plan.per * plan.world, dtype=partial_f32.dtype,
                         device="cpu" if host else dev)
    padded[: plan.n_f32].copy_(partial_f32[: plan.n_f32])
    out = torch.empty(plan.per, dtype=partial_f32.dtype, device=padded.device)
    dist.reduce_scatter_tensor(out, padded, op=dist.ReduceOp.SUM, group=group)
    return out.to(dev)


def client_shard(k: int, world: int, rank: int) -> list[int]:
    """Clients owned by ``rank`` in client-sharded mode (client j on rank j mod world)."""
    return list(range(rank, k, world))


class BucketAggregator:
    """This rank's share of a bucket-sharded FedAvg, on its GPU (bit-exact).

    Holds its bucket of the baseline and of up to ``capacity`` client arenas in
    HBM.  ``stage_client`` copies only this rank's slice of a full host arena,
    so with N GPUs each PCIe link carries 1/N of every payload.
    """

    def __init__(self, layout: ArenaLayout, capacity: int, world: int, rank: int, device=None,
                 engine=None):
        from .engine import FedAvgEngine

        self.layout = layout
        self.plan = BucketPlan.for_layout(layout, world)
        self.rank = rank
        self.engine = engine or FedAvgEngine(device)
        dev = self.engine.device
        self.lo, self.hi = self.plan.f32_range(rank)
        self.ilo, self.ihi = self.plan.i64_range(rank)
        self.n = self.hi - self.lo
        self.ni = self.ihi - self.ilo
        per = self.plan.per
        self.bucket_layout = ArenaLayout([], self.n, self.ni)
        self.clients_f32 = torch.empty((capacity, per), dtype=torch.float32, device=dev)
        self.clients_i64 = torch.empty((capacity, max(self.ni, 1)), dtype=torch.int64, device=dev)
        self.base_f32 = torch.zeros(per, dtype=torch.float32, device=dev)
        self.base_i64 = torch.zeros(max(self.ni, 1), dtype=torch.int64, device=dev)
        self.out_f32 = torch.zeros(per, dtype=torch.float32, device=dev)
        self.out_i64f = torch.zeros(max(self.ni, 1), dtype=torch.float32, device=dev)
        self.capacity = capacity

    # host arenas are flat fp32 [n_f32] / int64 [n_i64] tensors (pinned for async copies)
    def stage_baseline(self, flat_f32: torch.Tensor, flat_i64: torch.Tensor | None) -> None:
        self.base_f32[: self.n].copy_(flat_f32[self.lo : self.hi], non_blocking=True)
        if self.ni:
            self.base_i64[: self.ni].copy_(flat_i64[self.ilo : self.ihi], non_blocking=True)

    def stage_client(self, slot: int, flat_f32: torch.Tensor, flat_i64: torch.Tensor | None) -> None:
        self.clients_f32[slot, : self.n].copy_(flat_f32[self.lo : self.hi], non_blocking=True)
        if self.ni:
            self.clients_i64[slot, : self.ni].copy_(flat_i64[self.ilo : self.ihi], non_blocking=True)

    def launch(self, weights: Sequence[float], scales: Sequence[float] | None = None,
               order: Sequence[int] | None = None, stream=None) -> None:
        from .engine import fp32_weights

        eng = self.engine
        order = list(range(len(weights))) if order is None else list(order)
        k = len(order)
        rows = torch.tensor(order, dtype=torch.int64)
        pf = (self.clients_f32.data_ptr() + rows * self.clients_f32.stride(0) * 4).to(eng.device)
        pi = (self.clients_i64.data_ptr() + rows * self.clients_i64.stride(0) * 8).to(eng.device)
        w = torch.from_numpy(fp32_weights(weights)).to(eng.device)
        s = None if scales is None else torch.from_numpy(fp32_weights(scales)).to(eng.device)
        self._keep = (pf, pi, w, s)
        eng.launch_fedavg(self.bucket_layout, pf, pi, w, s, k, self.base_f32, self.base_i64,
                          self.out_f32, self.out_i64f, stream)

    def gather(self, group=None) -> tuple[torch.Tensor, torch.Tensor]:
        return gather_buckets(self.plan, self.out_f32, self.out_i64f, group)
