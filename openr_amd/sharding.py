"""Multi-GPU sharding of SPF batches (one process per GPU, torch.distributed).

Two ways a node's worth of SPF work spreads over ranks:

* ``weak``: each rank owns an independent LSDB snapshot and solves all of its
  sources -- the what-if / per-iteration pattern of ``BM_DecisionFabric``
  (RoutingBenchmarkUtils.cpp:406-447: every iteration drains one rack
  switch).  Snapshot r drains node ``(r * 7919) mod N`` (r > 0).
* ``strong``: one LSDB, its sources interleaved over ranks (source i -> rank
  i mod world) so per-rank cost is balanced across switch roles.

For all-sources SPF neither puts a collective on the data path: results stay
in each GPU's HBM; only timings (MAX) and, for verification, 64-bit digests of
per-source results (all_gather) cross ranks.  KSP2 (sources dealt over ranks)
and what-if batches (failed links dealt over ranks) end with one exchange:
``gather_padded`` moves every rank's variable-length result buffer to rank 0
(RCCL on GPU tensors, gloo on CPU tensors in the tests).
"""

from __future__ import annotations

from typing import List, Sequence

import numpy as np

from .lsdb import PackedLsdb

VICTIM_STRIDE = 7919


def snapshot_for_rank(lsdb: PackedLsdb, rank: int) -> PackedLsdb:
    """Rank r's LSDB snapshot (a copy; rank 0 = the unmodified topology)."""
    dbs = lsdb.dbs.copy()
    if rank > 0:
        dbs["is_overloaded"][(rank * VICTIM_STRIDE) % len(dbs)] = 1
    return PackedLsdb(lsdb.blob, dbs, lsdb.adjs)


def victim_node(n_nodes: int, rank: int) -> int:
    return -1 if rank == 0 else (rank * VICTIM_STRIDE) % n_nodes


def source_shard(n_sources: int, rank: int, world: int) -> np.ndarray:
    """Interleaved source ids owned by `rank` (strong scaling)."""
    return np.arange(rank, n_sources, world, dtype=np.uint32)


_M1 = np.uint64(0x9E3779B97F4A7C15)
_M2 = np.uint64(0xBF58476D1CE4E5B9)


def row_digest(dist_row: np.ndarray, nh_words: np.ndarray) -> int:
    """Order-sensitive 64-bit digest of one source's result (host side)."""
    with np.errstate(over="ignore"):
        d = dist_row.astype(np.uint64)
        h = np.bitwise_xor.reduce((d + np.arange(len(d), dtype=np.uint64)) * _M1)
        if len(nh_words):
            w = nh_words.astype(np.uint64).ravel()
            h ^= np.bitwise_xor.reduce((w + np.arange(len(w), dtype=np.uint64) * _M2) * _M2)
    return int(h)


def gather_digests(local: Sequence[int], group=None) -> List[List[int]]:
    """all_gather of per-rank digest lists (small, int64)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = torch.tensor([len(local)], dtype=torch.int64)
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    cap = int(max(s.item() for s in sizes))
    buf = torch.zeros(cap, dtype=torch.int64)
    buf[: len(local)] = torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in local],
                                     dtype=torch.int64)
    out = [torch.zeros(cap, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    return [[int(v) & ((1 << 64) - 1) for v in o[: int(s.item())].tolist()]
            for o, s in zip(out, sizes)]


def gather_padded(t, length: int, dst: int = 0, group=None):
    """Gather the first `length` elements of the 1-D tensor `t` from every
    rank to rank `dst`: lengths are all_gathered, buffers padded to the
    longest, one ``dist.gather``.  Returns the per-rank tensors (trimmed) on
    `dst`, None elsewhere.  `t` must hold at least the longest length."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = torch.tensor([length], dtype=torch.int64, device=t.device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=t.device) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    lens = [int(x.item()) for x in sizes]
    cap = max(lens)
    if t.numel() < cap:  # pad a short local buffer
        pad = torch.zeros(cap, dtype=t.dtype, device=t.device)
        pad[: t.numel()] = t
        t = pad
    send = t[:cap].contiguous()
    out = [torch.empty(cap, dtype=t.dtype, device=t.device) for _ in range(world)] \
        if rank == dst else None
    dist.gather(send, out, dst=dst, group=group)
    if rank != dst:
        return None
    return [o[:m] for o, m in zip(out, lens)]


def max_over_ranks(x: float, device=None) -> float:
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
