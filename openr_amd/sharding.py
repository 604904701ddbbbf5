"""Multi-GPU sharding of SPF batches (one process per GPU, torch.distributed).

All-sources SPF + ECMP (the ``bench.py`` default):
one LSDB replicated on every GPU, its sources split over ranks
(:class:`AllSourcesLayout`), every rank solving its share.  By default the
per-source results -- distance rows and next-hop bitmaps in the engine's
layout -- stay resident in the owning rank's HBM (``Decision::
getDecisionRouteDb`` for a node is answered by the rank that owns it,
Decision.cpp:1480-1500); rank 0 gathers only per-source digests
(:meth:`AllSourcesLayout.assemble_digests`).  The dense mode gathers every
rank's rows and bitmaps to rank 0 over RCCL instead.  Sources go to ranks
balanced by next-hop work, grouped so that each rank's closure stays small:
a source's next hops need the distance rows of its neighbours, which the
rank computes too (the plan's closure).  Contiguous id blocks keep it small
on grids; a fabric needs the locality partition (:func:`locality_partition`:
a pod's switches together), which halves the largest closure of 8 ranks.

Weak scaling over per-rank LSDB snapshots (``snapshot_for_rank``, the
per-iteration drain of ``BM_DecisionFabric``, RoutingBenchmarkUtils.cpp:
406-447) stays available as a labelled extra (``bench.py --scaling weak``).

KSP2 (sources dealt over ranks) and what-if batches (failed links dealt over
ranks) end with one exchange too: ``gather_padded`` moves every rank's
variable-length result buffer to rank 0 (RCCL on GPU tensors, gloo on CPU
tensors in the tests).
"""

from __future__ import annotations

from typing import List, Optional, Sequence

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
    """Interleaved source ids owned by `rank`."""
    return np.arange(rank, n_sources, world, dtype=np.uint32)


def closure_sizes(srcs: Sequence[np.ndarray], nbrs: Sequence, n: int) -> List[int]:
    """Rows each rank's plan solves: its sources and their distinct up
    neighbours (the next-hop pass of source s reads the rows of s's
    neighbours, spf_plan_closure_rows)."""
    out = []
    for ss in srcs:
        m = np.zeros(n, bool)
        m[np.asarray(ss, np.int64)] = True
        if len(ss):
            m[np.concatenate([np.asarray(nbrs[int(s)], np.int64) for s in ss])] = True
        out.append(int(m.sum()))
    return out


def locality_partition(nbrs: Sequence, cost: np.ndarray, world: int,
                       slack: float = 0.03) -> List[np.ndarray]:
    """Sources to ranks so that each rank's closure (its sources plus their
    neighbours, all of which its plan must solve) stays small: a one-pass
    streaming partition (in the manner of linear deterministic greedy):
    nodes in ascending degree, each to the rank whose closure it grows least
    among the ranks whose source cost stays within (1 + slack) of the mean,
    ties to the least-loaded rank.  Low-degree nodes first: a fabric's rack
    switches gather by pod (they share their pod's fabric switches), the
    fabric switches follow their pod and a plane's spines land together --
    the closure of a rank of 8 is ~1.8k rows instead of up to 4.8k for id
    blocks (FSW blocks need every rack switch of their pods).  Generic: only
    the neighbour lists are used."""
    n = len(nbrs)
    deg = np.array([len(x) for x in nbrs], np.int64)
    order = np.lexsort((np.arange(n), deg))
    cost = np.asarray(cost, np.float64)
    cap = cost.sum() / world * (1.0 + slack)
    clo = np.zeros((world, n), bool)
    load = np.zeros(world)
    owner = np.empty(n, np.int64)
    for v in order:
        nb = np.append(np.asarray(nbrs[v], np.int64), v)
        new = (~clo[:, nb]).sum(axis=1).astype(np.float64)
        ok = load + cost[v] <= cap
        if not ok.any():
            ok[:] = True
        new[~ok] = np.inf
        best = np.flatnonzero(new == new.min())
        r = int(best[np.argmin(load[best])])
        owner[v] = r
        clo[r, nb] = True
        load[r] += cost[v]
    return [np.flatnonzero(owner == r).astype(np.uint32) for r in range(world)]


class AllSourcesLayout:
    """Where every source's result lives when the all-sources pass is split
    over `world` ranks and gathered to rank 0.

    ``k[v]`` = distinct up neighbours of v (the number of next-hop bitmaps of
    source v, ``spf_src_neighbors``), ``pitch`` = the engine's row pitch.
    Rank r solves ``srcs[r]`` (one plan, sources in ascending id) and writes
    its results into one contiguous send buffer of u32 words:
    ``[dist rows: len(srcs[r]) x pitch][next-hop bitmaps: nh_words[r]]`` --
    exactly the plan's own output layout (``spf_plan_nh_layout``), so the
    kernels write the send buffer directly.  With ``dist_bytes=1`` the
    distance rows are the plan's u8 rows (``spf_plan_copy_narrow_rows``,
    a quarter of the bytes on the wire; lossless while every distance is
    below 254, which the caller checks).  Buffers are padded to
    ``cap`` words so one ``gather`` moves them; rank 0 ends up with
    ``world x cap`` words from which :meth:`dist_row` / :meth:`nh_block`
    read any source's result."""

    # a source's cost in next-hop bitmaps (N/8 bytes each): its k bitmaps plus
    # its distance rows (u32 + u8 copy = 5N bytes = 40 bitmaps) -- the bytes
    # every rank's kernels write dominate a pass
    ROW_COST = 40
    LOCALITY_MAX_NODES = 1 << 16

    def __init__(self, k: np.ndarray, pitch: int, world: int, dist_bytes: int = 4,
                 row_cost: float = ROW_COST, nbrs: Optional[Sequence] = None,
                 partition: str = "auto") -> None:
        k = np.asarray(k, np.int64)
        n = len(k)
        assert dist_bytes in (1, 4) and (pitch * dist_bytes) % 4 == 0
        self.n, self.pitch, self.world = n, pitch, world
        self.dist_bytes = dist_bytes
        row_words = pitch * dist_bytes // 4  # a distance row in u32 words
        self.k = k
        wpm = pitch // 32
        # contiguous blocks balanced by the bytes each source's results take
        cost = np.cumsum(k + row_cost, dtype=np.float64)
        total = cost[-1] if n else 0.0
        bounds = [0] + [int(np.searchsorted(cost, total * r / world, side="right"))
                        for r in range(1, world)] + [n]
        self.srcs = [np.arange(bounds[r], bounds[r + 1], dtype=np.uint32) for r in range(world)]
        self.partition = "contiguous"
        self.closure = None
        if nbrs is not None and world > 1 and n <= self.LOCALITY_MAX_NODES:
            # a rank also solves its sources' neighbours (the next-hop pass
            # reads their rows): take the locality partition when its largest
            # closure is smaller than the contiguous blocks'.  The engine's
            # spf_partition_sources decides (the rule spf_mplan uses too; the
            # numpy restatement locality_partition is its test oracle)
            from .engine import partition_sources

            cont = closure_sizes(self.srcs, nbrs, n)
            self.closure = cont
            if partition in ("auto", "locality") and row_cost == self.ROW_COST:
                nb_ptr = np.concatenate([[0], np.cumsum([len(x) for x in nbrs])]).astype(np.uint32)
                nb_id = (np.concatenate([np.asarray(x, np.uint32) for x in nbrs])
                         if n else np.zeros(0, np.uint32))
                part, used = partition_sources(nb_ptr, nb_id, np.arange(n, dtype=np.uint32), world,
                                               partition)
                if used == "locality":
                    loc = [np.flatnonzero(part == r).astype(np.uint32) for r in range(world)]
                    self.srcs, self.closure, self.partition = loc, closure_sizes(loc, nbrs, n), "locality"
            elif partition in ("auto", "locality"):
                loc = locality_partition(nbrs, k + row_cost, world)
                loc_c = closure_sizes(loc, nbrs, n)
                if partition == "locality" or max(loc_c) < max(cont):
                    self.srcs, self.closure, self.partition = loc, loc_c, "locality"
        self.rank_of = np.zeros(n, np.int64)
        self.index_of = np.zeros(n, np.int64)
        self.nh_off = np.zeros(n, np.int64)  # word offset within the rank's send buffer
        self.dist_off = np.zeros(n, np.int64)
        self.words = []
        for r, ss in enumerate(self.srcs):
            m = len(ss)
            self.rank_of[ss] = r
            self.index_of[ss] = np.arange(m)
            self.dist_off[ss] = np.arange(m, dtype=np.int64) * row_words
            nh_local = np.concatenate([[0], np.cumsum(k[ss] * wpm)[:-1]]).astype(np.int64) \
                if m else np.zeros(0, np.int64)
            self.nh_off[ss] = m * row_words + nh_local
            self.words.append(int(m * row_words + (k[ss] * wpm).sum()))
        self.dist_words = [len(ss) * row_words for ss in self.srcs]
        self.cap = max(self.words) if self.words else 0

    def plan_nh_off(self, rank: int) -> np.ndarray:
        """The plan-relative next-hop offsets rank `rank`'s plan must report."""
        ss = self.srcs[rank]
        return (self.nh_off[ss] - self.dist_words[rank]).astype(np.uint64)

    def dist_row(self, recv: Sequence, s: int):
        """Source s's distances (u32, SPF_UNREACHABLE) from host buffers; u8
        rows (dist_bytes 1: the engine's narrow rows, lossless below 254)
        are widened, 255 -> unreachable."""
        r = int(self.rank_of[s])
        o = int(self.dist_off[s])
        if self.dist_bytes == 4:
            return recv[r][o: o + self.n]
        b = np.asarray(recv[r]).view(np.uint8)[4 * o: 4 * o + self.n]
        return np.where(b == 255, np.uint32(0xFFFFFFFF), b.astype(np.uint32))

    def nh_block(self, recv: Sequence, s: int):
        """Next-hop bitmaps of source s: k[s] rows of pitch/32 words."""
        r = int(self.rank_of[s])
        o = int(self.nh_off[s])
        return recv[r][o: o + int(self.k[s]) * (self.pitch // 32)]

    def owner(self, s: int):
        """(rank, row index in that rank's plan) holding source s's result."""
        return int(self.rank_of[s]), int(self.index_of[s])

    def assemble_digests(self, parts: Sequence) -> np.ndarray:
        """Per-source u64 digests of the whole graph from every rank's list
        (rank r's plan order = ``srcs[r]``), as rank 0 receives them."""
        out = np.zeros(self.n, np.uint64)
        for r, part in enumerate(parts):
            a = np.asarray(part.cpu() if hasattr(part, "cpu") else part)
            out[self.srcs[r]] = a.view(np.uint64)[: len(self.srcs[r])]
        return out

    def dense(self, recv: Sequence):
        """Rank 0's gathered buffers as whole-graph arrays (host numpy):
        dist [n, n] u32 and the next-hop words with per-source offsets
        (nh_off, k) -- the layout a single-rank plan over all sources has."""
        dist = np.zeros((self.n, self.n), np.uint32)
        wpm = self.pitch // 32
        nh_off = np.concatenate([[0], np.cumsum(self.k * wpm)[:-1]]).astype(np.uint64)
        nh = np.zeros(max(1, int((self.k * wpm).sum())), np.uint32)
        host = [np.asarray(b.cpu() if hasattr(b, "cpu") else b).view(np.uint32) for b in recv]
        for s in range(self.n):
            dist[s] = self.dist_row(host, s)
            blk = self.nh_block(host, s)
            nh[int(nh_off[s]): int(nh_off[s]) + len(blk)] = blk
        return dist, nh, nh_off, self.k.astype(np.uint32)


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
