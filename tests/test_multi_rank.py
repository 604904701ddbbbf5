"""The multi-GPU sharding logic on CPU with the gloo backend (world size 2).

Each rank builds its own LSDB snapshot (weak scaling) or its interleaved
source shard (strong scaling), solves it with the CPU oracle standing in for
the GPU (no device here), and all_gathers 64-bit per-source digests; rank 0
recomputes every rank's work alone and checks the gathered digests, the
timing MAX reduction, and that shards partition the sources.
"""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solve(lsdb, srcs):
    from oracle import OracleLinkState
    from openr_amd.engine import graph_from_lsdb
    from openr_amd.sharding import row_digest

    names = graph_from_lsdb(lsdb)[0]
    orc = OracleLinkState()
    orc.update_packed(lsdb)
    dist, mats = orc.dense(names, list(srcs))
    return [row_digest(dist[i], np.packbits(mats[i], axis=1, bitorder="little"))
            for i in range(len(srcs))]


def _worker(rank, world, port, mode, q):
    import sys
    from pathlib import Path

    here = Path(__file__).resolve().parent
    sys.path.insert(0, str(here))
    sys.path.insert(0, str(here.parent))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from openr_amd import sharding as S
    from openr_amd import topology as T

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        topo = T.fabric(700, full=True)
        n = topo.n_nodes
        if mode == "weak":
            lsdb = S.snapshot_for_rank(topo.lsdb, rank)
            srcs = np.arange(0, n, 37, dtype=np.uint32)
        else:
            lsdb = topo.lsdb
            srcs = S.source_shard(n, rank, world)[::9]
        digests = _solve(lsdb, srcs)
        gathered = S.gather_digests(digests)
        tmax = S.max_over_ranks(float(rank + 1))
        if rank == 0:
            expect = []
            for r in range(world):
                if mode == "weak":
                    expect.append(_solve(S.snapshot_for_rank(topo.lsdb, r),
                                         np.arange(0, n, 37, dtype=np.uint32)))
                else:
                    expect.append(_solve(topo.lsdb, S.source_shard(n, r, world)[::9]))
            q.put((gathered == expect, tmax))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["weak", "strong"])
def test_two_rank_sharding_gloo(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok, tmax = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok
    assert tmax == 2.0


def test_shards_partition_sources():
    from openr_amd.sharding import source_shard

    for world in (1, 2, 3, 8):
        allv = np.concatenate([source_shard(9976, r, world) for r in range(world)])
        assert np.array_equal(np.sort(allv), np.arange(9976))


def test_snapshots_differ_only_in_one_drain_bit():
    from openr_amd import topology as T
    from openr_amd.sharding import snapshot_for_rank, victim_node

    topo = T.fabric(1000, full=True)
    base = snapshot_for_rank(topo.lsdb, 0)
    assert np.array_equal(base.dbs, topo.lsdb.dbs)
    for r in (1, 2, 7):
        snap = snapshot_for_rank(topo.lsdb, r)
        diff = np.nonzero(snap.dbs["is_overloaded"] != topo.lsdb.dbs["is_overloaded"])[0]
        assert list(diff) == [victim_node(topo.n_nodes, r)]
