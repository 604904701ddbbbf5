"""The multi-GPU sharding logic on CPU with the gloo backend (world size 2-3).

Each rank builds its own LSDB snapshot (weak scaling) or its interleaved
source shard, solves it with the CPU oracle standing in for the GPU (no
device here), and all_gathers 64-bit per-source digests; rank 0 recomputes
every rank's work alone and checks the gathered digests, the timing MAX
reduction, and that shards partition the sources.  The all-sources layout
(contiguous blocks balanced by next-hop work, bench.py's default) is
covered in both result modes: resident rows with per-source digests
gathered to rank 0, and the dense gather of rows + bitmaps.  The engine's
own per-rank plans and GPU digests are checked against the oracle's
full-size digests in tests/test_gpu_sharded.py.
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


# ---- KSP2 and what-if: sharded work + one gather_padded exchange -------------
def _ksp2_pack(topo, srcs):
    """Oracle getKthPaths(s, d, 1/2) for srcs x all d, packed like
    spf_ksp2_pair + path pool (link = index of its sorted key)."""
    import json

    from oracle import OracleLinkState

    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    names = sorted(topo.nodes)
    keys = {}
    pairs, pool = [], []
    for s in srcs:
        for d in names:
            hdr = [0xFFFFFFFF, 0xFFFFFFFF, 0, 0]
            for k in (1, 2):
                prev = None
                for path in orc.kth_paths(names[s], d, k):
                    at = len(pool)
                    pool += [len(path), 0xFFFFFFFF]
                    pool += [keys.setdefault(json.dumps(l), len(keys)) for l in path]
                    if prev is None:
                        hdr[k - 1] = at
                    else:
                        pool[prev + 1] = at
                    prev = at
                    hdr[k + 1] += 1
            pairs += hdr
    return pairs, pool, keys


def _ksp2_unpack(pairs, pool, keys, n_src, n):
    inv = {v: k for k, v in keys.items()}
    out = []
    for i in range(n_src * n):
        rec = pairs[4 * i: 4 * i + 4]
        one = []
        for k in (0, 1):
            at, paths = rec[k], []
            for _ in range(rec[k + 2]):
                ln = pool[at]
                paths.append([inv[x] for x in pool[at + 2: at + 2 + ln]])
                at = pool[at + 1]
            one.append(paths)
        out.append(one)
    return out


def _exchange_worker(rank, world, port, q):
    import sys
    from pathlib import Path

    here = Path(__file__).resolve().parent
    sys.path.insert(0, str(here))
    sys.path.insert(0, str(here.parent))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from oracle import NameTable, OracleLinkState, whatif_digests
    from openr_amd import sharding as S
    from openr_amd import topology as T
    from openr_amd.link_state import LinkState

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok = True
        # KSP2: sources dealt round-robin, pairs + pools gathered to rank 0
        # (link ids index each shard's own key table, rebuilt on rank 0)
        topo = T.wan(30, 15, seed=4)
        n = topo.n_nodes
        srcs = S.source_shard(n, rank, world)
        pairs, pool, _ = _ksp2_pack(topo, srcs)
        t_pairs = torch.tensor([x - (1 << 32) if x >= (1 << 31) else x for x in pairs],
                               dtype=torch.int32)
        t_pool = torch.tensor([(x - (1 << 32) if x >= (1 << 31) else x) for x in pool] or [0],
                              dtype=torch.int32)
        gp = S.gather_padded(t_pairs, len(pairs))
        gq = S.gather_padded(t_pool, len(pool))
        # what-if: failed links dealt round-robin, 16-byte digests gathered
        ba = T.barabasi_albert(300, 2, seed=3)
        ls = LinkState(device=-1)
        ls.updateAdjacencyDatabases(ba.lsdb)
        names, rp, col, met, lid, ovl = ls.flatten()
        links = sorted(set(int(x) for x in lid))
        mine = links[rank::world]
        orc = OracleLinkState()
        orc.update_packed(ba.lsdb)
        fails = [(ls._link(l)._n1, ls._link(l)._if1) for l in mine]
        _, dg = whatif_digests(orc, NameTable(names), names[0], fails)
        t_dg = torch.tensor([v for d in dg for v in (d[0], d[1], d[2] - (1 << 64)
                                                     if d[2] >= (1 << 63) else d[2])] or [0],
                            dtype=torch.int64)
        gd = S.gather_padded(t_dg, 3 * len(dg))
        if rank == 0:
            u32 = lambda t: [int(x) & 0xFFFFFFFF for x in t.tolist()]  # noqa: E731
            # KSP2: every rank's shard decodes to the oracle's full answer
            for r in range(world):
                rs = list(S.source_shard(n, r, world))
                got = _ksp2_unpack(u32(gp[r]), u32(gq[r]), _ksp2_pack(topo, rs)[2], len(rs), n)
                want_p, want_q, want_k = _ksp2_pack(topo, rs)
                ok &= got == _ksp2_unpack(want_p, want_q, want_k, len(rs), n)
            # what-if: interleave the shards back into link order
            full = [None] * len(links)
            for r in range(world):
                vals = [int(x) & ((1 << 64) - 1) for x in gd[r].tolist()]
                for j, i in enumerate(range(r, len(links), world)):
                    full[i] = tuple(vals[3 * j: 3 * j + 3])
            allf = [(ls._link(l)._n1, ls._link(l)._if1) for l in links]
            _, want = whatif_digests(orc, NameTable(names), names[0], allf)
            ok &= full == [tuple(w) for w in want]
            q.put(bool(ok))
    finally:
        dist.destroy_process_group()


def test_two_rank_ksp2_and_whatif_exchange_gloo():
    """The one collective of the KSP2 and what-if paths (gather_padded of
    variable-length per-rank results) reassembles exactly the single-rank
    answer."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok


# ---- all-sources split + gather to rank 0 ------------
def _all_sources_worker(rank, world, port, q, dist_bytes=4, locality=False):
    import sys
    from pathlib import Path

    here = Path(__file__).resolve().parent
    sys.path.insert(0, str(here))
    sys.path.insert(0, str(here.parent))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from helpers import planar_rows
    from oracle import OracleLinkState
    from openr_amd import topology as T
    from openr_amd.engine import graph_from_lsdb
    from openr_amd.sharding import AllSourcesLayout

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        topo = T.fabric(700, full=True)
        names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
        n = len(names)
        pitch = (n + 63) // 64 * 64
        nbrs = [np.unique(col[rp[v]:rp[v + 1]]) for v in range(n)]
        k = np.array([len(x) for x in nbrs])
        lay = AllSourcesLayout(k, pitch, world, dist_bytes, nbrs=nbrs if locality else None,
                               partition="locality" if locality else "auto")
        assert lay.partition == ("locality" if locality else "contiguous")
        orc = OracleLinkState()
        orc.update_packed(topo.lsdb)
        # this rank's share, in the plan layout, written into the send buffer
        srcs = lay.srcs[rank]
        d, mats = orc.dense(names, list(srcs))
        d32, nh = planar_rows(k[srcs], d, mats, pitch)
        if dist_bytes == 1:  # the engine's narrow rows: min(d, 254), 255 = unreachable
            rows = np.where(d32 == 0xFFFFFFFF, 255, np.minimum(d32, 254)).astype(np.uint8)
            d32 = rows.ravel().view(np.uint32)
        send = torch.zeros(lay.cap, dtype=torch.int32)
        flat = np.concatenate([d32.ravel(), nh]).view(np.int32)
        assert len(flat) == lay.words[rank]
        send[: len(flat)] = torch.from_numpy(flat)
        recv = [torch.zeros(lay.cap, dtype=torch.int32) for _ in range(world)] if rank == 0 else None
        dist.gather(send, recv, dst=0)
        if rank == 0:
            got_d, got_nh, got_off, got_k = lay.dense(recv)
            # the single-rank answer: every source in one plan layout
            d_all, mats_all = orc.dense(names, list(range(n)))
            e32, enh = planar_rows(k, d_all, mats_all, pitch)
            q.put((np.array_equal(got_d, e32[:, :n]), np.array_equal(got_nh[: len(enh)], enh),
                   sorted(np.concatenate(lay.srcs).tolist()) == list(range(n))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dist_bytes,locality", [(2, 4, False), (3, 4, False), (2, 1, False),
                                                       (3, 1, False), (2, 4, True), (3, 1, True)])
def test_all_sources_split_and_gather_reassembles_single_rank_result(world, dist_bytes, locality):
    """One LSDB, sources split over ranks (contiguous id blocks, or the
    locality partition bench.py takes for fabrics), every rank's dist rows
    (u32, or the engine's u8 rows) + next-hop bitmaps gathered to rank 0
    (gloo here, RCCL in bench.py): rank 0's reassembled arrays equal the
    single-rank all-sources result bit for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_all_sources_worker, args=(r, world, port, q, dist_bytes, locality))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == (True, True, True)


def test_locality_partition_shrinks_fabric_closures():
    """sharding.locality_partition on fabric_full (the bench's 8-rank split):
    every source on exactly one rank, each rank's sources ascending, source
    cost within the slack of the mean (plus one source), and the largest
    closure -- the rows a rank's plan must solve -- well below the
    contiguous blocks' (which need every rack switch of a fabric block's
    pods).  A grid keeps its contiguous blocks."""
    from openr_amd import topology as T
    from openr_amd.engine import graph_from_lsdb
    from openr_amd.sharding import AllSourcesLayout, closure_sizes, locality_partition

    topo = T.fabric(10000, full=True)
    names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
    n = len(names)
    nbrs = [np.unique(col[rp[v]:rp[v + 1]]) for v in range(n)]
    k = np.array([len(x) for x in nbrs], np.int64)
    cost = k + AllSourcesLayout.ROW_COST
    for world in (2, 4, 8):
        parts = locality_partition(nbrs, cost, world)
        allv = np.concatenate(parts)
        assert sorted(allv.tolist()) == list(range(n))
        assert all(np.all(np.diff(p.astype(np.int64)) > 0) for p in parts)
        load = [int(cost[p].sum()) for p in parts]
        assert max(load) <= cost.sum() / world * 1.03 + cost.max()
        lay = AllSourcesLayout(k, 10240, world, nbrs=nbrs)
        cont = closure_sizes(AllSourcesLayout(k, 10240, world).srcs, nbrs, n)
        assert lay.partition == "locality" and max(lay.closure) < 0.75 * max(cont)
    gt = T.grid(30)
    names, rp, col, met, lid, ovl = graph_from_lsdb(gt.lsdb)
    nb = [np.unique(col[rp[v]:rp[v + 1]]) for v in range(len(names))]
    lay = AllSourcesLayout(np.array([len(x) for x in nb]), 1024, 4, nbrs=nb)
    assert lay.partition in ("contiguous", "locality")
    assert sorted(np.concatenate(lay.srcs).tolist()) == list(range(len(names)))


def test_all_sources_layout_blocks_balance_next_hop_work():
    from openr_amd.sharding import AllSourcesLayout

    rng = np.random.default_rng(0)
    k = rng.integers(1, 200, 9976)
    rc = AllSourcesLayout.ROW_COST
    for world in (1, 2, 4, 8):
        lay = AllSourcesLayout(k, 10048, world)
        assert np.array_equal(np.concatenate(lay.srcs), np.arange(9976))
        work = [int((k[s] + rc).sum()) for s in lay.srcs]
        assert max(work) - min(work) <= 2 * (k.max() + rc)
        assert lay.cap == max(lay.words)


def _resident_worker(rank, world, port, q):
    """bench.py's resident mode: rank r solves its share of the sources, digests
    its own rows (the oracle's digest_planar over the engine's output layout
    standing in for spf_plan_digest), rank 0 gathers the digests
    (gather_padded) and reassembles them with the layout."""
    import sys
    from pathlib import Path

    here = Path(__file__).resolve().parent
    sys.path.insert(0, str(here))
    sys.path.insert(0, str(here.parent))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from oracle import NameTable, OracleLinkState, source_digests
    from openr_amd import topology as T
    from openr_amd.engine import graph_from_lsdb
    from openr_amd.sharding import AllSourcesLayout, gather_padded

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        topo = T.fabric_rtt(num_sws=700)
        names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
        n = len(names)
        nbrs = [np.unique(col[rp[v]:rp[v + 1]]) for v in range(n)]
        k = np.array([len(x) for x in nbrs], np.int64)
        layout = AllSourcesLayout(k, 1024, world, nbrs=nbrs)  # bench.py's layout
        orc = OracleLinkState()
        orc.update_packed(topo.lsdb)
        table = NameTable(names)
        mine = source_digests(orc, table, layout.srcs[rank], threads=1)
        t = torch.from_numpy(mine.view(np.int64).copy())
        got = gather_padded(t, len(mine))
        if rank == 0:
            whole = layout.assemble_digests(got)
            alone = source_digests(orc, table, np.arange(n, dtype=np.uint32), threads=1)
            q.put(("ok", bool(np.array_equal(whole, alone)),
                   sorted(np.concatenate(layout.srcs).tolist()) == list(range(n))))
    except Exception as e:  # noqa: BLE001
        q.put(("err", repr(e), False))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_resident_mode_digest_gather_reassembles_single_rank_digests(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_resident_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    status, same, partition = q.get(timeout=600)
    for p in ps:
        p.join(timeout=120)
    assert status == "ok", same
    assert same and partition
