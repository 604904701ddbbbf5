"""Sharded-resident all-sources on the GPU (bench.py's default multi-GPU mode,
SURVEY.md §8(e) row 1): every rank of a world-size-N run executes one plan
over its share of the sources (sharding.AllSourcesLayout: contiguous id
blocks or the locality partition) and keeps the rows in its own HBM; after the run rank 0 gathers per-source digests
computed on the GPU (spf_plan_digest).

On one GPU each rank's plan is run in turn, into its own buffers, exactly as
that rank would run it; the digests of all ranks together are compared with
the oracle's digests of every source (tests/golden/fullsize_*.npz).  Also:
spf_plan_digest equals the oracle's digest of the same output
(oracle.digest_planar) on small graphs in every plan mode.
"""

import numpy as np
import pytest

from oracle import digest_planar
from openr_amd import topology as T
from openr_amd.engine import SpfEngine, graph_from_lsdb
from openr_amd.hiprt import DeviceArray
from openr_amd.sharding import AllSourcesLayout
from test_gpu_fullsize import _make, golden

pytestmark = pytest.mark.gpu


def _run_rank(eng, srcs, dist64=False):
    plan = eng.plan(srcs, dist64=dist64)
    lab = 2 if dist64 else 1
    d = DeviceArray(max(1, len(srcs) * eng.pitch * lab), np.uint32, zero=True)
    nh = DeviceArray(max(1, plan.nh_words), np.uint32, zero=True)
    dg = DeviceArray(max(1, len(srcs)), np.uint64, zero=True)
    try:
        plan.execute(d.ptr, nh.ptr)
        plan.digest(d.ptr, nh.ptr, dg.ptr)
        eng.check()
        return dg.numpy()[: len(srcs)].copy()
    finally:
        plan.close()
        for b in (d, nh, dg):
            b.free()


@pytest.mark.parametrize("name", ["fabric_full", "grid100", "fabric_rtt"])
@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("partition", ["contiguous", "bench"])
def test_emulated_ranks_resident_digests_match_oracle(name, world, partition):
    """Every rank's plan of a world-N split -- the contiguous id blocks, and
    the layout bench.py builds (neighbour lists given: the locality
    partition where it shrinks the closures; team BFS plans for the rank
    shares of unit-metric graphs) -- digested on the GPU and reassembled,
    against the oracle's digest of every source."""
    meta, g = golden(name)
    ls, names, csr, cd = _make(name)
    assert cd == meta["csr_digest"]
    want = np.zeros(len(names), np.uint64)
    want[g["srcs"].astype(np.int64)] = g["digest"]
    eng = SpfEngine(0)
    try:
        eng.load(*csr)
        nbrs = [eng.neighbors(s) for s in range(len(names))]
        k = np.array([len(x) for x in nbrs], np.int64)
        layout = AllSourcesLayout(k, eng.pitch, world, nbrs=nbrs if partition == "bench" else None)
        if partition == "bench" and name != "grid100":
            assert layout.partition == "locality"  # fabrics: pods together
        got = np.zeros(len(names), np.uint64)
        for r in range(world):
            got[layout.srcs[r]] = _run_rank(eng, layout.srcs[r])
        assert sorted(np.concatenate(layout.srcs).tolist()) == list(range(len(names)))
        if name == "fabric_full" and world == 8 and partition == "bench":
            assert eng.plan(layout.srcs[0]).kernels()[0] == "msbfs_team_kernel"
    finally:
        eng.close()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{name} world {world}: {len(bad)} sources differ, first {bad[:5]}"


@pytest.mark.parametrize("case", ["unit", "hop", "weighted", "zero_metric", "dist64", "drained"])
def test_gpu_digest_equals_oracle_digest_of_same_output(case):
    topo = T.wan(300, 200, seed=3, max_metric=20) if case in ("weighted", "zero_metric", "dist64") \
        else T.fabric(1000, full=True)
    names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
    if case == "zero_metric":
        met = met.copy()
        met[::7] = 0
    if case == "drained":
        ovl = ovl.copy()
        ovl[::13] = 1
    srcs = list(range(0, len(names), 3))
    eng = SpfEngine(0)
    try:
        eng.load(rp, col, met, lid, ovl)
        hop, d64 = case == "hop", case == "dist64"
        with eng.plan(srcs, hop=hop, dist64=d64) as p:
            res = p.execute_host()
        if d64:  # the oracle digest reads u32 rows: compare through them
            assert res.dist.max(initial=0) < 2**32 - 1 or (res.dist == 2**64 - 1).any()
            dist32 = np.where(res.dist == np.uint64(2**64 - 1), np.uint64(0xFFFFFFFF),
                              res.dist).astype(np.uint32)
        else:
            dist32 = res.dist
        want = digest_planar(dist32, res.nh, res.nh_off, res.words, res.pitch)
        plan = eng.plan(srcs, hop=hop, dist64=d64)
        lab = 2 if d64 else 1
        d = DeviceArray(len(srcs) * eng.pitch * lab, np.uint32, zero=True)
        nh = DeviceArray(max(1, plan.nh_words), np.uint32, zero=True)
        dg = DeviceArray(len(srcs), np.uint64, zero=True)
        plan.execute(d.ptr, nh.ptr)
        plan.digest(d.ptr, nh.ptr, dg.ptr)
        eng.check()
        got = dg.numpy()[: len(srcs)]
        plan.close()
        for b in (d, nh, dg):
            b.free()
    finally:
        eng.close()
    assert np.array_equal(got, want)
