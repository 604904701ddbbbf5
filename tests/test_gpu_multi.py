"""Several GPUs behind one C-ABI context (spf_mctx / spf_mplan,
include/openr_spf.h) and the LinkState facade over it (ls_create_multi,
ls_prefetch_all_sources), on the one-GPU test box with repeated device ids:
members of one device run one after another on its stream, so a world of
N members there computes exactly what N GPUs would.

* every source of fabric_full / grid100 / fabric_rtt split over 2, 4, 8
  members: per-source digests computed on the owning member against the
  oracle's (tests/golden/fullsize_*.npz);
* a member's resident rows, bitmaps and pathLinks equal one plan's;
* hipGraph replays of the members' executes (spf_mplan_set_graphs), also
  interleaved with another context's grid-resident launches;
* the facade: getSpfResult(node) answered from the resident pass equals the
  oracle (metrics, next hops, pathLinks order) and counts spf_runs like the
  reference's lazy getSpfResult (LinkState.cpp:815); a publication drops the
  pass (LinkState.cpp:509-512);
* the execute contract: work on the legacy null stream (hipMemset) before
  spf_plan_execute(..., stream = NULL) is ordered before it.
"""

import ctypes as C

import numpy as np
import pytest

from helpers import spf_canonical
from oracle import OracleLinkState
from openr_amd import hiprt
from openr_amd import topology as T
from openr_amd.engine import SpfEngine, SpfMultiEngine
from openr_amd.link_state import LinkState
from test_gpu_fullsize import _make, golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,world", [("fabric_full", 2), ("fabric_full", 4), ("fabric_full", 8),
                                        ("grid100", 2), ("fabric_rtt", 4)])
def test_multi_context_every_source_matches_oracle(name, world):
    meta, g = golden(name)
    ls, names, csr, cd = _make(name)
    assert cd == meta["csr_digest"]
    want = np.zeros(len(names), np.uint64)
    want[g["srcs"].astype(np.int64)] = g["digest"]
    with SpfMultiEngine([0] * world) as m:
        m.load(*csr)
        p = m.plan(np.arange(len(names)))
        assert sum(p.shard_sizes()) == len(names) and min(p.shard_sizes()) > 0
        if name == "fabric_full":
            assert p.partition == "locality"
            if world == 8:  # rank shares run on the team BFS
                assert p.member_kernels(0)[0] == "msbfs_team_kernel"
        p.execute()
        p.synchronize()
        got = p.digest()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{name} x{world}: {len(bad)} sources differ, first {bad[:5]}"


def test_multi_context_enqueue_threads_every_source_matches_oracle():
    """Each member's execute issued from its own host thread
    (spf_mplan_set_enqueue_threads(1)): the same digests, repeated executes,
    and the enqueue times are reported for every member."""
    meta, g = golden("fabric_full")
    ls, names, csr, cd = _make("fabric_full")
    want = np.zeros(len(names), np.uint64)
    want[g["srcs"].astype(np.int64)] = g["digest"]
    with SpfMultiEngine([0] * 4) as m:
        m.load(*csr)
        p = m.plan(np.arange(len(names)))
        p.set_enqueue_threads(1)
        for _ in range(3):
            p.execute()
            ns, threaded = p.enqueue_ns()
            assert threaded and len(ns) == 4 and (ns > 0).all()
        p.synchronize()
        got = p.digest()
        p.set_enqueue_threads(0)
        p.execute()
        ns, threaded = p.enqueue_ns()
        assert not threaded and (np.diff(ns.astype(np.int64)) > 0).all()  # one after another
        p.synchronize()
        assert np.array_equal(p.digest(), got)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} sources differ, first {bad[:5]}"


def test_multi_context_rows_bitmaps_preds_equal_one_plan():
    topo = T.fabric(1000, full=True)
    ls = LinkState(device=-1)
    ls.updateAdjacencyDatabases(topo.lsdb)
    names, *csr = ls.flatten()
    n = len(names)
    srcs = np.arange(0, n, 3, dtype=np.uint32)[::-1].copy()  # a subset, not in id order
    with SpfEngine(0) as e1, SpfMultiEngine([0, 0, 0]) as m:
        e1.load(*csr)
        m.load(*csr)
        ref = e1.solve(srcs)
        p = m.plan(srcs, mode="locality")
        p.execute()
        p.synchronize()
        for i in range(0, len(srcs), 17):
            dist, nh = p.read(i)
            assert np.array_equal(dist, ref.dist[i])
            assert np.array_equal(nh, ref.nh_matrix(i))
            pp, pe = p.preds(i)
            rp, re_ = e1.preds(int(srcs[i]), ref.dist[i])
            assert np.array_equal(pp, rp) and np.array_equal(pe, re_)
        owners = {p.owner(i)[0] for i in range(len(srcs))}
        assert owners == {0, 1, 2}


def test_multi_context_graph_replay_and_patch():
    """hipGraph replays of every member's execute give the oracle's digests;
    an in-place patch (drain a node on every replica) re-derives and
    re-captures, and the replays follow the new graph."""
    meta, g = golden("fabric_full")
    ls, names, csr, cd = _make("fabric_full")
    want = np.zeros(len(names), np.uint64)
    want[g["srcs"].astype(np.int64)] = g["digest"]
    with SpfMultiEngine([0, 0, 0, 0]) as m, SpfEngine(0) as e1:
        m.load(*csr)
        p = m.plan(np.arange(len(names)))
        p.set_graphs(True)
        for _ in range(3):  # execute, capture, replay
            p.execute()
        p.synchronize()
        assert np.array_equal(p.digest(), want)
        victim = names.index("3-1-7")
        m.set_overload([victim], [1])
        for _ in range(3):
            p.execute()
        p.synchronize()
        got = p.digest()
        csr2 = list(csr)
        csr2[4] = csr[4].copy()
        csr2[4][victim] = 1
        e1.load(*csr2)
        q = e1.plan(np.arange(len(names)))
        d = hiprt.DeviceArray(len(names) * e1.pitch, np.uint32, zero=True)
        nh = hiprt.DeviceArray(max(1, q.nh_words), np.uint32, zero=True)
        dg = hiprt.DeviceArray(len(names), np.uint64, zero=True)
        q.execute(d.ptr, nh.ptr)
        q.digest(d.ptr, nh.ptr, dg.ptr)
        e1.check()
        ref = dg.numpy()
        q.close()
        for b in (d, nh, dg):
            b.free()
    assert (got != want).any()  # the drain changed results
    assert np.array_equal(got, ref)


def test_patch_right_after_execute_is_ordered_after_it():
    """a drain patched onto every replica right after an execute
    (no synchronize between) waits for the members' executes still reading
    the graph (repeated ids: members run on the first member's stream), and
    the next execute follows the patched graph."""
    ls, names, csr, cd = _make("fabric_full")
    victim = names.index("3-2-5")
    csr2 = list(csr)
    csr2[4] = csr[4].copy()
    csr2[4][victim] = 1
    with SpfMultiEngine([0, 0, 0, 0]) as m, SpfMultiEngine([0]) as ref:
        m.load(*csr)
        p = m.plan(np.arange(len(names)))
        for _ in range(2):
            p.execute()
            m.set_overload([victim], [1])  # no synchronize before the patch
            p.execute()
            m.set_overload([victim], [0])
        m.set_overload([victim], [1])
        p.execute()
        p.synchronize()
        got = p.digest()
        ref.load(*csr2)
        q = ref.plan(np.arange(len(names)))
        q.execute()
        q.synchronize()
        want = q.digest()
    assert np.array_equal(got, want)


def test_graph_replays_beside_another_contexts_resident_launches():
    """replays of captured team-BFS executes (grid-resident) and a
    second context's grid-resident what-if launches, issued back to back on
    the same device with no synchronisation between the two contexts, stay
    ordered per device (resident_order around every replay): both results
    are exact and no team barrier gives up."""
    from openr_amd.engine import DIGEST_DTYPE

    meta, g = golden("fabric_full")
    ls, names, csr, cd = _make("fabric_full")
    want = np.zeros(len(names), np.uint64)
    want[g["srcs"].astype(np.int64)] = g["digest"]
    topo = T.barabasi_albert(3000, 3, seed=5)
    ls2 = LinkState(device=-1)
    ls2.updateAdjacencyDatabases(topo.lsdb)
    csr2 = ls2.flatten()[1:]
    with SpfMultiEngine([0] * 8) as m, SpfEngine(0) as e2:
        m.load(*csr)
        p = m.plan(np.arange(len(names)))
        assert p.member_kernels(0)[0] == "msbfs_team_kernel"
        p.set_graphs(True)
        e2.load(*csr2)
        links, ref, base = e2.whatif(0)
        wp = e2.whatif_plan(0)
        out = hiprt.DeviceArray(2 * len(links), np.uint64, zero=True)
        for _ in range(4):  # execute, capture, replays -- each beside a what-if launch
            p.execute()
            wp.execute(out.ptr)
        p.synchronize()
        e2.check()
        assert np.array_equal(p.digest(), want)
        got = out.numpy().view(DIGEST_DTYPE)[: len(links)]
        out.free()
    for f in ("n_dist_changed", "n_nh_changed", "hash"):
        assert np.array_equal(got[f], ref[f])


@pytest.mark.parametrize("ulm", [True, False], ids=["metric", "hops"])
def test_facade_serves_get_spf_result_from_resident_pass(ulm):
    topo = T.fabric(1000, full=True)
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    ls = LinkState(devices=[0, 0])
    ls.updateAdjacencyDatabases(topo.lsdb)
    runs0 = ls.spfRuns()
    ls.prefetchAllSources(ulm)
    assert ls.spfRuns() == runs0  # nothing read yet (the reference is lazy)
    dg = ls.allSourcesDigests()
    assert dg is not None and len(dg) == len(topo.nodes)
    sample = list(dict.fromkeys(topo.nodes[::37] + ["2-0-0", "1-0-0", "3-5-9"]))
    for i, node in enumerate(sample):
        assert spf_canonical(ls.getSpfResult(node, ulm)) == orc.spf(node, ulm), node
        assert ls.spfRuns() == runs0 + i + 1
    # a publication changes the topology: the resident pass is dropped, the
    # next query is a fresh solve of the new graph
    node = "3-1-7"
    i = topo.nodes.index(node)
    one = topo.lsdb.slice(i, i + 1)
    one.dbs["is_overloaded"] = 1
    orc.update_packed(one)
    ls.updateAdjacencyDatabases(one)
    assert ls.allSourcesDigests() is None
    assert spf_canonical(ls.getSpfResult("2-0-0", ulm)) == orc.spf("2-0-0", ulm)
    ls.prefetchAllSources(ulm)  # again, on the patched replicas
    for node in sample[:6]:
        assert spf_canonical(ls.getSpfResult(node, ulm)) == orc.spf(node, ulm), node
    ls.close()


def test_facade_multi_equals_single_device_digests():
    meta, g = golden("fabric_full")
    ls_m = LinkState(devices=[0, 0, 0, 0])
    ls_m.updateAdjacencyDatabases(T.fabric(10000, full=True).lsdb)
    ls_m.prefetchAllSources()
    got = ls_m.allSourcesDigests()
    ls_m.close()
    want = np.zeros(len(got), np.uint64)
    want[g["srcs"].astype(np.int64)] = g["digest"]
    assert np.array_equal(got, want)


def test_null_stream_work_is_ordered_before_execute_on_context_stream():
    """a hipMemset on the legacy null stream, then
    spf_plan_execute(..., stream = NULL) into the same buffers: the execute
    must see the memset done (the context stream is blocking)."""
    meta, g = golden("fabric_full")
    ls, names, csr, cd = _make("fabric_full")
    lib = hiprt._lib
    lib.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
    with SpfEngine(0) as eng:
        eng.load(*csr)
        srcs = g["srcs"][:2048]
        p = eng.plan(srcs)
        d = hiprt.DeviceArray(len(srcs) * eng.pitch, np.uint32)
        nh = hiprt.DeviceArray(max(1, p.nh_words), np.uint32)
        dg = hiprt.DeviceArray(len(srcs), np.uint64)
        for _ in range(3):
            # garbage the outputs on the null stream, no host wait
            assert lib.hipMemsetAsync(C.c_void_p(nh.ptr), 0x5A, nh.nbytes, None) == 0
            assert lib.hipMemsetAsync(C.c_void_p(d.ptr), 0x5A, d.nbytes, None) == 0
            p.execute(d.ptr, nh.ptr)  # NULL stream argument = the context's stream
            p.digest(d.ptr, nh.ptr, dg.ptr)
            eng.check()
            assert np.array_equal(dg.numpy(), g["digest"][:2048])
        p.close()
        for b in (d, nh, dg):
            b.free()
