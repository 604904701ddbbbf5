"""Route selection for every node from a resident all-sources pass
(spf_mplan_route_digests / spf_mplan_routes, include/openr_spf.h): what
Decision::getDecisionRouteDb(node) for every node (Decision.cpp:1480-1500,
CS-2) computes, with no SPF per node.

* every node's digest over every destination set (single advertisers and
  anycast sets, SP and LFA) against the oracle's restatement of
  getMinCostNodes / getNextHopsWithMetric / getNextHopsThrift
  (oracle/spf_oracle.cpp orc_ls_route_digests), on random multigraphs with
  drained nodes and links, a WAN and a fabric, members of 1, 2 and 3 on one
  GPU;
* every node's materialised route database (spf_mplan_route_records) read
  back and reduced with the same digest, against the oracle's;
* SpfSolver.buildRouteDb answered from the resident pass (spf_mplan_routes)
  equals the one-node plan path (spf_routes), before and after a
  publication drops the pass.
"""

import numpy as np
import pytest

from helpers import route_db_digest
from oracle import NameTable, OracleLinkState, route_digests
from openr_amd import topology as T
from openr_amd.link_state import LinkState
from openr_amd.spf_solver import PrefixEntry, PrefixState, SpfSolver

pytestmark = pytest.mark.gpu

GRAPHS = [
    ("rand0", lambda: T.random_graph(60, 170, 12, max_metric=6, parallel_frac=0.25,
                                     overload_frac=0.1, link_overload_frac=0.05)),
    ("rand1", lambda: T.random_graph(45, 90, 7, max_metric=3, parallel_frac=0.1,
                                     overload_frac=0.2)),
    ("wan120", lambda: T.wan(120, 60, seed=8)),
    ("fabric1000", lambda: T.fabric(1000, full=True)),
]


def sets_for(n, rng):
    """Every node alone (loopbacks, node labels), then anycast sets."""
    sets = [[v] for v in range(n)]
    for _ in range(40):
        sets.append(sorted(int(x) for x in rng.choice(n, int(rng.integers(2, 5)), replace=False)))
    ptr = np.zeros(len(sets) + 1, np.uint32)
    ptr[1:] = np.cumsum([len(s) for s in sets])
    return ptr, np.concatenate([np.asarray(s, np.uint32) for s in sets])


@pytest.mark.parametrize("name,make", GRAPHS, ids=[g[0] for g in GRAPHS])
@pytest.mark.parametrize("members", [1, 2, 3])
@pytest.mark.parametrize("lfa", [False, True], ids=["sp", "lfa"])
def test_every_node_route_digests_match_oracle(name, make, members, lfa):
    topo = make()
    with LinkState(devices=[0] * members) as ls:
        ls.updateAdjacencyDatabases(topo.lsdb)
        ls.prefetchAllSources()
        names = list(ls.flatten()[0])
        ptr, nodes = sets_for(len(names), np.random.default_rng(len(names)))
        got, ms = ls.allSourcesRouteDigests(ptr, nodes, lfa)
        assert ms >= 0
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    want = route_digests(orc, NameTable(names), np.arange(len(names)), ptr, nodes, lfa)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} nodes differ, first {[names[i] for i in bad[:5]]}"
    assert np.count_nonzero(want) > len(names) // 2  # routes exist


@pytest.mark.parametrize("name,make", GRAPHS, ids=[g[0] for g in GRAPHS])
@pytest.mark.parametrize("members", [1, 3])
@pytest.mark.parametrize("lfa", [False, True], ids=["sp", "lfa"])
def test_every_node_materialised_route_db_matches_oracle(name, make, members, lfa):
    """spf_mplan_route_records: every node's database, read back and reduced
    with the digest formula, equals the oracle's digest; the record count
    is the sum of the headers' counts; a second call (regions sized from the
    first) gives the same databases."""
    topo = make()
    with LinkState(devices=[0] * members) as ls:
        ls.updateAdjacencyDatabases(topo.lsdb)
        ls.prefetchAllSources()
        names, _rp, _col, _met, lid = ls.flatten()[:5]
        names = list(names)
        lh = ls.linkValueHashes()
        ptr, nodes = sets_for(len(names), np.random.default_rng(len(names)))
        dig_kernel, _ = ls.allSourcesRouteDigests(ptr, nodes, lfa)
        for call in range(2):
            total, ms = ls.allSourcesRouteRecords(ptr, nodes, lfa)
            assert ms >= 0
            got = np.zeros(len(names), np.uint64)
            seen = 0
            for t in range(len(names)):
                hdr, rec = ls.allSourcesRouteDb(t)
                assert len(hdr) == len(ptr) - 1
                assert int((hdr >> np.uint64(32)).sum()) == len(rec)
                seen += len(rec)
                got[t] = route_db_digest(hdr, rec, lid, lh)
            assert seen == total
            if not lfa:  # (keyed alike only without LFA)
                assert np.array_equal(got, dig_kernel), f"call {call}: records differ from the digest kernel"
            if call == 0:
                first = got.copy()
            else:
                assert np.array_equal(got, first)
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    want = route_digests(orc, NameTable(names), np.arange(len(names)), ptr, nodes, lfa, kept_min=True)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} nodes differ, first {[names[i] for i in bad[:5]]}"


@pytest.mark.parametrize("lfa", [False, True], ids=["sp", "lfa"])
def test_route_db_from_resident_pass_equals_plan_path(lfa):
    topo = T.random_graph(50, 140, 77, max_metric=4, parallel_frac=0.2, overload_frac=0.05)
    ps = PrefixState()
    rng = np.random.default_rng(2)
    names = topo.nodes
    for i, node in enumerate(names):
        ps.updatePrefix(node, "0", PrefixEntry(f"fd00:{i:x}::/64"))
    for i in range(10):  # anycast
        for a in rng.choice(len(names), 3, replace=False):
            ps.updatePrefix(names[int(a)], "0", PrefixEntry(f"fd01:{i:x}::/64"))

    def rows(db):
        return {p: sorted((n.ifName, n.metric, n.neighborNodeName) for n in r.nexthops)
                for p, r in db.unicastRoutes.items()}

    with LinkState(devices=[0, 0]) as res, LinkState() as one:
        for ls in (res, one):
            ls.updateAdjacencyDatabases(topo.lsdb)
        res.prefetchAllSources()
        for me in [names[int(i)] for i in rng.choice(len(names), 5, replace=False)]:
            a = SpfSolver(me, True, lfa).buildRouteDb(me, {"0": res}, ps)
            b = SpfSolver(me, True, lfa).buildRouteDb(me, {"0": one}, ps)
            assert rows(a) == rows(b), me
            assert {l: sorted((n.ifName, n.metric) for n in r.nexthops) for l, r in a.mplsRoutes.items()} \
                == {l: sorted((n.ifName, n.metric) for n in r.nexthops) for l, r in b.mplsRoutes.items()}
        # a publication drops the pass: the plan path answers, same routes
        from openr_amd.wire import unpack

        db0 = unpack(topo.lsdb)[0]
        db0.isOverloaded = not db0.isOverloaded
        res.updateAdjacencyDatabase(db0)
        one.updateAdjacencyDatabase(db0)
        me = names[3]
        assert rows(SpfSolver(me, True, lfa).buildRouteDb(me, {"0": res}, ps)) == \
            rows(SpfSolver(me, True, lfa).buildRouteDb(me, {"0": one}, ps))


@pytest.mark.parametrize("v4,bgp_dry", [(False, False), (True, True)], ids=["v6", "v4_bgpdry"])
def test_single_advertiser_fast_path_equals_generic_walk(v4, bgp_dry):
    """buildRouteDb's one-advertiser shortcut (no selection walk, no drained
    filter) yields the same route DB, best-routes cache and counters as the
    generic walk: loopbacks, v4 prefixes, a BGP prefix with a metric vector and
    one without, SR_MPLS SP_ECMP / KSP2 prefixes, self-advertised prefixes with
    and without a prepend label, a drained advertiser, anycast sets."""
    from openr_amd.spf_solver import MetricEntity, MetricVector

    topo = T.random_graph(40, 110, 5, max_metric=4, parallel_frac=0.2, overload_frac=0.1)
    names = topo.nodes
    ps = PrefixState()
    mv = MetricVector(1, [MetricEntity(1, 10, metric=(5,))])
    for i, node in enumerate(names):
        ps.updatePrefix(node, "0", PrefixEntry(f"fd00:{i:x}::/64"))
        ps.updatePrefix(node, "0", PrefixEntry(f"10.{i}.0.0/16"))
        if i % 5 == 0:
            ps.updatePrefix(node, "0", PrefixEntry(f"fd02:{i:x}::/64", type="BGP", mv=mv))
        if i % 7 == 0:
            ps.updatePrefix(node, "0", PrefixEntry(f"fd03:{i:x}::/64", type="BGP"))
        if i % 4 == 0:
            ps.updatePrefix(node, "0", PrefixEntry(f"fd04:{i:x}::/64", forwardingType="SR_MPLS"))
        if i % 6 == 0:
            ps.updatePrefix(node, "0", PrefixEntry(f"fd05:{i:x}::/64", forwardingType="SR_MPLS",
                                                   forwardingAlgorithm="KSP2_ED_ECMP"))
        if i % 3 == 0:
            ps.updatePrefix(node, "0", PrefixEntry(f"fd06:{i:x}::/64", prependLabel=70000 + i,
                                                   minNexthop=1))
    for k in range(6):  # anycast (the generic walk on both sides)
        for a in (k, k + 11, k + 23):
            ps.updatePrefix(names[a], "0", PrefixEntry(f"fd01:{k:x}::/64"))

    def dump(solver, db):
        uni = {p: (sorted(db.unicastRoutes[p].nexthops, key=repr), db.unicastRoutes[p].bestArea,
                   db.unicastRoutes[p].bestPrefixEntry, db.unicastRoutes[p].doNotInstall)
               for p in db.unicastRoutes}
        mpls = {l: sorted(r.nexthops, key=repr) for l, r in db.mplsRoutes.items()}
        return uni, mpls, solver.getBestRoutesCache(), dict(solver.counters)

    with LinkState() as ls:
        ls.updateAdjacencyDatabases(topo.lsdb)
        for me in (names[0], names[3], names[17]):
            out = []
            for fast in (True, False):
                SpfSolver._single_fast = fast
                try:
                    sol = SpfSolver(me, v4, True, bgpDryRun=bgp_dry)
                    out.append(dump(sol, sol.buildRouteDb(me, {"0": ls}, ps)))
                finally:
                    SpfSolver._single_fast = True
            assert out[0] == out[1], me
            assert out[0][0]  # routes exist


@pytest.mark.parametrize("lfa", [False, True], ids=["sp", "lfa"])
def test_route_sums_u32_and_u64_paths_agree(lfa, monkeypatch):
    """The many-me route kernel runs its sums in u32 when the host proves no
    finite sum reaches kInf (routes.hip, route_quads_kernel<MODE, Dist>):
    digests and materialised records equal the u64 kernel's (SPF_ROUTE_U64=1)
    on a small-metric graph, and a graph whose metrics rule u32 out (up to
    2^26 per link: 2 x max metric x (N - 1) passes 2^32 while the distances
    themselves still fit u32) takes the u64 kernel and matches the oracle."""
    topo = T.random_graph(60, 170, 12, max_metric=6, parallel_frac=0.25, overload_frac=0.1,
                          link_overload_frac=0.05)
    with LinkState(devices=[0]) as ls:
        ls.updateAdjacencyDatabases(topo.lsdb)
        ls.prefetchAllSources()
        names = list(ls.flatten()[0])
        ptr, nodes = sets_for(len(names), np.random.default_rng(3))
        d32, _ = ls.allSourcesRouteDigests(ptr, nodes, lfa)
        ls.allSourcesRouteRecords(ptr, nodes, lfa)
        r32 = [ls.allSourcesRouteDb(t) for t in range(len(names))]
        monkeypatch.setenv("SPF_ROUTE_U64", "1")
        d64, _ = ls.allSourcesRouteDigests(ptr, nodes, lfa)
        ls.allSourcesRouteRecords(ptr, nodes, lfa)
        r64 = [ls.allSourcesRouteDb(t) for t in range(len(names))]
        monkeypatch.delenv("SPF_ROUTE_U64")
    assert np.array_equal(d32, d64)
    for (h32, c32), (h64, c64) in zip(r32, r64):
        assert np.array_equal(h32, h64) and np.array_equal(c32, c64)
    wide = T.random_graph(50, 140, 9, max_metric=1 << 26, parallel_frac=0.2, overload_frac=0.1)
    with LinkState(devices=[0]) as ls:
        ls.updateAdjacencyDatabases(wide.lsdb)
        ls.prefetchAllSources()
        names = list(ls.flatten()[0])
        ptr, nodes = sets_for(len(names), np.random.default_rng(4))
        got, _ = ls.allSourcesRouteDigests(ptr, nodes, lfa)
    orc = OracleLinkState()
    orc.update_packed(wide.lsdb)
    want = route_digests(orc, NameTable(names), np.arange(len(names)), ptr, nodes, lfa)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("members", [1, 2])
def test_route_lfa_u8_row_loads_match_oracle(members, monkeypatch):
    """With unit metrics and every member's BFS rows below depth 254, the
    many-me route kernel's LFA reads the members' u8 row copies (4 bytes per
    4 destinations, multi.cpp route_prepare): every node's digests and
    materialised databases equal the u32 loads' (SPF_ROUTE_U8=0) and the
    oracle's.  (Team plans keep no u8 rows: SPF_MSBFS_TEAM=0 gives every
    member the one-workgroup-per-batch BFS that writes them.)"""
    monkeypatch.setenv("SPF_MSBFS_TEAM", "0")
    topo = T.fabric(1000, full=True)
    out = {}
    for u8 in ("1", "0"):
        monkeypatch.setenv("SPF_ROUTE_U8", u8)
        with LinkState(devices=[0] * members) as ls:
            ls.updateAdjacencyDatabases(topo.lsdb)
            ls.prefetchAllSources()
            names, _rp, _col, _met, lid = ls.flatten()[:5]
            names = list(names)
            lh = ls.linkValueHashes()
            ptr, nodes = sets_for(len(names), np.random.default_rng(9))
            dig, _ = ls.allSourcesRouteDigests(ptr, nodes, True)
            ls.allSourcesRouteRecords(ptr, nodes, True)
            recs = np.array([route_db_digest(*ls.allSourcesRouteDb(t), lid, lh) for t in range(len(names))],
                            np.uint64)
        out[u8] = (dig, recs)
    assert np.array_equal(out["1"][0], out["0"][0])
    assert np.array_equal(out["1"][1], out["0"][1])
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    want = route_digests(orc, NameTable(names), np.arange(len(names)), ptr, nodes, True)
    assert np.array_equal(out["1"][0], want)
    want_min = route_digests(orc, NameTable(names), np.arange(len(names)), ptr, nodes, True, kept_min=True)
    assert np.array_equal(out["1"][1], want_min)
