"""SpfSolver with several areas, enable_best_route_selection and BGP metric
vectors on the MI355X engine, transcribed from the reference's DecisionTest:

  * Decision.BestRouteSelection          DecisionTest.cpp:1070-1203
  * BGPRedistribution.BasicOperation     DecisionTest.cpp:715-905
  * BGPRedistribution.IgpMetric          DecisionTest.cpp:907-1068
  * MultiAreaBestPathCalculation         DecisionTest.cpp:4930-5050 (the
    fixture's publications become one LinkState per area; Decision's
    getDecisionRouteDb(node) = buildRouteDb(node, areaLinkStates, prefixState))
  * PrefixWithMixedTypeRoutes            DecisionTest.cpp:6412-6478 (the
    decision.skipped_unicast_route counter)

plus a cross-check of the several-area walk against the batched one-area
kernel path (same routes on random multigraphs, SP and LFA, SR prefixes).
"""

import copy

import numpy as np
import pytest

from openr_amd import topology as T
from openr_amd.link_state import LinkState
from openr_amd.lsdb import create_adj_db, create_adjacency
from openr_amd.spf_solver import (MetricEntity, MetricVector, MplsAction, PrefixEntry,
                                  PrefixMetrics, PrefixState, SpfSolver)

pytestmark = pytest.mark.gpu

K = "0"  # kDefaultArea
# DecisionTest.cpp:47-86
adj12 = create_adjacency("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 10, 100002)
adj13 = create_adjacency("3", "1/3", "3/1", "fe80::3", "192.168.0.3", 10, 100003)
adj21 = create_adjacency("1", "2/1", "1/2", "fe80::1", "192.168.0.1", 10, 100001)
adj24 = create_adjacency("4", "2/4", "4/2", "fe80::4", "192.168.0.4", 10, 100004)
adj31 = create_adjacency("1", "3/1", "1/3", "fe80::1", "192.168.0.1", 10, 100001)
adj34 = create_adjacency("4", "3/4", "4/3", "fe80::4", "192.168.0.4", 10, 100004)
adj42 = create_adjacency("2", "4/2", "2/4", "fe80::2", "192.168.0.2", 10, 100002)
adj43 = create_adjacency("3", "4/3", "3/4", "fe80::3", "192.168.0.3", 10, 100003)
addr1, addr2, addr3, addr4 = ("::ffff:10.1.1.1/128", "::ffff:10.2.2.2/128",
                              "::ffff:10.3.3.3/128", "::ffff:10.4.4.4/128")


def nh(adj, metric, area=K, action=None):
    """createNextHopFromAdj (DecisionTest.cpp:202-215) as a comparable row."""
    return (adj.ifName, metric, adj.otherNodeName, area, action)


def rows(nhs):
    return {(n.ifName, n.metric, n.neighborNodeName, n.area, n.mplsAction) for n in nhs}


def adj_db(node, adjs, label, area=K):
    """createAdjDb with copies of the adjacencies (thrift structs are values
    in the reference; the tests below edit a database's adjacencies)."""
    return create_adj_db(node, [copy.deepcopy(a) for a in adjs], label, area=area)


def one_area(dbs, area=K):
    ls = LinkState(area)
    for db in dbs:
        ls.updateAdjacencyDatabase(db)
    return ls


def test_best_route_selection():
    """DecisionTest.cpp:1070-1203."""
    solver = SpfSolver("1", False, False, False, False, True)
    ls = one_area([adj_db("1", [adj12, adj13], 1), adj_db("2", [adj21], 2),
                   adj_db("3", [adj31], 3)])
    areas = {K: ls}
    ps = PrefixState()
    ps.updatePrefix("2", K, PrefixEntry(addr1, type="DEFAULT", metrics=PrefixMetrics(200, 0, 0)))
    ps.updatePrefix("3", K, PrefixEntry(addr1, type="DEFAULT", metrics=PrefixMetrics(200, 0, 0)))
    assert solver.getBestRoutesCache() == {}
    # case 1: ECMP towards {2, 3}
    db = solver.buildRouteDb("1", areas, ps)
    assert list(db.unicastRoutes) == [addr1]
    assert rows(db.unicastRoutes[addr1].nexthops) == {nh(adj12, 10), nh(adj13, 10)}
    best = solver.getBestRoutesCache()[addr1]
    assert best.allNodeAreas == [("2", K), ("3", K)] and best.bestNodeArea[0] == "2"
    # case 2: node 2 preferred by its prefix metrics
    ps.updatePrefix("2", K, PrefixEntry(addr1, type="DEFAULT", metrics=PrefixMetrics(200, 100, 0)))
    db = solver.buildRouteDb("1", areas, ps)
    assert rows(db.unicastRoutes[addr1].nexthops) == {nh(adj12, 10)}
    best = solver.getBestRoutesCache()[addr1]
    assert best.allNodeAreas == [("2", K)] and best.bestNodeArea[0] == "2"
    # case 3: the best entry's forwarding type (SR_MPLS) decides; from node 3
    ps.updatePrefix("2", K, PrefixEntry(addr1, type="DEFAULT", forwardingType="SR_MPLS",
                                        metrics=PrefixMetrics(200, 100, 0)))
    db = solver.buildRouteDb("3", areas, ps)
    assert list(db.unicastRoutes) == [addr1]
    assert rows(db.unicastRoutes[addr1].nexthops) == {
        nh(adj31, 20, action=MplsAction("PUSH", None, (2,)))}
    # the several-area walk agrees with the one-area kernel path
    assert rows(SpfSolver("3", False, False, False, False, True).buildRouteDb(
        "3", areas, ps, _generic=True).unicastRoutes[addr1].nexthops) == \
        rows(db.unicastRoutes[addr1].nexthops)


def _mv(tie_last=False, last=None):
    n = 5
    m = [MetricEntity(i, i, "WIN_IF_PRESENT", tie_last and i == n - 1, (i,)) for i in range(n)]
    if last is not None:
        m[n - 1].metric = (last,)
    return MetricVector(0, m)


@pytest.mark.parametrize("generic", [False, True], ids=["kernel", "walk"])
def test_bgp_redistribution_basic(generic):
    """DecisionTest.cpp:715-905 (node labels 0: no MPLS routes)."""
    solver = SpfSolver("1", False, False)
    ls = one_area([adj_db("1", [adj12, adj13], 0), adj_db("2", [adj21], 0),
                   adj_db("3", [adj31], 0)])
    areas = {K: ls}
    ps = PrefixState()
    ps.updatePrefix("1", K, PrefixEntry(addr1))  # prefixDb1
    ps.updatePrefix("2", K, PrefixEntry(addr2))  # prefixDb2
    bgp1 = PrefixEntry(addr3, type="BGP", mv=_mv(), data=b"data1")
    ps.updatePrefix("1", K, bgp1)

    def build(me):
        return solver.buildRouteDb(me, areas, ps, _generic=generic)

    db = build("2")
    assert len(db.unicastRoutes) == 2
    r = db.unicastRoutes[addr3]
    assert rows(r.nexthops) == {nh(adj21, 10)} and r.prefixType == "BGP" and r.data == b"data1"
    assert r.doNotInstall is False
    # node 2 advertises the same metric vector: no best path, no BGP route
    bgp2 = PrefixEntry(addr3, type="BGP", mv=_mv(), data=b"data2")
    ps.updatePrefix("2", K, bgp2)
    assert len(build("1").unicastRoutes) == 1
    # node 2's last metric one lower: back to node 1's (thrift entries are
    # values: the changed entry is published again, as the reference test does)
    bgp2.mv.metrics[-1].metric = (bgp2.mv.metrics[-1].metric[0] - 1,)
    ps.updatePrefix("2", K, bgp2)
    db = build("2")
    assert len(db.unicastRoutes) == 2 and db.unicastRoutes[addr3].data == b"data1"
    assert rows(db.unicastRoutes[addr3].nexthops) == {nh(adj21, 10)}
    # node 2 better
    bgp2.mv.metrics[-1].metric = (bgp2.mv.metrics[-1].metric[0] + 2,)
    ps.updatePrefix("2", K, bgp2)
    db = build("1")
    assert len(db.unicastRoutes) == 2 and db.unicastRoutes[addr3].data == b"data2"
    assert rows(db.unicastRoutes[addr3].nexthops) == {nh(adj12, 10)}
    # a tie-breaker metric: multipath; nodes 1 and 2 program no BGP route
    bgp1.mv.metrics[-1].isBestPathTieBreaker = True
    bgp2.mv.metrics[-1].isBestPathTieBreaker = True
    ps.updatePrefix("1", K, bgp1)
    ps.updatePrefix("2", K, bgp2)
    assert len(build("1").unicastRoutes) == 1
    db = build("3")
    assert len(db.unicastRoutes) == 3
    r = db.unicastRoutes[addr3]
    assert r.data == b"data2" and rows(r.nexthops) == {nh(adj31, 10)}
    # disconnect: every node considers its own BGP route best
    ls.updateAdjacencyDatabase(adj_db("1", [], 0))
    for me in ("1", "2"):
        assert addr3 not in build(me).unicastRoutes


@pytest.mark.parametrize("generic", [False, True], ids=["kernel", "walk"])
def test_bgp_redistribution_igp_metric(generic):
    """DecisionTest.cpp:907-1068."""
    solver = SpfSolver("1", False, False, False, False)
    db1 = adj_db("1", [adj12, adj13], 0)
    ls = one_area([db1, adj_db("2", [adj21], 0), adj_db("3", [adj31], 0)])
    areas = {K: ls}
    ps = PrefixState()
    ps.updatePrefix("2", K, PrefixEntry(addr2))
    ps.updatePrefix("2", K, PrefixEntry(addr1, type="BGP", mv=_mv(tie_last=True), data=b"data1"))
    ps.updatePrefix("3", K, PrefixEntry(addr3))
    ps.updatePrefix("3", K, PrefixEntry(addr1, type="BGP", mv=_mv(tie_last=True, last=100),
                                        data=b"data1"))

    def route1():
        db = solver.buildRouteDb("1", areas, ps, _generic=generic)
        return len(db.unicastRoutes), rows(db.unicastRoutes[addr1].nexthops)

    assert route1() == (3, {nh(adj12, 10), nh(adj13, 10)})
    db1.adjacencies[1].metric = 20  # towards node 3
    ls.updateAdjacencyDatabase(db1)
    assert route1() == (3, {nh(adj12, 10)})
    db1.adjacencies[0].isOverloaded = True  # link towards node 2 drained
    ls.updateAdjacencyDatabase(db1)
    assert route1() == (2, {nh(adj13, 20)})
    db1.adjacencies[0].metric = 20
    ls.updateAdjacencyDatabase(db1)
    assert route1() == (2, {nh(adj13, 20)})
    db1.adjacencies[0].isOverloaded = False
    ls.updateAdjacencyDatabase(db1)
    assert route1() == (3, {nh(adj12, 20), nh(adj13, 20)})


def test_multi_area_best_path_calculation():
    """DecisionTest.cpp:4930-5050.  Area A: 1-2-4; area B: 1-3-4."""
    A, B = "A", "B"
    la = one_area([adj_db("1", [adj12], 1, area=A), adj_db("2", [adj21, adj24], 2, area=A),
                   adj_db("4", [create_adjacency("2", "4/2", "2/4", "fe80::2", "192.168.0.2", 10,
                                                        100002)], 4, area=A)], A)
    lb = one_area([adj_db("1", [adj13], 1, area=B), adj_db("3", [adj31, adj34], 3, area=B),
                   adj_db("4", [adj43], 4, area=B)], B)
    areas = {A: la, B: lb}
    ps = PrefixState()
    for node, area, pfx in (("1", A, addr1), ("2", A, addr2), ("3", B, addr3), ("4", B, addr4)):
        ps.updatePrefix(node, area, PrefixEntry(pfx))

    def routes(me):
        db = SpfSolver(me, False, False).buildRouteDb(me, areas, ps)
        return {p: rows(r.nexthops) for p, r in db.unicastRoutes.items()}

    assert routes("1") == {addr2: {nh(adj12, 10, A)}, addr3: {nh(adj13, 10, B)},
                           addr4: {nh(adj12, 20, A), nh(adj13, 20, B)}}
    assert routes("2") == {addr1: {nh(adj21, 10, A)}}
    assert routes("3") == {addr4: {nh(adj34, 10, B)}}
    assert routes("4") == {addr2: {nh(adj42, 10, A)}, addr3: {nh(adj43, 10, B)},
                           addr1: {nh(adj42, 20, A), nh(adj43, 20, B)}}
    # "1" also originates addr1 into B
    ps.updatePrefix("1", B, PrefixEntry(addr1))
    assert routes("3")[addr1] == {nh(adj31, 10, B)}
    assert routes("4")[addr1] == {nh(adj43, 20, B), nh(adj42, 20, A)}


@pytest.mark.parametrize("brs", [False, True], ids=["off", "on"])
def test_prefix_with_mixed_type_routes(brs):
    """DecisionTest.cpp:6412-6478: a prefix advertised as BGP (empty metric
    vector) and as RIB is skipped unless best-route selection is on."""
    ls = one_area([adj_db("1", [adj12, adj13], 1), adj_db("2", [adj21], 2),
                   adj_db("3", [adj31], 3)])
    ps = PrefixState()
    for node, a6, a4 in (("2", addr2, "10.2.2.2/32"), ("3", addr3, "10.3.3.3/32")):
        ps.updatePrefix(node, K, PrefixEntry(a6))
        ps.updatePrefix(node, K, PrefixEntry(a4))
    ps.updatePrefix("2", K, PrefixEntry("10.1.0.0/16", type="BGP", mv=MetricVector(),
                                        data=b"data=10.1.0.0/16"))
    ps.updatePrefix("3", K, PrefixEntry("10.1.0.0/16", type="RIB"))
    solver = SpfSolver("1", True, False, False, False, brs)
    db = solver.buildRouteDb("1", {K: ls}, ps)
    assert solver.counters.get("decision.skipped_unicast_route", 0) == (0 if brs else 1)
    assert ("10.1.0.0/16" in db.unicastRoutes) == brs


GRAPHS = [
    ("rand0", lambda: T.random_graph(30, 80, 61, max_metric=5, parallel_frac=0.2,
                                     overload_frac=0.1, link_overload_frac=0.05)),
    ("wan60", lambda: T.wan(60, 30, seed=4)),
]


@pytest.mark.parametrize("name,make", GRAPHS, ids=[g[0] for g in GRAPHS])
@pytest.mark.parametrize("lfa", [False, True], ids=["sp", "lfa"])
def test_walk_equals_kernel_path_one_area(name, make, lfa):
    """The several-area walk (Decision.cpp's per-prefix code) and the batched
    one-area kernel path build identical route databases: IP and SR_MPLS
    (SP_ECMP / KSP2_ED_ECMP) prefixes, anycast sets with drained advertisers,
    prepend labels, node labels."""
    from openr_amd.lsdb import PackedLsdb

    topo = make()
    dbs = topo.lsdb.dbs.copy()
    dbs["node_label"] = 70000 + np.arange(len(dbs), dtype=np.int32)
    lsdb = PackedLsdb(topo.lsdb.blob, dbs, topo.lsdb.adjs)
    ls = LinkState()
    ls.updateAdjacencyDatabases(lsdb)
    names = topo.nodes
    rng = np.random.default_rng(5)
    ps = PrefixState()
    for i in range(24):
        adv = [names[int(j)] for j in rng.choice(len(names), int(rng.integers(1, 4)), replace=False)]
        ftype = ("IP", "SR_MPLS", "SR_MPLS")[i % 3]
        falgo = "KSP2_ED_ECMP" if i % 3 == 2 else "SP_ECMP"
        for a in adv:
            pre = int(rng.integers(100, 200)) if (ftype == "SR_MPLS" and rng.random() < 0.3) else None
            ps.updatePrefix(a, ls.getArea(), PrefixEntry(f"fd00:{i:x}::/64", forwardingType=ftype,
                                                          forwardingAlgorithm=falgo, prependLabel=pre))
    for me in [names[int(i)] for i in rng.choice(len(names), 3, replace=False)]:
        k = SpfSolver(me, True, lfa).buildRouteDb(me, {ls.getArea(): ls}, ps)
        w = SpfSolver(me, True, lfa).buildRouteDb(me, {ls.getArea(): ls}, ps, _generic=True)
        assert {p: rows(r.nexthops) for p, r in k.unicastRoutes.items()} == \
            {p: rows(r.nexthops) for p, r in w.unicastRoutes.items()}, me
        assert {l: rows(r.nexthops) for l, r in k.mplsRoutes.items()} == \
            {l: rows(r.nexthops) for l, r in w.mplsRoutes.items()}, me
