"""SpfSolver route computation on the MI355X (spf_routes + openr_amd.spf_solver)
against the oracle's restatement of getMinCostNodes / getNextHopsWithMetric /
getNextHopsThrift (Decision.cpp:1082-1305), which tests/test_oracle_reference.py
pins to DecisionTest's route expectations.

Random multigraphs (parallel links, drained nodes and links) and a fabric:
every node's unicast + node-label routes from several vantage points, with and
without LFA, v4 and v6; anycast destination sets; adjacency-label and POP
routes of buildRouteDb.
"""

import numpy as np
import pytest

from adapters import OracleAdapter, ProductAdapter
from oracle import nexthops
from openr_amd import topology as T
from openr_amd.link_state import LinkState
from openr_amd.spf_solver import SpfSolver

pytestmark = pytest.mark.gpu

GRAPHS = [
    ("fabric_full1000", lambda: T.fabric(1000, full=True)),
    ("wan120", lambda: T.wan(120, 60, seed=8)),
] + [
    (f"rand{seed}", (lambda s: lambda: T.random_graph(
        40, 110, 400 + s, max_metric=6, parallel_frac=0.25, overload_frac=0.1,
        link_overload_frac=0.05))(seed))
    for seed in range(4)
]


def load(topo):
    o, p = OracleAdapter(), ProductAdapter()
    o.update_packed(topo.lsdb)
    p.update_packed(topo.lsdb)
    return o, p


@pytest.mark.parametrize("name,make", GRAPHS, ids=[g[0] for g in GRAPHS])
@pytest.mark.parametrize("lfa", [False, True], ids=["sp", "lfa"])
def test_route_db_matches_oracle(name, make, lfa):
    topo = make()
    o, p = load(topo)
    labels = p.ls.getAdjacencyDatabaseLabels()
    rng = np.random.default_rng(3)
    mes = [topo.nodes[int(i)] for i in rng.choice(len(topo.nodes), 3, replace=False)]
    for me in mes:
        for v4 in (False, True):
            assert p.routes(me, lfa, v4, labels) == o.routes(me, lfa, v4, labels), (me, v4)


@pytest.mark.parametrize("lfa", [False, True], ids=["sp", "lfa"])
def test_anycast_sets_match_oracle(lfa):
    topo = T.random_graph(50, 140, 77, max_metric=4, parallel_frac=0.2, overload_frac=0.05)
    o, p = load(topo)
    rng = np.random.default_rng(9)
    solver = SpfSolver("x", True, lfa)
    names = topo.nodes
    for _ in range(6):
        me = names[int(rng.integers(len(names)))]
        sets = [[names[int(i)] for i in rng.choice(len(names), int(rng.integers(1, 5)),
                                                   replace=False)] for _ in range(12)]
        got = solver.getNextHopsBatch(p.ls, me, sets)
        for s, (mn, nhs) in zip(sets, got):
            want = nexthops(o.ls, me, s, lfa)
            assert mn == want["min"] or (not nhs and not want["nh"])
            rows = sorted(([n.ifName, n.metric, n.neighborNodeName, n.address.hex(), None, None]
                           for n in nhs), key=str)
            assert rows == sorted(want["nh"], key=str), (me, s)


def test_pop_and_adjacency_label_routes():
    topo = T.random_graph(20, 40, 5, parallel_frac=0.3)
    ls = LinkState()
    ls.updateAdjacencyDatabases(topo.lsdb)
    from openr_amd.spf_solver import PrefixState

    me = topo.nodes[3]
    db = SpfSolver(me, True, False).buildRouteDb(me, {ls.getArea(): ls}, PrefixState())
    labels = ls.getAdjacencyDatabaseLabels()
    pop = db.mplsRoutes[labels[me]]
    assert [n.mplsAction.action for n in pop.nexthops] == ["POP_AND_LOOKUP"]
    for link in ls.linksFromNode(me):
        lab = link.getAdjLabelFromNode(me)
        if lab:
            (nh,) = db.mplsRoutes[lab].nexthops
            assert nh.mplsAction.action == "PHP" and nh.ifName == link.getIfaceFromNode(me)
            assert nh.metric == link.getMetricFromNode(me)


def test_no_prefixes_no_node_labels_fresh_solver():
    """A single-area build with nothing to select (no prefixes, every node
    label 0: non-SR mode) on a FRESH solver still returns the adjacency-label
    routes (Decision.cpp:667-698) and static MPLS routes (:700-707); a reused
    solver does not read the previous build's selection."""
    from openr_amd.lsdb import PackedLsdb
    from openr_amd.spf_solver import NextHopThrift, PrefixEntry, PrefixState

    topo = T.grid(4)
    dbs = topo.lsdb.dbs.copy()
    dbs["node_label"] = 0  # non-SR mode: adjacency labels only
    with LinkState() as ls:
        ls.updateAdjacencyDatabases(PackedLsdb(topo.lsdb.blob, dbs, topo.lsdb.adjs))
        assert not any(ls.getAdjacencyDatabaseLabels().values())
        me = topo.nodes[5]
        s = SpfSolver(me, True, False)
        s.updateStaticMplsRoutes({77: [NextHopThrift(bytes(16), None, 0, None, None, None)]})
        db = s.buildRouteDb(me, {ls.getArea(): ls}, PrefixState())
        adj = {l.getAdjLabelFromNode(me) for l in ls.linksFromNode(me)}
        assert not db.unicastRoutes and set(db.mplsRoutes) == adj | {77}
        ps = PrefixState()
        for node in topo.nodes:
            ps.updatePrefix(node, ls.getArea(), PrefixEntry(f"fc00::{topo.nodes.index(node)}/128"))
        assert len(s.buildRouteDb(me, {ls.getArea(): ls}, ps).unicastRoutes) == len(topo.nodes) - 1
        db2 = s.buildRouteDb(me, {ls.getArea(): ls}, PrefixState())
        assert not db2.unicastRoutes and set(db2.mplsRoutes) == adj | {77}


@pytest.mark.parametrize("n", [2, 4, 6, 8])
def test_grid_route_count_and_distances(n):
    """DecisionTest.cpp:4301-4356 (GridTopologyFixture.ShortestPathTest): every
    node's buildRouteDb over the n x n grid (createGrid, :4238-4264: node
    label node + 1, one v6 loopback per node) programs n^2 (n^2 - 1) unicast,
    n^2 * n^2 node-label and 4n (n - 1) adjacency-label routes in total,
    2n^4 + 3n^2 - 4n (:4313), and corner-to-corner / any-pair metrics are the
    Manhattan distances."""
    from openr_amd.spf_solver import PrefixEntry, PrefixState

    topo = T.decision_test_grid(n)
    ps = PrefixState()
    pfx = {}
    for node in range(n * n):
        pfx[node] = f"::ffff:10.1.{node // 256}.{node % 256}/128"  # nodeToPrefixV6
        ps.updatePrefix(str(node), "0", PrefixEntry(pfx[node]))
    with LinkState() as ls:
        ls.updateAdjacencyDatabases(topo.lsdb)
        total, dbs = 0, {}
        for node in range(n * n):
            me = str(node)
            db = SpfSolver(me, False, False).buildRouteDb(me, {ls.getArea(): ls}, ps)
            total += len(db.unicastRoutes) + len(db.mplsRoutes)
            dbs[node] = db
        assert total == 2 * n ** 4 + 3 * n ** 2 - 4 * n

        def grid_distance(a, b):
            return abs(a % n - b % n) + abs(a // n - b // n)

        rng = np.random.default_rng(n)
        pairs = [(0, n * n - 1), (n - 1, n * (n - 1))] + \
            [tuple(int(x) for x in rng.choice(n * n, 2, replace=False)) for _ in range(8)]
        for src, dst in pairs:
            nhs = dbs[src].unicastRoutes[pfx[dst]].nexthops
            assert {h.metric for h in nhs} == {grid_distance(src, dst)}
