"""The C++ SpfSolver (openr_amd/csrc/decision.cpp, include/openr_decision.h)
against the Python restatement of Decision.cpp's route computation
(openr_amd/spf_solver.py, SpfSolver.native = False), which the other route
tests pin to the oracle and to DecisionTest's expectations.

Whole route databases are compared -- unicast routes (next-hop sets,
bestPrefixEntry, bestArea, doNotInstall), MPLS routes, the best-routes cache
and the decision.* counters -- over random multigraphs with drained nodes and
links, one and several areas, IP / SR_MPLS / KSP2_ED_ECMP prefixes, anycast
sets, prepend labels and static MPLS routes, v4 and v6, BGP metric vectors
(tie chains), best-route selection and min-nexthop requirements.
"""

import contextlib

import numpy as np
import pytest

from openr_amd import topology as T
from openr_amd.link_state import LinkState
from openr_amd.lsdb import PackedLsdb
from openr_amd.spf_solver import (MetricEntity, MetricVector, NextHopThrift, MplsAction,
                                  PrefixEntry, PrefixMetrics, PrefixState, SpfSolver)

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def impl(native: bool):
    old = SpfSolver.native
    SpfSolver.native = native
    try:
        yield
    finally:
        SpfSolver.native = old


def canon(db):
    if db is None:
        return None
    uni = {p: (frozenset(r.nexthops), id(r.bestPrefixEntry), r.bestArea, r.doNotInstall)
           for p, r in db.unicastRoutes.items()}
    mpls = {l: frozenset(r.nexthops) for l, r in db.mplsRoutes.items()}
    return uni, mpls


def build_both(me, areas, ps, flags=(True, True), static=None):
    out = []
    for native in (True, False):
        with impl(native):
            s = SpfSolver(me, *flags)
            if static:
                s.updateStaticMplsRoutes(static)
            db = s.buildRouteDb(me, areas, ps)
            cache = {p: (r.success, list(r.allNodeAreas), r.bestNodeArea)
                     for p, r in s.getBestRoutesCache().items()}
            out.append((canon(db), cache, {k: v for k, v in s.counters.items() if v}))
    return out


def labelled(topo, base):
    dbs = topo.lsdb.dbs.copy()
    dbs["node_label"] = base + np.arange(len(dbs), dtype=np.int32)
    return PackedLsdb(topo.lsdb.blob, dbs, topo.lsdb.adjs)


def random_prefixes(ps, names, area, rng, n, tag, bgp=False, ksp2=True):
    for i in range(n):
        adv = [names[int(j)] for j in rng.choice(len(names), int(rng.integers(1, 4)), replace=False)]
        v4 = i % 4 == 3
        pfx = f"10.{tag}.{i // 250}.{i % 250}/32" if v4 else f"fd{tag:02x}:{i:x}::/64"
        ftype = ("IP", "SR_MPLS", "SR_MPLS", "IP")[i % 4]
        falgo = "KSP2_ED_ECMP" if ksp2 and i % 8 == 2 else "SP_ECMP"
        for a in adv:
            pre = int(rng.integers(100, 200)) if (ftype == "SR_MPLS" and rng.random() < 0.3) else None
            mnh = int(rng.integers(1, 4)) if rng.random() < 0.15 else None
            mv = None
            typ = "LOOPBACK"
            if bgp and i % 5 == 0:
                typ = "BGP"
                mv = MetricVector(0, [MetricEntity(1, 9, "WIN_IF_PRESENT", False, (int(rng.integers(1, 3)),)),
                                      MetricEntity(2, 5, "WIN_IF_PRESENT", True, (int(rng.integers(1, 4)),))])
            ps.updatePrefix(a, area, PrefixEntry(
                pfx, type=typ, forwardingType=ftype, forwardingAlgorithm=falgo, prependLabel=pre,
                minNexthop=mnh, mv=mv,
                metrics=PrefixMetrics(int(rng.integers(0, 2)), int(rng.integers(0, 2)),
                                      int(rng.integers(0, 2)))))


GRAPHS = [
    ("rand0", lambda: T.random_graph(30, 80, 61, max_metric=5, parallel_frac=0.2, overload_frac=0.1,
                                     link_overload_frac=0.05)),
    ("rand1", lambda: T.random_graph(40, 110, 62, max_metric=3, parallel_frac=0.3, overload_frac=0.15)),
    ("wan60", lambda: T.wan(60, 30, seed=4)),
    ("fabric1000", lambda: T.fabric(1000, full=True)),
]


@pytest.mark.parametrize("name,make", GRAPHS, ids=[g[0] for g in GRAPHS])
@pytest.mark.parametrize("lfa", [False, True], ids=["sp", "lfa"])
@pytest.mark.parametrize("brs", [False, True], ids=["openr", "best_route"])
def test_native_equals_restatement_one_area(name, make, lfa, brs):
    topo = make()
    with LinkState() as ls:
        ls.updateAdjacencyDatabases(labelled(topo, 70000))
        names = topo.nodes
        rng = np.random.default_rng(11)
        ps = PrefixState()
        random_prefixes(ps, names, ls.getArea(), rng, 40, 1, bgp=not brs)
        static = {300001: [NextHopThrift(bytes(16), "eth9", 0, None, None, None)],
                  150: [NextHopThrift(bytes([1] * 16), None, 0, MplsAction("PUSH", None, (5, 6)),
                                      None, None)]}
        for me in [names[int(i)] for i in rng.choice(len(names), 3, replace=False)]:
            nat, py = build_both(me, {ls.getArea(): ls}, ps, (True, lfa, False, False, brs), static)
            assert nat == py, me


def test_native_equals_restatement_several_areas():
    """Two areas sharing a node set: per-prefix walk, LFA per area, ECMP across
    areas, node labels from both areas (a node present in both).  No
    KSP2_ED_ECMP prefixes: with several areas the reference's
    prefixEntries.at({node, area}) throws for a path's destination in another
    area (Decision.cpp:982), as both implementations do."""
    ta, tb = T.random_graph(25, 60, 71, max_metric=4, parallel_frac=0.2), T.random_graph(
        25, 60, 72, max_metric=4, overload_frac=0.1)
    la, lb = LinkState("A"), LinkState("B")
    with la, lb:
        la.updateAdjacencyDatabases(labelled(ta, 80000))
        lb.updateAdjacencyDatabases(labelled(tb, 80000))
        rng = np.random.default_rng(3)
        ps = PrefixState()
        random_prefixes(ps, ta.nodes, "A", rng, 20, 2, ksp2=False)
        random_prefixes(ps, tb.nodes, "B", rng, 20, 3, ksp2=False)
        for order in (("A", "B"), ("B", "A")):
            areas = {k: {"A": la, "B": lb}[k] for k in order}
            for me in ta.nodes[:4]:
                for lfa in (False, True):
                    nat, py = build_both(me, areas, ps, (True, lfa))
                    assert nat == py, (order, me, lfa)


def test_native_equals_restatement_after_updates():
    """Publications in between builds: link metric change, overload toggles,
    prefix withdrawals and re-advertisements (the PrefixEntries map order after
    erasures), a reused solver."""
    topo = T.random_graph(30, 80, 9, max_metric=5, parallel_frac=0.2)
    lsdb = labelled(topo, 90000)
    from openr_amd.wire import unpack

    dbs = {d.thisNodeName: d for d in unpack(lsdb)}
    with LinkState() as ls:
        ls.updateAdjacencyDatabases(lsdb)
        names = topo.nodes
        rng = np.random.default_rng(4)
        ps = PrefixState()
        random_prefixes(ps, names, ls.getArea(), rng, 30, 4, bgp=True)
        me = names[0]
        solvers = {}
        for native in (True, False):
            with impl(native):
                solvers[native] = SpfSolver(me, True, True)
        for step in range(6):
            victim = dbs[names[1 + step]]
            if step % 2:
                victim.isOverloaded = not victim.isOverloaded
            elif victim.adjacencies:
                victim.adjacencies[0].metric += 3
            ls.updateAdjacencyDatabase(victim)
            for p in list(ps.prefixes())[:3]:
                for na in list(ps.prefixes()[p])[:1]:
                    e = ps.prefixes()[p][na]
                    ps.deletePrefix(na[0], na[1], p)
                    if step % 3 == 0:
                        ps.updatePrefix(na[0], na[1], e)
            got = []
            for native in (True, False):
                with impl(native):
                    s = solvers[native]
                    db = s.buildRouteDb(me, {ls.getArea(): ls}, ps)
                    got.append((canon(db), {p: (r.success, list(r.allNodeAreas), r.bestNodeArea)
                                            for p, r in s.getBestRoutesCache().items()},
                                {k: v for k, v in s.counters.items() if v}))
            assert got[0] == got[1], step


def test_native_no_route_for_absent_node():
    topo = T.grid(4)
    with LinkState() as ls:
        ls.updateAdjacencyDatabases(topo.lsdb)
        assert SpfSolver("nope", True, False).buildRouteDb("nope", {ls.getArea(): ls},
                                                           PrefixState()) is None


def test_native_route_db_counts_match_tables():
    """NativeRouteDb's count accessors (unicastCount / mplsCount /
    nexthopCount: no copy, what the CS-1 bench reads) agree with the
    materialised tables."""
    topo = T.fabric(1000, full=True)
    with LinkState() as ls:
        ls.updateAdjacencyDatabases(labelled(topo, 70000))
        ps = PrefixState()
        random_prefixes(ps, topo.nodes, ls.getArea(), np.random.default_rng(5), 30, 2)
        me = topo.nodes[7]
        with impl(True):
            ndb = SpfSolver(me, True, True).buildRouteDbNative(me, {ls.getArea(): ls}, ps)
        try:
            db = ndb.routeDb()
            assert ndb.nexthopCount() == len(ndb.nexthopRecords()) > 0
            assert ndb.unicastCount() == len(db.unicastRoutes)
            assert ndb.mplsCount() == len(db.mplsRoutes)
        finally:
            ndb.close()
