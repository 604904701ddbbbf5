"""SR_MPLS / KSP2_ED_ECMP route synthesis on the MI355X (SURVEY.md §8(f)
rank 3) against the oracle's restatement of selectBestPathsSpf with
perDestination (Decision.cpp:829-893, 1107-1305) and selectBestPathsKsp2
(:895-1018, pathAInPathB LinkState.h:395-410), row-exact.

Prefixes per scenario: single advertisers with and without prepend labels,
anycast sets (2-3 advertisers, so the k = 2 anycast filter fires), drained
advertisers (maybeFilterDrainedNodes), a min-nexthop threshold.  The product
builds every KSP2 route from ONE batched KSP2 launch (prefetchKthPaths).
"""

import zlib

import numpy as np
import pytest

from adapters import OracleAdapter, ProductAdapter
from oracle import sr_nexthops
from openr_amd import topology as T
from openr_amd.lsdb import PackedLsdb
from openr_amd.spf_solver import PrefixEntry, PrefixState, SpfSolver

pytestmark = pytest.mark.gpu


def labelled(topo, base=50000):
    dbs = topo.lsdb.dbs.copy()
    dbs["node_label"] = base + np.arange(len(dbs), dtype=np.int32)
    return PackedLsdb(topo.lsdb.blob, dbs, topo.lsdb.adjs)


def db_names(lsdb):
    return [bytes(lsdb.blob[o: o + n]).decode()
            for o, n in zip(lsdb.dbs["name_off"], lsdb.dbs["name_len"])]


def scenario(names, me, rng, algo, v4):
    """[(prefix, {advertiser: prependLabel|None}, minNexthop|None)]"""
    out = []
    others = [n for n in names if n != me]
    for i in range(10):
        k = 1 if i < 5 else int(rng.integers(2, 4))
        adv = [others[int(j)] for j in rng.choice(len(others), k, replace=False)]
        if i == 9:
            adv.append(me)  # self-advertised anycast with a prepend label
        pre = {a: (int(rng.integers(100, 200)) if (rng.random() < 0.4 or a == me) else None)
               for a in adv}
        mnh = 99 if i == 4 else None
        pfx = f"10.9.{i}.0/24" if v4 else f"fd00:{i:x}::/64"
        out.append((pfx, pre, mnh))
    return out


def expected(o, me, pre, mnh, lfa, v4, ksp2, area):
    """createRouteForPrefix's filtering around the oracle next hops."""
    mine = o.spf(me)
    reach = {a: p for a, p in pre.items() if a in mine}
    if not reach:
        return None
    best = {a: p for a, p in reach.items() if not o.overloaded(a)} or reach
    if me in best and best[me] is None:
        return None  # self-advertised without prepend label
    rows = sr_nexthops(o.ls, me, best, lfa, v4, ksp2)
    if not rows:
        return None
    if mnh is not None and mnh > len(rows):
        return None
    return rows


def product_rows(nhs):
    return sorted(([n.ifName, n.metric, n.neighborNodeName, n.address.hex(),
                    n.mplsAction.action if n.mplsAction else None,
                    list(n.mplsAction.pushLabels) if n.mplsAction else None] for n in nhs),
                  key=str)


GRAPHS = [
    ("rand0", lambda: T.random_graph(40, 100, 31, max_metric=5, parallel_frac=0.2,
                                     overload_frac=0.1)),
    ("rand1", lambda: T.random_graph(30, 90, 32, max_metric=3, parallel_frac=0.3)),
    ("fabric1000", lambda: T.fabric(1000, full=True)),
    ("wan80", lambda: T.wan(80, 40, seed=5)),
]


@pytest.mark.parametrize("name,make", GRAPHS, ids=[g[0] for g in GRAPHS])
@pytest.mark.parametrize("algo", ["SP_ECMP", "KSP2_ED_ECMP"])
@pytest.mark.parametrize("lfa", [False, True], ids=["sp", "lfa"])
def test_sr_mpls_routes_match_oracle(name, make, algo, lfa):
    topo = make()
    lsdb = labelled(topo)
    o, p = OracleAdapter(), ProductAdapter()
    o.update_packed(lsdb)
    p.update_packed(lsdb)
    names = db_names(lsdb)
    rng = np.random.default_rng(zlib.crc32(f"{name}/{algo}".encode()))
    area = p.ls.getArea()
    n_routes = n_push = 0
    for me in [names[int(i)] for i in rng.choice(len(names), 2, replace=False)]:
        for v4 in (False, True):
            ps = PrefixState()
            sc = scenario(names, me, rng, algo, v4)
            for pfx, pre, mnh in sc:
                for a, lab in pre.items():
                    ps.updatePrefix(a, area, PrefixEntry(pfx, forwardingType="SR_MPLS",
                                                         forwardingAlgorithm=algo,
                                                         prependLabel=lab, minNexthop=mnh))
            db = SpfSolver(me, True, lfa).buildRouteDb(me, {area: p.ls}, ps)
            for pfx, pre, mnh in sc:
                want = expected(o, me, pre, mnh, lfa, v4, algo == "KSP2_ED_ECMP", area)
                got = db.unicastRoutes.get(pfx)
                got_rows = None if got is None else product_rows(got.nexthops)
                if got_rows == []:
                    got_rows = None
                assert got_rows == (None if want is None else sorted(want, key=str)), \
                    (name, me, pfx, pre)
                if got_rows:
                    n_routes += 1
                    n_push += sum(r[4] == "PUSH" for r in got_rows)
    assert n_routes >= 10 and n_push > 0, (n_routes, n_push)  # the cases are not vacuous


def test_ksp2_prefetch_keeps_spf_run_counts():
    """Route build via the batched prefetch counts runSpf like per-pair queries."""
    topo = T.wan(50, 25, seed=9)
    lsdb = labelled(topo)
    a, b = ProductAdapter(), ProductAdapter()
    a.update_packed(lsdb)
    b.update_packed(lsdb)
    names = db_names(lsdb)
    me = names[3]
    b.ls.prefetchKthPaths(me)
    for d in names[:20]:
        for k in (1, 2):
            assert a.kth(me, d, k) == b.kth(me, d, k), (me, d, k)
    assert a.spf_runs() == b.spf_runs()


def test_ksp2_incompatible_forwarding_type_is_skipped():
    """KSP2_ED_ECMP with IP forwarding gets no route (Decision.cpp:905-913)."""
    topo = T.wan(30, 15, seed=4)
    lsdb = labelled(topo)
    p = ProductAdapter()
    p.update_packed(lsdb)
    names = db_names(lsdb)
    area = p.ls.getArea()
    ps = PrefixState()
    ps.updatePrefix(names[5], area, PrefixEntry("fd00:1::/64", forwardingType="IP",
                                                forwardingAlgorithm="KSP2_ED_ECMP"))
    db = SpfSolver(names[0], True, False).buildRouteDb(names[0], {area: p.ls}, ps)
    assert "fd00:1::/64" not in db.unicastRoutes
