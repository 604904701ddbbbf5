"""In-place graph patches on the MI355X (spf_graph_set_overload /
spf_graph_set_metric) against the oracle run on the
modified LSDB, bit-exact.

The reference re-runs updateAdjacencyDatabase (LinkState.cpp:564-719) for a
publication that drains a node or changes a metric and recomputes from
scratch; here the loaded CSR is patched and an existing all-sources plan
re-derives its state on the next execute.  Also: the LinkState facade takes
the patch path for overload flips (BM_DecisionFabric's per-iteration
perturbation, RoutingBenchmarkUtils.cpp:453-479) and metric changes, and its
results match the oracle facade after each update.
"""

import numpy as np
import pytest

from oracle import OracleLinkState
from openr_amd import topology as T
from openr_amd.engine import SpfEngine, graph_from_lsdb
from openr_amd.lsdb import PackedLsdb

pytestmark = pytest.mark.gpu

U32_INF = np.uint32(0xFFFFFFFF)


def modified(lsdb: PackedLsdb, drain=(), undrain=(), metric=None) -> PackedLsdb:
    dbs = lsdb.dbs.copy()
    adjs = lsdb.adjs.copy()
    for i in drain:
        dbs["is_overloaded"][i] = 1
    for i in undrain:
        dbs["is_overloaded"][i] = 0
    if metric is not None:
        idx, vals = metric
        adjs["metric"][idx] = vals
    return PackedLsdb(lsdb.blob, dbs, adjs)


def check(names, eng, plan, lsdb, hop):
    res = plan.execute_host()
    orc = OracleLinkState()
    orc.update_packed(lsdb)
    srcs = list(range(len(names)))
    dist, mats = orc.dense(names, srcs, ulm=not hop)
    exp = np.where(dist == np.iinfo(np.uint64).max, U32_INF, dist).astype(np.uint32)
    assert np.array_equal(res.dist, exp), "distance mismatch"
    for i, s in enumerate(srcs):
        k = int(res.words[i])
        assert np.array_equal(res.nh_matrix(i), mats[i][:k]), f"next hops of {names[s]}"


GRAPHS = [
    ("fabric_full1000", lambda: T.fabric(1000, full=True), True),
    ("grid12", lambda: T.grid(12), True),
    ("rand_w", lambda: T.random_graph(80, 220, 5, max_metric=7, parallel_frac=0.25,
                                      overload_frac=0.1), False),
]


@pytest.mark.parametrize("name,make,hop", GRAPHS, ids=[g[0] for g in GRAPHS])
def test_overload_patch_matches_reload(name, make, hop):
    topo = make()
    names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
    eng = SpfEngine(0)
    eng.load(rp, col, met, lid, ovl)
    plan = eng.plan(list(range(len(names))), hop=hop)
    check(names, eng, plan, topo.lsdb, hop)
    rng = np.random.default_rng(11)
    # drain a few nodes, then undrain one of them and drain another
    db_names = [bytes(topo.lsdb.blob[o: o + n]).decode()
                for o, n in zip(topo.lsdb.dbs["name_off"], topo.lsdb.dbs["name_len"])]
    picks = [int(x) for x in rng.choice(len(db_names), 4, replace=False)]
    cur = topo.lsdb
    epoch = eng.epoch
    cur = modified(cur, drain=picks[:3])
    eng.set_overload([names.index(db_names[i]) for i in picks[:3]], [1, 1, 1])
    assert eng.epoch > epoch
    check(names, eng, plan, cur, hop)
    cur = modified(cur, drain=picks[3:], undrain=picks[:1])
    eng.set_overload([names.index(db_names[picks[0]]), names.index(db_names[picks[3]])], [0, 1])
    check(names, eng, plan, cur, hop)


def test_metric_patch_matches_reload():
    topo = T.random_graph(90, 260, 21, max_metric=9, parallel_frac=0.3, overload_frac=0.05)
    names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
    eng = SpfEngine(0)
    eng.load(rp, col, met, lid, ovl)
    plan = eng.plan(list(range(len(names))), hop=False)
    check(names, eng, plan, topo.lsdb, False)
    rng = np.random.default_rng(4)
    cur = topo.lsdb
    for _ in range(3):
        idx = rng.choice(len(cur.adjs), 25, replace=False)
        cur = modified(cur, metric=(idx, rng.integers(1, 12, len(idx))))
        names2, rp2, col2, met2, lid2, ovl2 = graph_from_lsdb(cur)
        assert names2 == names and np.array_equal(rp2, rp) and np.array_equal(col2, col)
        edges = np.nonzero(met2 != eng._graph[2])[0]
        eng.set_metric(edges, met2[edges])
        check(names, eng, plan, cur, False)


def test_unit_to_weighted_switches_plan_mode():
    """A metric patch that ends unit metrics moves the plan off the BFS path."""
    topo = T.grid(8)
    names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
    eng = SpfEngine(0)
    eng.load(rp, col, met, lid, ovl)
    plan = eng.plan(list(range(len(names))), hop=False)
    check(names, eng, plan, topo.lsdb, False)
    cur = modified(topo.lsdb, metric=(np.arange(0, len(topo.lsdb.adjs), 7), 3))
    _, _, _, met2, _, _ = graph_from_lsdb(cur)
    edges = np.nonzero(met2 != met)[0]
    eng.set_metric(edges, met2[edges])
    check(names, eng, plan, cur, False)


def test_ksp2_and_whatif_plans_refuse_a_patched_graph():
    from openr_amd._native import SpfError

    topo = T.wan(60, 30, seed=2)
    names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
    eng = SpfEngine(0)
    eng.load(rp, col, met, lid, ovl)
    kp = eng.ksp2_plan([0, 1])
    wp = eng.whatif_plan(0, [0, 1, 2])
    ptr = 16  # never dereferenced: the epoch check comes first
    eng.set_overload([5], [1])
    with pytest.raises(SpfError, match="recreate"):
        kp.execute(ptr, ptr, 16, ptr)
    with pytest.raises(SpfError, match="recreate"):
        wp.execute(ptr, ptr)
    # fresh plans see the patched graph
    res = eng.ksp2([0, 1])
    assert res is not None
    _, dig, _ = eng.whatif(0, [0, 1, 2])
    assert len(dig) == 3


def test_linkstate_overload_flips_take_the_patch_path():
    """Facade: drain/undrain publications patch the engine (epoch moves, no
    reload) and every result matches the oracle facade."""
    from adapters import OracleAdapter, ProductAdapter

    topo = T.fabric(600, full=True)
    o, p = OracleAdapter(), ProductAdapter()
    o.update_packed(topo.lsdb)
    p.update_packed(topo.lsdb)
    db_names = [bytes(topo.lsdb.blob[a: a + n]).decode()
                for a, n in zip(topo.lsdb.dbs["name_off"], topo.lsdb.dbs["name_len"])]
    probe = [db_names[0], db_names[len(db_names) // 2], db_names[-1]]
    for me in probe:
        assert p.spf(me) == o.spf(me)
    eng = SpfEngine(handle=p.ls.engine_handle())
    epoch0, loads0 = eng.epoch, eng.loads
    cur = topo.lsdb
    rng = np.random.default_rng(3)
    for step in range(4):
        runs = p.spf_runs()
        i = int(rng.integers(len(db_names)))
        flip = 1 - int(cur.dbs["is_overloaded"][i])
        cur = modified(cur, drain=[i] if flip else [], undrain=[] if flip else [i])
        o.update_packed(cur.slice(i, i + 1))
        p.update_packed(cur.slice(i, i + 1))
        for me in probe:
            assert p.spf(me) == o.spf(me), (step, me)
        # the flip cleared the memo: one logical runSpf per probe (spf_runs
        # semantics of LinkState.cpp:815)
        assert p.spf_runs() == runs + len(probe)
    assert eng.epoch > epoch0
    assert eng.loads == loads0  # patched in place, never reloaded


# ---- links going down and up without a reload (dead slots, row patches) ------
FLAP_GRAPHS = [
    ("fabric600", lambda: T.fabric(600, full=True)),
    ("rand_par", lambda: T.random_graph(40, 120, 17, max_metric=5, parallel_frac=0.35,
                                        overload_frac=0.1, link_overload_frac=0.05)),
    ("wan80", lambda: T.wan(80, 40, seed=6)),
]


@pytest.mark.parametrize("name,make", FLAP_GRAPHS, ids=[g[0] for g in FLAP_GRAPHS])
def test_link_flaps_patch_rows_and_match_oracle(name, make):
    """Publications that take links down (an adjacency's overload bit,
    Link::isUp LinkState.cpp:233-236) and up again, withdraw adjacencies and
    advertise them again (the link leaves linksFromNode and comes back first
    in its order, LinkState.cpp:564-719): every one patches the engine's rows
    in place -- no graph reload -- and getSpfResult (metrics, next hops,
    pathLinks in order), getKthPaths and spf_runs match the oracle after each."""
    import copy

    from adapters import OracleAdapter, ProductAdapter
    from openr_amd import _native as N
    from openr_amd.wire import unpack

    topo = make()
    o, p = OracleAdapter(), ProductAdapter()
    o.update_packed(topo.lsdb)
    p.update_packed(topo.lsdb)
    dbs = {d.thisNodeName: d for d in unpack(topo.lsdb)}
    names = sorted(dbs)
    rng = np.random.default_rng(5)
    probe = [names[int(i)] for i in rng.choice(len(names), 4, replace=False)]
    for me in probe:
        assert p.spf(me) == o.spf(me)
    eng = SpfEngine(handle=p.ls.engine_handle())
    loads0 = eng.loads
    patches0 = int(N.lib.ls_debug_row_patches(p.ls._h))
    withdrawn = []  # (node, adjacency) taken out of a database
    for step in range(10):
        kind = step % 3
        if kind == 0 or (kind == 2 and not withdrawn):  # overload bit of one adjacency
            node = names[int(rng.integers(len(names)))]
            db = dbs[node]
            if not db.adjacencies:
                continue
            a = db.adjacencies[int(rng.integers(len(db.adjacencies)))]
            a.isOverloaded = not a.isOverloaded
        elif kind == 1:  # withdraw an adjacency
            node = names[int(rng.integers(len(names)))]
            db = dbs[node]
            if not db.adjacencies:
                continue
            a = db.adjacencies.pop(int(rng.integers(len(db.adjacencies))))
            withdrawn.append((node, a))
        else:  # advertise a withdrawn adjacency again
            node, a = withdrawn.pop(0)
            db = dbs[node]
            db.adjacencies.append(a)
        assert o.update([copy.deepcopy(db)]) == p.update([copy.deepcopy(db)])
        for me in probe:
            assert p.spf(me) == o.spf(me), (step, me)
        for src, dst in [(probe[0], probe[1]), (probe[2], probe[3])]:
            for k in (1, 2):
                assert p.kth(src, dst, k) == o.kth(src, dst, k), (step, src, dst, k)
    assert eng.loads == loads0  # every flap patched rows in place
    assert int(N.lib.ls_debug_row_patches(p.ls._h)) > patches0


def test_link_flap_route_build_and_resident_pass():
    """After link flaps: the C++ SpfSolver's route DB equals the Python
    restatement's, and a resident all-sources pass over several members
    (rebuilt after the row patch changed next-hop layouts) gives every node's
    SPF result equal to the oracle's."""
    import copy

    from adapters import OracleAdapter
    from openr_amd.link_state import LinkState
    from openr_amd.spf_solver import PrefixEntry, PrefixState, SpfSolver
    from openr_amd.wire import unpack
    from helpers import spf_canonical

    topo = T.fabric(600, full=True)
    o = OracleAdapter()
    o.update_packed(topo.lsdb)
    dbs = {d.thisNodeName: d for d in unpack(topo.lsdb)}
    names = sorted(dbs)
    with LinkState(devices=[0, 0, 0]) as ls:
        ls.updateAdjacencyDatabases(topo.lsdb)
        ps = PrefixState()
        for i, n in enumerate(names):
            ps.updatePrefix(n, ls.getArea(), PrefixEntry(f"fd00::{i:x}/128"))
        me = names[len(names) // 2]
        held = None
        for step, node in enumerate([names[3], names[40], names[3]]):
            db = dbs[node]
            if step == 0:
                held = db.adjacencies.pop(0)  # withdrawn
            elif step == 1:
                db.adjacencies[0].isOverloaded = True  # down
            else:
                db.adjacencies.append(held)  # advertised again
            o.update([copy.deepcopy(db)])
            ls.updateAdjacencyDatabase(copy.deepcopy(db))
            got = []
            for native in (True, False):
                old = SpfSolver.native
                SpfSolver.native = native
                try:
                    db_ = SpfSolver(me, True, True).buildRouteDb(me, {ls.getArea(): ls}, ps)
                finally:
                    SpfSolver.native = old
                got.append({p_: frozenset(r.nexthops) for p_, r in db_.unicastRoutes.items()})
            assert got[0] == got[1], step
            ls.prefetchAllSources()
            for n in names[::37]:
                assert spf_canonical(ls.getSpfResult(n)) == o.spf(n), (step, n)


def test_row_patch_keeps_metric_facts():
    """spf_graph_patch_rows keeps the graph's metric facts (unit, max metric)
    from per-edge counts: taking down the only heavy link of a unit grid
    makes the graph unit again (plans go back to the BFS kernels), bringing
    it up makes it weighted; results equal a fresh load of the same CSR."""
    import ctypes as C

    from openr_amd import _native as N

    topo = T.grid(6)
    names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
    met = met.copy()
    u = 7
    e = int(rp[u])  # u's first slot and its reverse slot carry metric 5
    v = int(col[e])
    r = [q for q in range(int(rp[v]), int(rp[v + 1])) if lid[q] == lid[e]][0]
    met[e] = met[r] = 5
    eng = SpfEngine(0)
    eng.load(rp, col, met, lid, ovl)
    srcs = list(range(len(names)))
    assert eng.plan(srcs, hop=False).kernels()[0] not in ("msbfs_kernel", "msbfs_planes_kernel",
                                                          "msbfs_team_kernel")

    def patch(up):
        nodes = np.array([u, v], np.uint32)
        rows_c, rows_m, rows_l = [], [], []
        for x in (u, v):
            for q in range(int(rp[x]), int(rp[x + 1])):
                dead = (q in (e, r)) and not up
                rows_c.append(x if dead else int(col[q]))
                rows_m.append(1 if dead else int(met[q]))
                rows_l.append(int(lid[q]))
        cc = np.array(rows_c, np.uint32)
        mm = np.array(rows_m, np.int32)
        ll = np.array(rows_l, np.uint32)
        eng._err(N.lib.spf_graph_patch_rows(eng._h, N.ptr(nodes), 2, N.ptr(cc), N.ptr(mm, C.c_int32),
                                            N.ptr(ll)))
        return cc, mm

    def same_as_fresh(cc, mm):
        col2, met2 = col.copy(), met.copy()
        o = 0
        for x in (u, v):
            for q in range(int(rp[x]), int(rp[x + 1])):
                col2[q], met2[q] = cc[o], mm[o]
                o += 1
        ref = SpfEngine(0)
        ref.load(rp, col2, met2, lid, ovl)
        got = eng.plan(srcs, hop=False).execute_host()
        exp = ref.plan(srcs, hop=False).execute_host()
        assert np.array_equal(got.dist, exp.dist)
        for i in range(len(srcs)):
            assert np.array_equal(got.nh_matrix(i), exp.nh_matrix(i))
        ref.close()

    cc, mm = patch(up=False)  # the heavy link down: every live edge has metric 1
    assert eng.plan(srcs, hop=False).kernels()[0] in ("msbfs_kernel", "msbfs_planes_kernel",
                                                      "msbfs_team_kernel")
    same_as_fresh(cc, mm)
    cc, mm = patch(up=True)  # and up again: weighted
    assert eng.plan(srcs, hop=False).kernels()[0] not in ("msbfs_kernel", "msbfs_planes_kernel",
                                                          "msbfs_team_kernel")
    same_as_fresh(cc, mm)
    eng.close()
