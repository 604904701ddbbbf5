"""Host-side LinkState logic of the product (no GPU): LSDB bookkeeping and the
CSR flatten, compared with the oracle on random update/delete/hold sequences.

LinkState(device=-1) runs the C++ facade without an engine; shortest-path
queries are not made here (they are GPU tests).
"""

import numpy as np
import pytest

from adapters import HostOnlyProductAdapter, OracleAdapter
from helpers import link_key
from oracle import OracleLinkState
from refcases import load_cases, dbs_from_json
from openr_amd import topology as T
from openr_amd.link_state import LinkState
from openr_amd.lsdb import pack


def _lsdb_steps_only(case):
    return [st for st in case["steps"] if "update" in st or "delete" in st or "check_links" in st]


@pytest.mark.parametrize("case", [c for c in load_cases() if c["steps"]],
                         ids=lambda c: c["name"])
def test_reference_change_flags_and_links(case):
    ls = LinkState(device=-1)
    for step in _lsdb_steps_only(case):
        if "update" in step:
            got = [(c.topologyChanged, c.linkAttributesChanged, c.nodeLabelChanged)
                   for c in ls.updateAdjacencyDatabases(dbs_from_json(step["update"]))]
            if "expect_change" in step:
                assert got == [tuple(x) for x in step["expect_change"]]
        if "delete" in step:
            c = ls.deleteAdjacencyDatabase(step["delete"])
            assert (c.topologyChanged, c.linkAttributesChanged,
                    c.nodeLabelChanged) == tuple(step["expect_change"])
        for node, links in step.get("check_links", {}).items():
            assert sorted(link_key(l) for l in ls.linksFromNode(node)) == sorted(links)
        for node, ovl in step.get("check_overloaded", {}).items():
            assert ls.isNodeOverloaded(node) == ovl


def _random_ops(seed, n=30, links=60, steps=40):
    rng = np.random.default_rng(seed)
    topo = T.random_graph(n, links, seed, max_metric=6, parallel_frac=0.25,
                          overload_frac=0.1, link_overload_frac=0.05)
    dbs = {}
    p = topo.lsdb
    blob = p.blob
    for r in p.dbs:
        name = blob[r["name_off"]: r["name_off"] + r["name_len"]].decode()
        dbs[name] = r
    names = list(dbs)
    ops = [("update_all", None)]
    for _ in range(steps):
        kind = rng.choice(["metric", "overload", "drop_adj", "node_ovl", "delete", "readd",
                           "holds"])
        ops.append((str(kind), (names[int(rng.integers(len(names)))], int(rng.integers(1, 9)),
                                int(rng.integers(0, 3)), int(rng.integers(0, 3)))))
    return topo, names, ops


def _slice_one(packed, i, mutate=None):
    one = packed.slice(i, i + 1)
    one = type(packed)(packed.blob, one.dbs.copy(), packed.adjs.copy())
    if mutate:
        mutate(one)
    return one


@pytest.mark.parametrize("seed", range(12))
def test_random_lsdb_sequences_match_oracle(seed):
    topo, names, ops = _random_ops(seed)
    orc = OracleLinkState()
    ls = LinkState(device=-1)
    idx = {n: i for i, n in enumerate(names)}
    for kind, arg in ops:
        if kind == "update_all":
            a = orc.update_packed(topo.lsdb)
            b = ls.updateAdjacencyDatabases(topo.lsdb)
        elif kind == "holds":
            a = [orc.decrement_holds()]
            b = [ls.decrementHolds()]
        elif kind == "delete":
            a = [orc.delete(arg[0])]
            b = [ls.deleteAdjacencyDatabase(arg[0])]
        else:
            node, val, up, down = arg
            i = idx[node]

            def mutate(one, kind=kind, val=val):
                r = one.dbs[0]
                b0, cnt = int(r["adj_begin"]), int(r["adj_count"])
                if kind == "node_ovl":
                    one.dbs["is_overloaded"][0] ^= 1
                elif cnt and kind == "metric":
                    one.adjs["metric"][b0 + val % cnt] = val
                elif cnt and kind == "overload":
                    one.adjs["is_overloaded"][b0 + val % cnt] ^= 1
                elif cnt and kind == "drop_adj":
                    one.dbs["adj_count"][0] = cnt - 1
            one = _slice_one(topo.lsdb, i, mutate)
            a = orc.update_packed(one, up, down)
            b = ls.updateAdjacencyDatabases(one, up, down)
        assert a == [(c.topologyChanged, c.linkAttributesChanged, c.nodeLabelChanged)
                     for c in b], (kind, arg)
        assert orc.num_links() == ls.numLinks()
        assert orc.num_nodes() == ls.numNodes()
        assert orc.has_holds() == ls.hasHolds()
        for n in names:
            assert [l[0] for l in orc.links(n)] == [link_key(l) for l in ls.linksFromNode(n)]
            assert orc.is_overloaded(n) == ls.isNodeOverloaded(n)


def test_flatten_is_every_link_in_iteration_order_down_links_dead():
    """The flattened CSR holds a slot for every link of a node in linksFromNode
    order: an up link towards its other end with the metric advertised by the
    node, a down link as a dead slot (a self-loop of metric 1, openr_spf.h),
    so that a link going down or up later patches its rows in place."""
    topo = T.random_graph(40, 90, 7, max_metric=9, parallel_frac=0.3, overload_frac=0.1,
                          link_overload_frac=0.1)
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    ls = LinkState(device=-1)
    ls.updateAdjacencyDatabases(topo.lsdb)
    names, rp, col, met, lid, ovl = ls.flatten()
    assert names == sorted(names)  # ids are ascending-name ranks (LinkState.h:488-498)
    n_dead = 0
    for u, name in enumerate(names):
        want = orc.links(name)  # (key, metric from u, up) in iteration order
        assert rp[u + 1] - rp[u] == len(want)
        for e, (k, m, up) in zip(range(rp[u], rp[u + 1]), want):
            if up:
                assert int(met[e]) == m
                assert names[int(col[e])] == (k[2] if k[0] == name else k[0])
            else:
                n_dead += 1
                assert int(col[e]) == u and int(met[e]) == 1
        assert bool(ovl[u]) == orc.is_overloaded(name)
    assert n_dead > 0
    # every link id appears exactly twice (both directions)
    _, counts = np.unique(lid, return_counts=True)
    assert (counts == 2).all()


def test_fabric_ingest_sizes():
    topo = T.fabric(10000, full=True)
    ls = LinkState(device=-1)
    ls.updateAdjacencyDatabases(topo.lsdb)
    assert ls.numLinks() == 116256
    names, rp, col, *_ = ls.flatten()
    assert len(names) == 9976 and len(col) == 232512
    ref = T.fabric(10000, full=False)
    ls2 = LinkState(device=-1)
    ls2.updateAdjacencyDatabases(ref.lsdb)
    # the reference generator's per-pod emplace keeps one SSW adjacency
    # (RoutingBenchmarkUtils.cpp:261-271): only pod 0's FSWs reach the spine
    assert ls2.numLinks() == 173 * 8 * 48 + 288
