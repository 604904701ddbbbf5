"""Batched KSP2 on the MI355X (spf_ksp2_*) against the CPU oracle's
getKthPaths (LinkState.cpp:762-791), path for path and link for link.

Small graphs (parallel links, drained nodes and links): every pair.  WAN-like
graphs (BASELINE config 4 generator): sampled pairs exact, plus
size-independent properties over every pair of a source batch: k = 1 paths are
shortest and pairwise link-disjoint, k = 2 paths avoid every k = 1 link and
have equal cost, path counts are bounded by the destination's degree.
"""

import numpy as np
import pytest

from helpers import link_key
from oracle import OracleLinkState
from openr_amd import topology as T
from openr_amd.engine import SpfEngine
from openr_amd.link_state import LinkState

pytestmark = pytest.mark.gpu


def setup(topo):
    ls = LinkState(device=-1)
    ls.updateAdjacencyDatabases(topo.lsdb)
    names, rp, col, met, lid, ovl = ls.flatten()
    eng = SpfEngine(0)
    eng.load(rp, col, met, lid, ovl)
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    keys = {}

    def key(l):
        k = keys.get(l)
        if k is None:
            k = keys[l] = link_key(ls._link(l))
        return k

    return names, eng, orc, key, (rp, col, met, lid, ovl)


def check_pairs(names, eng, orc, key, srcs, dsts=None):
    res = eng.ksp2(srcs)
    n = len(names)
    for i, s in enumerate(srcs):
        for d in (range(n) if dsts is None else dsts):
            for k in (1, 2):
                got = [[key(l) for l in p] for p in res.paths(i, d, k)]
                want = orc.kth_paths(names[s], names[d], k)
                assert got == want, (names[s], names[d], k, got, want)
    return res


SMALL = [
    ("grid6", lambda: T.grid(6)),
    ("wan80", lambda: T.wan(80, 40, seed=5)),
    ("fabric_ref1000", lambda: T.fabric(1000, full=False)),
] + [
    (f"rand{seed}", (lambda s: lambda: T.random_graph(
        30, 70, 200 + s, max_metric=6, parallel_frac=0.25, overload_frac=0.1,
        link_overload_frac=0.05))(seed))
    for seed in range(6)
]


@pytest.mark.parametrize("name,make", SMALL, ids=[s[0] for s in SMALL])
def test_ksp2_all_pairs_exact(name, make):
    names, eng, orc, key, _ = setup(make())
    n = len(names)
    srcs = list(range(n)) if n <= 80 else list(range(0, n, max(1, n // 24)))
    check_pairs(names, eng, orc, key, srcs)


def test_ksp2_wan2000_sampled_exact_and_properties():
    """BASELINE config 4 topology (wan N=2000, 1000 chords)."""
    topo = T.wan(2000, 1000, seed=1)
    names, eng, orc, key, (rp, col, met, lid, ovl) = setup(topo)
    n = len(names)
    rng = np.random.default_rng(7)
    srcs = sorted(int(x) for x in rng.choice(n, 64, replace=False))
    res = eng.ksp2(srcs)
    # exact against the oracle on sampled pairs
    for i in (0, 37):
        for d in sorted(int(x) for x in rng.choice(n, 40, replace=False)):
            for k in (1, 2):
                got = [[key(l) for l in p] for p in res.paths(i, d, k)]
                assert got == orc.kth_paths(names[srcs[i]], names[d], k)
    # properties over every pair of the batch
    tail = np.repeat(np.arange(n), np.diff(rp))
    w_of = {}
    for e in range(len(col)):
        w_of[(int(lid[e]), int(tail[e]))] = int(met[e])
    ends = {}
    for e in range(len(col)):
        ends.setdefault(int(lid[e]), set()).update((int(tail[e]), int(col[e])))
    dist = eng.solve(srcs).dist

    def walk(s, path):
        cost, at = 0, s
        for l in path:
            a, b = ends[l]
            nxt = b if at == a else a
            assert at in (a, b)
            cost += w_of[(l, at)]
            at = nxt
        return cost, at

    deg = np.diff(rp)
    for i, s in enumerate(srcs[:24]):
        for d in range(n):
            p1, p2 = res.paths(i, d, 1), res.paths(i, d, 2)
            if d == s:
                assert not p1 and not p2
                continue
            assert 1 <= len(p1) <= deg[d]
            used = set()
            for p in p1:
                c, end = walk(s, p)
                assert end == d and c == dist[i, d]
                assert not used & set(p)
                used |= set(p)
            c2 = None
            for p in p2:
                c, end = walk(s, p)
                assert end == d and not used & set(p)
                assert c2 is None or c == c2
                c2 = c
                assert c >= dist[i, d]


def test_ksp2_counts_k2_spf_runs():
    names, eng, orc, key, _ = setup(T.wan(60, 30, seed=2))
    before = eng.solves()
    eng.ksp2([0, 1])
    # n_src k=1 SPFs plus one k=2 SPF per reachable pair other than the source
    assert eng.solves() - before == 2 + 2 * (len(names) - 1)
