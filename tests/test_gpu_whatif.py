"""What-if batches on the MI355X (spf_whatif_*): the digest of
runSpf(src, true, {l}) for every single-link failure l, against the CPU
oracle's digests of full re-runs (LinkState.cpp:808-882 with linksToIgnore).

Small graphs (parallel links, drained nodes and links): a large sample of
failures, every one checked.  BASELINE config 5 (Barabasi-Albert, 250k nodes,
~1M links): every failure computed on the GPU, a sample of hot failures
(including the largest affected regions) checked against the oracle, plus
size-independent properties over all of them.
"""

import numpy as np
import pytest

from oracle import NameTable, OracleLinkState, whatif_digests
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
    return ls, names, eng, orc, (rp, col, met, lid, ovl)


def fail_of(ls, l):
    lk = ls._link(int(l))
    return (lk._n1, lk._if1)


def as_tuple(d):
    return int(d["n_dist_changed"]), int(d["n_nh_changed"]), int(d["hash"])


SMALL = [
    ("ba1500", lambda: T.barabasi_albert(1500, 3, seed=4), "0"),
    ("wan200", lambda: T.wan(200, 100, seed=6), None),
    ("grid12", lambda: T.grid(12), None),
] + [
    (f"rand{seed}", (lambda s: lambda: T.random_graph(
        70, 180, 300 + s, max_metric=5, parallel_frac=0.2, overload_frac=0.1,
        link_overload_frac=0.05))(seed), None)
    for seed in range(4)
]


@pytest.mark.parametrize("name,make,src", SMALL, ids=[s[0] for s in SMALL])
def test_whatif_matches_oracle(name, make, src):
    ls, names, eng, orc, _ = setup(make())
    s = names.index(src) if src else 0
    links, got, base = eng.whatif(s)
    table = NameTable(names)
    rng = np.random.default_rng(1)
    pick = rng.choice(len(links), min(len(links), 400), replace=False)
    obase, want = whatif_digests(orc, table, names[s], [fail_of(ls, links[i]) for i in pick])
    assert as_tuple(base) == obase
    for i, w in zip(pick, want):
        assert as_tuple(got[i]) == w, (names[s], fail_of(ls, links[i]))


def test_whatif_explicit_link_list_and_drained_source():
    topo = T.random_graph(50, 120, 17, max_metric=4, overload_frac=0.2)
    ls, names, eng, orc, (rp, col, met, lid, ovl) = setup(topo)
    s = int(np.nonzero(ovl)[0][0])  # a drained node still expands as the source
    links = sorted(set(int(x) for x in lid))[::3]
    got_links, got, base = eng.whatif(s, links)
    assert list(got_links) == links
    obase, want = whatif_digests(orc, NameTable(names), names[s],
                                 [fail_of(ls, l) for l in links])
    assert as_tuple(base) == obase
    assert [as_tuple(d) for d in got] == want


WIDE = [
    # U[1, 1000] metrics on a 3000-node WAN: the big repairs hold far more than
    # kDialLevels (1024) distinct distances, so the workgroup teams leave the
    # Dial loop for label-correcting sweeps + the level sort (whatif.hip:899-980)
    ("wan3000_m1e3", lambda: T.wan(3000, 1500, seed=2), 1_000),
    # U[1, 1e5]: the unfailed distances pass kLevelCap (65536), so the base
    # pass takes its fixed-point path (whatif.hip:321) and the repairs' level
    # span exceeds their cap (fixed-point sweeps, whatif.hip:981)
    ("wan3000_m1e5", lambda: T.wan(3000, 1500, seed=3, max_metric=100_000), 100_000),
]


@pytest.mark.parametrize("name,make,max_metric", WIDE, ids=[w[0] for w in WIDE])
def test_whatif_wide_metrics_fallback_paths(name, make, max_metric):
    """graphs whose distances leave the bucketed (levels / Dial)
    paths; the hottest failures plus a random sample, each against the
    oracle's full re-run."""
    ls, names, eng, orc, _ = setup(make())
    s = 0
    links, got, base = eng.whatif(s)
    d = eng.sssp(s)
    if max_metric >= 65536:
        assert int(d[d != 0xFFFFFFFF].max()) >= 65536  # base: non-levels path
    size = got["n_dist_changed"].astype(np.int64)
    assert size.max() > 1024  # a repair beyond the Dial level budget
    order = np.argsort(-size)
    rng = np.random.default_rng(3)
    pick = list(order[:12]) + list(rng.choice(len(links), 120, replace=False))
    obase, want = whatif_digests(orc, NameTable(names), names[s],
                                 [fail_of(ls, links[i]) for i in pick])
    assert as_tuple(base) == obase
    for i, w in zip(pick, want):
        assert as_tuple(got[i]) == w, (name, fail_of(ls, links[i]))


@pytest.fixture(scope="module")
def ba250k():
    return setup(T.barabasi_albert(250_000, 4, seed=1))


def test_whatif_ba250k_sampled_exact_and_properties(ba250k):
    """BASELINE config 5: every single-link failure of the 1M-link graph."""
    ls, names, eng, orc, (rp, col, met, lid, ovl) = ba250k
    s = names.index("0")
    plan = eng.whatif_plan(s)
    links, got, base = eng.whatif(s, plan.links)
    assert len(links) == len(set(int(x) for x in lid))  # every up link
    H = int(base["hash"])
    unchanged = (got["n_dist_changed"] == 0) & (got["n_nh_changed"] == 0)
    assert (got["hash"][unchanged] == H).all()
    assert (got["hash"][~unchanged] != H).all()
    # hot failures = tight links of the DAG: their heads change at least
    n_hot = int((~unchanged).sum())
    assert 0 < n_hot < len(links)
    # oracle on a sample: the largest affected regions, a few random hot and cold;
    rng = np.random.default_rng(5)
    size = got["n_nh_changed"].astype(np.int64)
    order = np.argsort(-size)
    hot = np.nonzero(~unchanged)[0]
    cold = np.nonzero(unchanged)[0]
    # ranks 0-1 and 5 are repaired by the workgroup teams classified up front
    # (second stream), ranks ~40 and ~150 straddle the wave-team capacity
    pick = list(order[:2]) + [order[5], order[40], order[150]] + \
        list(rng.choice(hot, 3, replace=False)) + list(rng.choice(cold, 1, replace=False))
    obase, want = whatif_digests(orc, NameTable(names), "0",
                                 [fail_of(ls, links[i]) for i in pick])
    assert as_tuple(base) == obase
    for i, w in zip(pick, want):
        assert as_tuple(got[i]) == w, fail_of(ls, links[i])


def test_big_graph_single_source_sssp(ba250k):
    """spf_sssp on a graph beyond the LDS kernels runs the global-memory
    kernel; distances equal an independent Dijkstra (scipy) on the same CSR
    (no drained nodes in this graph)."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import dijkstra

    ls, names, eng, orc, (rp, col, met, lid, ovl) = ba250k
    s = names.index("0")
    d = eng.sssp(s)
    n = len(names)
    A = sp.csr_matrix((met.astype(np.float64), col, rp), shape=(n, n))
    ref = dijkstra(A, indices=s)
    ref = np.where(np.isinf(ref), 0xFFFFFFFF, ref).astype(np.uint32)
    assert np.array_equal(d, ref)
