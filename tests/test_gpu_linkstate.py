"""The LinkState drop-in (openr_amd.link_state on libopenr_spf.so) on the
MI355X against the reference's test expectations and the oracle: SPF results
including pathLinks order, getKthPaths, hop counts, spf_runs."""

import numpy as np
import pytest

from adapters import OracleAdapter, ProductAdapter
from helpers import link_key, spf_canonical
from oracle import OracleLinkState
from refcases import load_cases, run_case
from openr_amd import topology as T
from openr_amd.link_state import LinkState

pytestmark = pytest.mark.gpu
CASES = load_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_product_matches_reference_tests(case):
    run_case(case, ProductAdapter)


@pytest.mark.parametrize("seed", range(8))
def test_spf_and_kth_paths_match_oracle(seed):
    topo = T.random_graph(24, 50, 100 + seed, max_metric=4, parallel_frac=0.3,
                          overload_frac=0.1, link_overload_frac=0.05)
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    ls = LinkState()
    ls.updateAdjacencyDatabases(topo.lsdb)
    for s in topo.nodes:
        for ulm in (True, False):
            assert spf_canonical(ls.getSpfResult(s, ulm)) == orc.spf(s, ulm), (s, ulm)
    for s in topo.nodes[:8]:
        for d in topo.nodes:
            for k in (1, 2, 3):
                got = [[link_key(l) for l in p] for p in ls.getKthPaths(s, d, k)]
                assert got == orc.kth_paths(s, d, k), (s, d, k)


def test_incremental_updates_invalidate_memo():
    """Benchmark pattern (RoutingBenchmarkUtils.cpp:453-479): toggle a node's
    overload bit and re-query; results track the oracle at each step."""
    topo = T.fabric(1000, full=True)
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    ls = LinkState()
    ls.updateAdjacencyDatabases(topo.lsdb)
    src = "2-0-0"
    node = "3-1-7"
    i = topo.nodes.index(node)
    one = topo.lsdb.slice(i, i + 1)
    for ovl in (1, 0, 1):
        one.dbs["is_overloaded"] = ovl
        c1 = orc.update_packed(one)
        c2 = ls.updateAdjacencyDatabases(one)
        assert c1 == [(c.topologyChanged, c.linkAttributesChanged, c.nodeLabelChanged) for c in c2]
        assert spf_canonical(ls.getSpfResult(src)) == orc.spf(src)


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("ulm", [True, False], ids=["metric", "hops"])
def test_prefetch_spf_results_equal_single_queries_and_count_runs(seed, ulm):
    """ls_prefetch_spf_results (one batched plan for me + every LFA
    neighbour, Decision.cpp:1158-1165): the same SpfResults as the one-by-one
    queries (metrics, next hops, pathLinks order, against the oracle), and
    spf_runs counts each node when it is first read, as the reference's
    getSpfResult calls would (LinkState.cpp:815)."""
    topo = T.random_graph(60, 150, 300 + seed, max_metric=6, parallel_frac=0.2,
                          overload_frac=0.1, link_overload_frac=0.05)
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    ls = LinkState()
    ls.updateAdjacencyDatabases(topo.lsdb)
    me = topo.nodes[seed]
    nbrs = sorted({l.getOtherNodeName(me) for l in ls.linksFromNode(me)})
    want = [me] + nbrs + ["not-a-node", me]
    runs0 = ls.spfRuns()
    ls.prefetchSpfResults(want, ulm)
    assert ls.spfRuns() == runs0  # nothing read yet
    for i, node in enumerate([me] + nbrs):
        assert spf_canonical(ls.getSpfResult(node, ulm)) == orc.spf(node, ulm), node
        assert ls.spfRuns() == runs0 + i + 1
    ls.getSpfResult(me, ulm)
    assert ls.spfRuns() == runs0 + 1 + len(nbrs)  # memoised


def test_prefetch_spf_results_fabric_all_neighbours():
    topo = T.fabric(1000, full=True)
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    ls = LinkState()
    ls.updateAdjacencyDatabases(topo.lsdb)
    me = "3-0-0"
    nbrs = sorted({l.getOtherNodeName(me) for l in ls.linksFromNode(me)})
    ls.prefetchSpfResults([me] + nbrs)
    for node in [me] + nbrs:
        assert spf_canonical(ls.getSpfResult(node)) == orc.spf(node), node


@pytest.mark.parametrize("ulm", [True, False], ids=["metric", "hops"])
def test_get_spf_result_on_big_plans(ulm, monkeypatch):
    """graphs beyond the LDS-resident kernels take
    spf_big_kernel plans; getSpfResult and the batched LFA prefetch must still
    give the reference's results (pathLinks from the big plan's rows).
    SPF_BIG=1 sends a small graph there."""
    monkeypatch.setenv("SPF_BIG", "1")
    topo = T.random_graph(60, 150, 900, max_metric=6, parallel_frac=0.2,
                          overload_frac=0.1, link_overload_frac=0.05)
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    ls = LinkState()
    ls.updateAdjacencyDatabases(topo.lsdb)
    for node in topo.nodes[:10]:
        assert spf_canonical(ls.getSpfResult(node, ulm)) == orc.spf(node, ulm), node
    me = topo.nodes[11]
    nbrs = sorted({l.getOtherNodeName(me) for l in ls.linksFromNode(me)})
    ls.prefetchSpfResults([me] + nbrs, ulm)
    for node in [me] + nbrs:
        assert spf_canonical(ls.getSpfResult(node, ulm)) == orc.spf(node, ulm), node
    ls.close()
