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
