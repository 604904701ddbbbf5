"""LinkState fed by KvStore publications (the wire path, csrc/lsdb_wire.cpp)
on the MI355X: SPF results, pathLinks order and k-th paths match the oracle
fed the same databases directly, including after a publication that drains a
node and one that expires databases (Decision.cpp:1709-1817)."""

import numpy as np
import pytest

from helpers import link_key, spf_canonical
from oracle import OracleLinkState, keyvals_order
from openr_amd import topology as T
from openr_amd.link_state import LinkState
from openr_amd.lsdb import pack
from openr_amd.wire import unpack
from thrift_compact import encode_adjacency_database, encode_publication

pytestmark = pytest.mark.gpu


def _pub(dbs, expired=()):
    return encode_publication([(f"adj:{d.thisNodeName}", encode_adjacency_database(d)) for d in dbs],
                              expired=[f"adj:{n}" for n in expired])


def _ref_order(dbs):
    """The databases of one publication in the order the reference applies
    them (its keyVals unordered_map, Decision.cpp:1726)."""
    return [dbs[i] for i in keyvals_order([f"adj:{d.thisNodeName}" for d in dbs])]


@pytest.mark.parametrize("name,make", [
    ("fabric", lambda: T.fabric(1000, full=True)),
    ("wan", lambda: T.wan(300, 150, seed=3)),
    ("rand", lambda: T.random_graph(40, 90, 5, max_metric=6, parallel_frac=0.2, overload_frac=0.1,
                                    link_overload_frac=0.05)),
], ids=["fabric", "wan", "rand"])
def test_link_state_from_publications_matches_oracle(name, make):
    topo = make()
    dbs = unpack(topo.lsdb)
    for d in dbs:
        d.area = "0"
    ls = LinkState()
    for i in range(0, len(dbs), 64):
        ls.processPublication(_pub(dbs[i:i + 64]))
    orc = OracleLinkState()
    for i in range(0, len(dbs), 64):
        orc.update_packed(pack(_ref_order(dbs[i:i + 64])))
    rng = np.random.default_rng(2)
    sample = [topo.nodes[int(i)] for i in rng.choice(len(topo.nodes), min(8, len(topo.nodes)), replace=False)]
    for s in sample:
        assert spf_canonical(ls.getSpfResult(s)) == orc.spf(s), s
    for d in sample[:3]:
        got = [[link_key(l) for l in p] for p in ls.getKthPaths(sample[0], d, 2)]
        assert got == orc.kth_paths(sample[0], d, 2)
    # drain one node, expire two others: both sides see the same LSDB
    drained = dbs[len(dbs) // 2]
    drained.isOverloaded = True
    gone = [dbs[1].thisNodeName, dbs[-1].thisNodeName]
    c = ls.processPublication(_pub([drained], expired=gone))
    assert c.topologyChanged
    orc.update_packed(pack([drained]))
    for g in gone:
        orc.delete(g)
    for s in sample:
        if s in gone:
            continue
        assert spf_canonical(ls.getSpfResult(s)) == orc.spf(s), s


def test_ordered_fib_holds_match_oracle():
    """enable_ordered_fib_programming (Decision.cpp:1750-1758): a publication
    that changes metrics and drains a node is applied with per-database
    hold-up = hops(me, originator), hold-down = maxHops(originator) - hold-up;
    until the holds expire SPF still sees the old values."""
    topo = T.random_graph(40, 90, 8, max_metric=6, parallel_frac=0.2)
    dbs = unpack(topo.lsdb)
    for d in dbs:
        d.area = "0"
    me = dbs[0].thisNodeName
    ls = LinkState()
    ls.processPublication(_pub(dbs))
    orc = OracleLinkState()
    orc.update_packed(pack(_ref_order(dbs)))
    changed = []
    for d in dbs[3:9]:
        for a in d.adjacencies:
            a.metric += 2
        changed.append(d)
    changed[1].isOverloaded = True
    ls.processPublication(_pub(changed), orderedFibNode=me)
    for d in _ref_order(changed):
        hops = orc.metric_a_to_b(me, d.thisNodeName, False)
        up = hops if hops is not None else 0
        down = orc.max_hops(d.thisNodeName) - up if hops is not None else 0
        orc.update_packed(pack([d]), up, down)
    assert ls.hasHolds() == orc.has_holds()
    for step in range(8):
        for s in (me, dbs[5].thisNodeName, dbs[20].thisNodeName):
            assert spf_canonical(ls.getSpfResult(s)) == orc.spf(s), (step, s)
        if not orc.has_holds():
            break
        c = ls.decrementHolds()
        assert (c.topologyChanged, ) == (orc.decrement_holds()[0], )
