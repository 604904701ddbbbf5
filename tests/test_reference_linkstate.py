"""Reference tests transcribed statement for statement and run against the
product through the C-ABI (host-side objects, no GPU):

* HoldableValueTest.BasicOperation   -- LinkStateTest.cpp:22-83
* LinkTest.BasicOperation            -- LinkStateTest.cpp:85-137
* LinkStateTest.pathAInPathB         -- LinkStateTest.cpp:202-242 (standalone
  links) and the same walk over links of a LinkState (link ids)
* DecisionTest grid route count       -- DecisionTest.cpp:4301-4313: the SpfSolver
  of every node of an n x n grid programs 2n^4 + 3n^2 - 4n routes in total
  (the GPU half of that check is in test_gpu_routes.py).
"""

import pytest

from openr_amd.link_state import HoldableValue, LinkState, OwnedLink
from openr_amd.lsdb import K_DEFAULT_AREA, create_adjacency


def test_holdable_value_basic_operation():
    hv = HoldableValue(True)
    assert hv.value()
    assert not hv.hasHold()
    assert not hv.decrementTtl()
    holdUpTtl, holdDownTtl = 10, 5
    assert not hv.updateValue(False, holdUpTtl, holdDownTtl)
    for _ in range(holdUpTtl - 1):
        assert hv.hasHold()
        assert hv.value()
        assert not hv.decrementTtl()
    # expire the hold
    assert hv.decrementTtl()
    assert not hv.hasHold()
    assert not hv.value()

    # expect no hold since the value didn't change
    assert not hv.updateValue(False, holdUpTtl, holdDownTtl)
    assert not hv.hasHold()
    assert not hv.value()

    # change is bringing down now
    assert not hv.updateValue(True, holdUpTtl, holdDownTtl)
    for _ in range(holdDownTtl - 1):
        assert hv.hasHold()
        assert not hv.value()
        assert not hv.decrementTtl()
    # expire the hold
    assert hv.decrementTtl()
    assert not hv.hasHold()
    assert hv.value()

    # change twice within ttl
    assert not hv.updateValue(False, holdUpTtl, holdDownTtl)
    assert hv.hasHold()
    assert hv.value()
    assert not hv.decrementTtl()

    assert hv.updateValue(True, holdUpTtl, holdDownTtl)
    assert not hv.hasHold()
    assert hv.value()

    # test with LinkMetric
    hvLsm = HoldableValue(10)
    assert hvLsm.value() == 10
    assert not hvLsm.hasHold()
    assert not hvLsm.decrementTtl()

    # change is bringing up
    assert not hvLsm.updateValue(5, holdUpTtl, holdDownTtl)
    for _ in range(holdUpTtl - 1):
        assert hvLsm.hasHold()
        assert hvLsm.value() == 10
        assert not hvLsm.decrementTtl()
    # expire the hold
    assert hvLsm.decrementTtl()
    assert not hvLsm.hasHold()
    assert hvLsm.value() == 5


def test_link_basic_operation():
    n1 = "node1"
    adj1 = create_adjacency(n1, "if1", "if2", "fe80::2", "10.0.0.2", 1, 1, 1)
    n2 = "node2"
    adj2 = create_adjacency(n2, "if2", "if1", "fe80::1", "10.0.0.1", 1, 2, 1)

    l1 = OwnedLink(K_DEFAULT_AREA, n1, adj1, n2, adj2)
    assert l1.getArea() == K_DEFAULT_AREA
    assert l1.getOtherNodeName(n1) == n2
    assert l1.getOtherNodeName(n2) == n1
    with pytest.raises(ValueError):
        l1.getOtherNodeName("node3")

    assert l1.getIfaceFromNode(n1) == adj1.ifName
    assert l1.getIfaceFromNode(n2) == adj2.ifName
    with pytest.raises(ValueError):
        l1.getIfaceFromNode("node3")

    assert l1.getMetricFromNode(n1) == adj1.metric
    assert l1.getMetricFromNode(n2) == adj2.metric
    with pytest.raises(ValueError):
        l1.getMetricFromNode("node3")

    assert l1.getAdjLabelFromNode(n1) == adj1.adjLabel
    assert l1.getAdjLabelFromNode(n2) == adj2.adjLabel
    with pytest.raises(ValueError):
        l1.getAdjLabelFromNode("node3")

    assert not l1.getOverloadFromNode(n1)
    assert not l1.getOverloadFromNode(n2)
    assert l1.isUp()
    with pytest.raises(ValueError):
        l1.getOtherNodeName("node3")

    assert l1.setMetricFromNode(n1, 2, 0, 0)
    assert l1.getMetricFromNode(n1) == 2

    assert l1.setOverloadFromNode(n2, True, 0, 0)
    assert not l1.getOverloadFromNode(n1)
    assert l1.getOverloadFromNode(n2)
    assert not l1.isUp()

    # compare equivalent links
    l2 = OwnedLink(K_DEFAULT_AREA, n2, adj2, n1, adj1)
    assert l1 == l2
    assert not l1 < l2
    assert not l2 < l1

    # compare non equal links
    n3 = "node3"
    adj3 = create_adjacency(n2, "if3", "if2", "fe80::3", "10.0.0.3", 1, 1, 1)
    l3 = OwnedLink(K_DEFAULT_AREA, n1, adj1, n3, adj3)
    assert not l1 == l3
    assert l1 < l3 or l3 < l1


def _bare(node_if):
    from openr_amd.lsdb import Adjacency

    return Adjacency(otherNodeName="", ifName=node_if, metric=1)


def test_path_a_in_path_b():
    l1 = OwnedLink(K_DEFAULT_AREA, "1", _bare("1/2"), "2", _bare("2/1"))
    l2 = OwnedLink(K_DEFAULT_AREA, "2", _bare("2/3"), "3", _bare("3/2"))
    l3 = OwnedLink(K_DEFAULT_AREA, "1", _bare("1/3"), "3", _bare("3/1"))
    p1, p2 = [], []
    f = LinkState.pathAInPathB

    assert f(p1, p2)
    assert f(p2, p1)

    p1.append(l1)

    assert not f(p1, p2)
    assert f(p2, p1)

    p2.append(l1)

    assert f(p1, p2)
    assert f(p2, p1)

    p1.append(l2)

    assert not f(p1, p2)
    assert f(p2, p1)

    p1.append(l3)
    p2.append(l2)

    assert not f(p1, p2)
    assert f(p2, p1)

    p1.clear()
    p2.clear()

    p1.append(l3)
    p1.append(l2)

    p2.append(l1)

    assert not f(p1, p2)
    assert not f(p2, p1)


def test_path_a_in_path_b_over_link_state_links():
    """The same walk with links of one LinkState (identity = link id)."""
    from helpers import get_link_state_dbs

    with LinkState(device=-1) as ls:
        ls.updateAdjacencyDatabases(get_link_state_dbs({1: [2, 3], 2: [1, 3], 3: [1, 2]}))
        by_key = {}
        for n in ("1", "2", "3"):
            for l in ls.linksFromNode(n):
                by_key[tuple(sorted([l.firstNodeName(), l.secondNodeName()]))] = l
        l1, l2, l3 = by_key[("1", "2")], by_key[("2", "3")], by_key[("1", "3")]
        f = LinkState.pathAInPathB
        assert f([l1], [l3, l1]) and not f([l1, l2], [l1]) and f([l1, l2], [l3, l1, l2])
        assert not f([l3, l2], [l1]) and f([], [l2])
        # a fresh snapshot of the same link is the same link
        l1b = [l for l in ls.linksFromNode("1") if l == l1][0]
        assert f([l1b], [l1])


def test_path_a_in_path_b_compares_by_value():
    """Links compare by value (Link::operator==, LinkState.cpp:356-361):
    two distinct OwnedLinks with the same endpoints are equal, and a link of
    a LinkState equals an OwnedLink with the same (hash, orderedNames)."""
    from helpers import get_link_state_dbs

    a = OwnedLink(K_DEFAULT_AREA, "1", _bare("1/2"), "2", _bare("2/1"))
    b = OwnedLink(K_DEFAULT_AREA, "2", _bare("2/1"), "1", _bare("1/2"))  # same link, sides swapped
    c = OwnedLink(K_DEFAULT_AREA, "2", _bare("2/3"), "3", _bare("3/2"))
    assert a is not b and a == b and a != c
    f = LinkState.pathAInPathB
    assert f([a], [c, b]) and f([b, c], [a, c]) and not f([a, c], [c, a])
    with LinkState(device=-1) as ls1, LinkState(device=-1) as ls2:
        dbs = get_link_state_dbs({1: [2], 2: [1, 3], 3: [2]})
        ls1.updateAdjacencyDatabases(dbs)
        ls2.updateAdjacencyDatabases(dbs)
        x = {l.getOtherNodeName("2"): l for l in ls1.linksFromNode("2")}
        y = {l.getOtherNodeName("2"): l for l in ls2.linksFromNode("2")}
        assert f([x["1"]], [y["3"], y["1"]]) and not f([x["1"], x["3"]], [y["3"], y["1"]])
        owned = OwnedLink(K_DEFAULT_AREA, "1", _bare(x["1"].getIfaceFromNode("1")),
                          "2", _bare(x["1"].getIfaceFromNode("2")))
        assert owned.hash == x["1"].hash
        assert f([owned], [y["1"]])
