"""PrefixEntries iteration order and the BGP best-path walk that depends on it
(host logic, no GPU).

The reference keeps a prefix's advertisers in PrefixEntries =
std::unordered_map<NodeAndArea, PrefixEntry> (openr/common/Types.h:24), filled
by PrefixState::updatePrefixDatabase (PrefixState.cpp:47-60), copied and
filtered in place by createRouteForPrefix (Decision.cpp:409-420), and walked
in that order by runBestPathSelectionBgp (Decision.cpp:795-832).  The checker
is the oracle's restatement of the container (orc_node_area_map_order, its
own folly-pair hash), and a restatement of the walk below over that order.
"""

import random

from oracle import node_area_map_order
from openr_amd.spf_solver import (ERROR, TIE, TIE_LOOSER, TIE_WINNER, WINNER, MetricEntity,
                                  MetricVector, PrefixEntry, PrefixState, SpfSolver,
                                  compareMetricVectors, nodeAreaMapOrder)


def test_map_order_matches_oracle_on_random_histories():
    rng = random.Random(7)
    for trial in range(200):
        keys = [(f"node{rng.randrange(40)}", f"area{rng.randrange(3)}") for _ in range(30)]
        ops, live = [], set()
        for _ in range(rng.randrange(1, 60)):
            k = rng.choice(keys)
            if k in live and rng.random() < 0.4:
                ops.append((0, k))
                live.discard(k)
            else:
                ops.append((1, k))
                live.add(k)
        got = nodeAreaMapOrder(ops)
        assert sorted(got) == sorted(live)
        assert got == node_area_map_order(ops), trial


def test_prefix_state_dict_follows_map_order():
    rng = random.Random(11)
    ps = PrefixState()
    hist = []
    for step in range(300):
        node, area = f"n{rng.randrange(25)}", f"a{rng.randrange(2)}"
        if (node, area) in ps.prefixes().get("p", {}) and rng.random() < 0.35:
            ps.deletePrefix(node, area, "p")
            hist.append((0, (node, area)))
        else:
            if (node, area) not in ps.prefixes().get("p", {}):
                hist.append((1, (node, area)))
            ps.updatePrefix(node, area, PrefixEntry("p"))
        if "p" not in ps.prefixes():
            hist = []  # the map is destroyed with its last entry (PrefixState.cpp:49-50)
            continue
        assert list(ps.prefixes()["p"]) == node_area_map_order(hist), step


def _tb(v):
    """A metric vector of one tie-breaker entity: two of them compare TIE when
    equal, TIE_WINNER / TIE_LOOSER otherwise (Util.cpp:1135-1151)."""
    return MetricVector(0, [MetricEntity(1, 1, "WIN_IF_PRESENT", True, (v,))])


def _walk(order, mvs):
    """runBestPathSelectionBgp (Decision.cpp:795-832) over a given order:
    (success, allNodeAreas, bestNodeArea)."""
    best, bestNA, chosen = None, None, set()
    for na in order:
        r = WINNER if best is None else compareMetricVectors(mvs[na], best)
        if r == WINNER:
            chosen = set()
        if r in (WINNER, TIE_WINNER):
            best, bestNA = mvs[na], na
        if r in (WINNER, TIE_WINNER, TIE_LOOSER):
            chosen.add(na)
        elif r in (TIE, ERROR):
            return False, sorted(chosen), bestNA
    return True, sorted(chosen), bestNA


class _Area:
    def isNodeOverloaded(self, node):
        return False


def test_bgp_walk_follows_map_order_where_sorted_order_differs():
    """Advertisers x (value 5), y (5) and z (7) of one tie-breaker metric:
    visiting x then y aborts on a TIE; visiting z first makes x and y
    TIE_LOOSERs and z the best -- so the outcome depends on the visit order.
    Node names are drawn until the map order and the sorted order disagree."""
    found = 0
    for i in range(400):
        names = [f"bgp-{i}-{j}" for j in range(3)]
        vals = {names[0]: 5, names[1]: 5, names[2]: 7}
        keys = [(n, "0") for n in names]
        mvs = {k: _tb(vals[k[0]]) for k in keys}
        order = node_area_map_order([(1, k) for k in keys])
        want = _walk(order, mvs)
        if want == _walk(sorted(keys), mvs):
            continue
        found += 1
        ps = PrefixState()
        for k in keys:
            ps.updatePrefix(k[0], k[1], PrefixEntry("10.1.0.0/16", type="BGP", mv=mvs[k]))
        ents = ps.prefixes()["10.1.0.0/16"]
        res = SpfSolver("me", True, False)._selectBestRoutes("me", ents, True, {"0": _Area()})
        assert (res.success, sorted(res.allNodeAreas), res.bestNodeArea) == want, names
        if found == 8:
            break
    assert found >= 4  # the case exists, and was exercised


def test_bgp_walk_order_after_withdrawal():
    """Erasing an advertiser keeps the survivors' relative order (and the map's
    buckets): the walk after a withdrawal follows the replayed history, not a
    fresh insertion of the survivors."""
    rng = random.Random(3)
    checked = 0
    for i in range(300):
        names = [f"r{i}-{j}" for j in range(12)]
        keys = [(n, "0") for n in names]
        ps = PrefixState()
        hist = []
        mvs = {k: _tb(rng.choice((5, 6, 7))) for k in keys}
        for k in keys:
            ps.updatePrefix(k[0], k[1], PrefixEntry("p", type="BGP", mv=mvs[k]))
            hist.append((1, k))
        for k in rng.sample(keys, 8):
            ps.deletePrefix(k[0], k[1], "p")
            hist.append((0, k))
        order = node_area_map_order(hist)
        ents = ps.prefixes()["p"]
        assert list(ents) == order
        res = SpfSolver("me", True, False)._selectBestRoutes("me", ents, True, {"0": _Area()})
        assert (res.success, sorted(res.allNodeAreas), res.bestNodeArea) == _walk(order, mvs)
        checked += 1
    assert checked == 300
