"""Best-route selection helpers of SpfSolver (host logic, no GPU), transcribed
from the reference's own unit tests:

  * openr/common/tests/UtilTest.cpp:756-818  getPrefixForwardingTypeAndAlgorithm
  * openr/common/tests/UtilTest.cpp:820-969  MetricVectorUtils (inverse,
    isDecisive, compareMetrics, resultForLoner, maybeUpdate,
    compareMetricVectors)
  * openr/common/tests/UtilTest.cpp:990-1093 selectBestPrefixMetrics /
    selectBestNodeArea
and the area-order helper against libstdc++'s std::unordered_map
(ls_string_map_order, the container Decision.cpp walks areaLinkStates in).
"""

import copy

from openr_amd.spf_solver import (ERROR, LOOSER, TIE, TIE_LOOSER, TIE_WINNER, WINNER, MetricEntity,
                                  MetricVector, PrefixEntry, PrefixMetrics, compareMetrics,
                                  compareMetricVectors, getPrefixForwardingTypeAndAlgorithm, inverse,
                                  isDecisive, maybeUpdate, resultForLoner, selectBestNodeArea,
                                  selectBestPrefixMetrics)


def test_forwarding_type_and_algorithm():  # UtilTest.cpp:756-818
    assert getPrefixForwardingTypeAndAlgorithm({}, set()) == ("IP", "SP_ECMP")
    p = {(f"node{i}", "area1"): PrefixEntry("10.0.0.0/8") for i in (1, 2, 3)}
    best = set(p)
    assert getPrefixForwardingTypeAndAlgorithm(p, best) == ("IP", "SP_ECMP")
    p[("node3", "area1")].forwardingType = "SR_MPLS"
    assert getPrefixForwardingTypeAndAlgorithm(p, best) == ("IP", "SP_ECMP")
    assert getPrefixForwardingTypeAndAlgorithm(p, {("node3", "area1")}) == ("SR_MPLS", "SP_ECMP")
    p[("node2", "area1")].forwardingType = "SR_MPLS"
    assert getPrefixForwardingTypeAndAlgorithm(p, best) == ("IP", "SP_ECMP")
    p[("node1", "area1")].forwardingType = "SR_MPLS"
    assert getPrefixForwardingTypeAndAlgorithm(p, best) == ("SR_MPLS", "SP_ECMP")
    p[("node3", "area1")].forwardingAlgorithm = "KSP2_ED_ECMP"
    assert getPrefixForwardingTypeAndAlgorithm(p, best) == ("SR_MPLS", "SP_ECMP")
    assert getPrefixForwardingTypeAndAlgorithm(p, {("node3", "area1")}) == ("SR_MPLS", "KSP2_ED_ECMP")
    p[("node2", "area1")].forwardingAlgorithm = "KSP2_ED_ECMP"
    assert getPrefixForwardingTypeAndAlgorithm(p, best) == ("SR_MPLS", "SP_ECMP")
    p[("node1", "area1")].forwardingAlgorithm = "KSP2_ED_ECMP"
    assert getPrefixForwardingTypeAndAlgorithm(p, best) == ("SR_MPLS", "KSP2_ED_ECMP")


def test_compare_result_inverse_and_decisive():  # UtilTest.cpp:820-840
    assert inverse(LOOSER) == WINNER and inverse(WINNER) == LOOSER
    assert inverse(TIE) == TIE
    assert inverse(TIE_LOOSER) == TIE_WINNER and inverse(TIE_WINNER) == TIE_LOOSER
    assert inverse(ERROR) == ERROR
    assert all(isDecisive(r) for r in (WINNER, LOOSER, ERROR))
    assert not any(isDecisive(r) for r in (TIE_WINNER, TIE_LOOSER, TIE))


def test_compare_metrics_loner_maybe_update():  # UtilTest.cpp:860-909
    assert compareMetrics([], [], True) == TIE
    assert compareMetrics([1], [], True) == ERROR
    assert compareMetrics([1, 2], [1, 2], True) == TIE
    assert compareMetrics([2], [1], False) == WINNER
    assert compareMetrics([2, 1], [2, 3], False) == LOOSER
    assert compareMetrics([-1], [-2], True) == TIE_WINNER
    assert compareMetrics([1, 1], [2, 0], True) == TIE_LOOSER
    e = MetricEntity(0, 0, "WIN_IF_PRESENT", False)
    assert resultForLoner(e) == WINNER
    e.isBestPathTieBreaker = True
    assert resultForLoner(e) == TIE_WINNER
    e.op, e.isBestPathTieBreaker = "WIN_IF_NOT_PRESENT", False
    assert resultForLoner(e) == LOOSER
    e.isBestPathTieBreaker = True
    assert resultForLoner(e) == TIE_LOOSER
    for tb in (False, True):
        e.op, e.isBestPathTieBreaker = "IGNORE_IF_NOT_PRESENT", tb
        assert resultForLoner(e) == TIE
    r = TIE
    for upd, want in ((TIE_WINNER, TIE_WINNER), (TIE_LOOSER, TIE_WINNER), (WINNER, WINNER),
                      (TIE_WINNER, WINNER), (ERROR, ERROR)):
        r = maybeUpdate(r, upd)
        assert r == want


def _mv(n=5):
    return MetricVector(1, [MetricEntity(i, i, "WIN_IF_PRESENT", False, (i,)) for i in range(n)])


def test_compare_metric_vectors():  # UtilTest.cpp:911-969
    assert compareMetricVectors(MetricVector(), MetricVector()) == TIE
    assert compareMetricVectors(MetricVector(1), MetricVector(2)) == ERROR
    n = 5
    l, r = _mv(n), _mv(n)
    assert compareMetricVectors(l, r) == TIE
    # the comparison sorted both vectors in place (decreasing priority), so
    # index i now names priority n - 1 - i, exactly as in the reference test
    assert [e.priority for e in l.metrics] == [4, 3, 2, 1, 0]
    r.metrics[n - 2].metric = (r.metrics[n - 2].metric[0] - 1,)
    assert compareMetricVectors(l, r) == WINNER
    assert compareMetricVectors(r, l) == LOOSER
    r.metrics[n - 2].isBestPathTieBreaker = True
    assert compareMetricVectors(l, r) == ERROR
    l.metrics[n - 2].isBestPathTieBreaker = True
    assert compareMetricVectors(l, r) == TIE_WINNER
    assert compareMetricVectors(r, l) == TIE_LOOSER
    r.metrics = r.metrics[: n - 1]
    assert compareMetricVectors(l, r) == WINNER
    assert compareMetricVectors(r, l) == LOOSER
    l.metrics[0].type -= 1  # same priority, different type
    assert compareMetricVectors(l, r) == ERROR
    assert compareMetricVectors(r, l) == ERROR
    l.metrics[0].type += 1
    l.metrics[n - 1].op = "WIN_IF_NOT_PRESENT"  # l's loner
    assert compareMetricVectors(l, r) == LOOSER
    assert compareMetricVectors(r, l) == WINNER
    l.metrics[n - 1].op = "IGNORE_IF_NOT_PRESENT"
    assert compareMetricVectors(l, r) == TIE_WINNER
    assert compareMetricVectors(r, l) == TIE_LOOSER


def test_sort_metric_vector_in_place():  # UtilTest.cpp:842-858
    mv = MetricVector(0, [MetricEntity(i, i) for i in range(5)])
    assert compareMetricVectors(mv, MetricVector(0, [])) in (WINNER, TIE_WINNER, TIE)
    assert [e.priority for e in mv.metrics] == [4, 3, 2, 1, 0]


def _pm(pp, sp, d):
    return PrefixEntry("10.0.0.0/8", metrics=PrefixMetrics(pp, sp, d))


def test_best_metrics_selection():  # UtilTest.cpp:990-1093
    assert selectBestPrefixMetrics({}) == []
    assert selectBestPrefixMetrics({"KEY1": _pm(0, 0, 0)}) == ["KEY1"]
    assert selectBestPrefixMetrics({"KEY1": _pm(100, 0, 0), "KEY2": _pm(200, 0, 0),
                                    "KEY3": _pm(300, 0, 0)}) == ["KEY3"]
    assert selectBestPrefixMetrics({"KEY1": _pm(100, 10, 0), "KEY2": _pm(100, 200, 0),
                                    "KEY3": _pm(100, 30, 0)}) == ["KEY2"]
    assert selectBestPrefixMetrics({"KEY1": _pm(100, 10, 1), "KEY2": _pm(100, 10, 2),
                                    "KEY3": _pm(100, 10, 3)}) == ["KEY1"]
    assert selectBestPrefixMetrics({"KEY1": _pm(100, 10, 1), "KEY2": _pm(100, 10, 2),
                                    "KEY3": _pm(100, 10, 1), "KEY4": _pm(100, 10, 1),
                                    "KEY5": _pm(100, 10, 2)}) == ["KEY1", "KEY3", "KEY4"]
    best = selectBestPrefixMetrics({("node1", "area1"): _pm(100, 10, 1),
                                    ("node1", "area2"): _pm(100, 10, 1),
                                    ("node2", "area1"): _pm(100, 10, 1)})
    assert len(best) == 3
    assert selectBestNodeArea(best, "node1") == ("node1", "area1")
    assert selectBestNodeArea(best, "node2") == ("node2", "area1")
    # entries below the (0, 0, 0) start never enter (Util.h:556-558)
    assert selectBestPrefixMetrics({"K": _pm(0, 0, 5)}) == []


def test_area_order_is_libstdcxx_unordered_map_order():
    """areaOrder walks the areas as the reference's
    std::unordered_map<std::string, LinkState> does: checked here against
    libstdc++'s bucket order computed by g++ from a tiny program."""
    import shutil
    import subprocess
    import tempfile
    from pathlib import Path

    import ctypes as C

    from openr_amd import _native as N

    keys = ["0", "A", "B", "area1", "area2", "spine", "pod-3", "plane_1", "B"]
    arr = (C.c_char_p * len(keys))(*[k.encode() for k in keys])
    order = (C.c_uint32 * len(keys))()
    n = C.c_uint32()
    assert N.lib.ls_string_map_order(arr, len(keys), order, C.byref(n)) == N.SPF_OK
    got = [keys[order[i]] for i in range(n.value)]
    assert sorted(got) == sorted(set(keys))
    gxx = shutil.which("g++")
    if gxx is None:
        return
    src = ("#include <unordered_map>\n#include <string>\n#include <cstdio>\nint main(int c,char**v){"
           "std::unordered_map<std::string,int> m;for(int i=1;i<c;++i)m.emplace(v[i],i);"
           "for(auto&kv:m)std::printf(\"%s\\n\",kv.first.c_str());}")
    with tempfile.TemporaryDirectory() as d:
        Path(d, "o.cpp").write_text(src)
        subprocess.run([gxx, "-O1", "-o", str(Path(d, "o")), str(Path(d, "o.cpp"))], check=True)
        out = subprocess.run([str(Path(d, "o")), *keys], check=True, capture_output=True,
                             text=True).stdout.split()
    assert got == out


def test_oracle_route_digests_equal_pinned_nexthops():
    """orc_ls_route_digests (the checker of spf_mplan_route_digests) reduces
    exactly what orc_ls_nexthops_json returns (the restatement pinned by
    tests/test_oracle_reference.py to DecisionTest's route expectations):
    both on random multigraphs with drained nodes and links, SP and LFA."""
    import numpy as np

    from oracle import NameTable, OracleLinkState, nexthops, route_digests
    from openr_amd import topology as T
    from openr_amd.wire import unpack

    M = (1 << 64) - 1

    def mix(z):
        z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M
        z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M
        return z ^ (z >> 31)

    def keyhash(a, b, c, d):
        f = 0xcbf29ce484222325
        for part in (a, b, c, d):
            for ch in part.encode():
                f = ((f ^ ch) * 0x100000001b3) & M
            f = ((f ^ 0x01) * 0x100000001b3) & M
        return mix(f)

    for seed in (3, 4):
        topo = T.random_graph(25, 60, seed, max_metric=4, parallel_frac=0.3, overload_frac=0.15,
                              link_overload_frac=0.1)
        dbs = {d.thisNodeName: d for d in unpack(topo.lsdb)}
        names = sorted(topo.nodes)
        orc = OracleLinkState()
        orc.update_packed(topo.lsdb)
        rng = np.random.default_rng(seed)
        sets = [[v] for v in range(len(names))] + [
            sorted(int(x) for x in rng.choice(len(names), 3, replace=False)) for _ in range(8)]
        ptr = np.concatenate([[0], np.cumsum([len(s) for s in sets])]).astype(np.uint32)
        flat = np.concatenate([np.asarray(s, np.uint32) for s in sets])
        mes = rng.choice(len(names), 6, replace=False)
        for lfa in (False, True):
            got = route_digests(orc, NameTable(names), mes, ptr, flat, lfa)
            for t, me_i in enumerate(mes):
                me = names[me_i]
                acc = 0
                for p, s in enumerate(sets):
                    r = nexthops(orc, me, [names[v] for v in s], lfa)
                    if not r["nh"]:
                        continue
                    rec = 0
                    for ifn, metric, nb, *_ in r["nh"]:
                        oif = next(a.otherIfName for a in dbs[me].adjacencies
                                   if a.ifName == ifn and a.otherNodeName == nb)
                        (a, b), (c, d) = sorted([(me, ifn), (nb, oif)])
                        rec = (rec + mix((keyhash(a, b, c, d) + (metric & 0xFFFFFFFF)) & M)) & M
                    acc = (acc + mix((mix((0x9e3779b97f4a7c15 * (p + 1) + r["min"]) & M) + rec + p) & M)) & M
                assert int(got[t]) == acc, (seed, lfa, me)
