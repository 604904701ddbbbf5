"""Runner for tests/golden/reference_expectations.json.

The same cases are replayed against the CPU oracle (tests/test_oracle_*.py,
no GPU) and against the product LinkState on the MI355X
(tests/test_gpu_linkstate.py) through a small adapter interface.
"""

from __future__ import annotations

import json
from pathlib import Path
from typing import Dict, List, Optional

from openr_amd.lsdb import AdjacencyDatabase, Adjacency

GOLDEN = Path(__file__).resolve().parent / "golden" / "reference_expectations.json"


def load_cases() -> List[dict]:
    return json.loads(GOLDEN.read_text())["cases"]


def dbs_from_json(items) -> List[AdjacencyDatabase]:
    out = []
    for d in items:
        adjs = [Adjacency(otherNodeName=a["other"], ifName=a["if"], otherIfName=a["oif"],
                          metric=a["metric"], adjLabel=a["label"],
                          isOverloaded=a["overloaded"], nextHopV6=bytes.fromhex(a["v6"]),
                          nextHopV4=bytes.fromhex(a["v4"]))
                for a in d["adjs"]]
        out.append(AdjacencyDatabase(thisNodeName=d["node"], isOverloaded=d["overloaded"],
                                     adjacencies=adjs, nodeLabel=d["nodeLabel"]))
    return out


class Adapter:
    """What a LinkState implementation must expose to the runner."""

    def update(self, dbs: List[AdjacencyDatabase]) -> List[tuple]: ...
    def delete(self, node: str) -> tuple: ...
    def links(self, node: str) -> List[list]: ...
    def overloaded(self, node: str) -> bool: ...
    def spf(self, src: str, ulm: bool) -> Dict[str, dict]: ...
    def kth(self, src: str, dst: str, k: int) -> List[List[list]]: ...
    def hops(self, a: str, b: str) -> Optional[int]: ...
    def max_hops(self, n: str) -> int: ...
    def spf_runs(self) -> int: ...


def _metric_from(dbs: Dict[str, AdjacencyDatabase], link: list, node: str) -> int:
    n1, if1, n2, if2 = link
    me_if = if1 if node == n1 else if2
    other = n2 if node == n1 else n1
    for a in dbs[node].adjacencies:
        if a.ifName == me_if and a.otherNodeName == other:
            return a.metric
    raise KeyError((node, link))


def _path_metric(dbs, path, src) -> int:
    cur, total = src, 0
    for link in path:
        total += _metric_from(dbs, link, cur)
        cur = link[2] if cur == link[0] else link[0]
    return total


def run_case(case: dict, make) -> None:
    """`make()` returns a fresh Adapter.  Raises AssertionError on mismatch."""
    ad = make()
    latest: Dict[str, AdjacencyDatabase] = {}
    if "grid" in case:
        from openr_amd.topology import decision_test_grid

        topo = decision_test_grid(case["grid"])
        ad.update_packed(topo.lsdb)
        for chk in case["checks"]:
            _check(chk, ad, latest, case)
        return
    for step in case["steps"]:
        if "update" in step:
            dbs = dbs_from_json(step["update"])
            got = ad.update(dbs)
            for d in dbs:
                latest[d.thisNodeName] = d
            if "expect_change" in step:
                exp = [tuple(x) for x in step["expect_change"]]
                assert got == exp, (case["name"], "changes", got, exp)
        if "delete" in step:
            got = ad.delete(step["delete"])
            latest.pop(step["delete"], None)
            assert got == tuple(step["expect_change"]), (case["name"], "delete", got)
        for node, links in step.get("check_links", {}).items():
            got = sorted(ad.links(node))
            assert got == sorted(links), (case["name"], node, got, links)
        for node, ovl in step.get("check_overloaded", {}).items():
            assert ad.overloaded(node) == ovl, (case["name"], node)
        for chk in step.get("checks", []):
            _check(chk, ad, latest, case)
    for chk in case["checks"]:
        _check(chk, ad, latest, case)


def _check(chk: dict, ad, dbs, case) -> None:
    where = (case["name"], chk.get("cite"))
    t = chk["type"]
    if t == "spf":
        res = ad.spf(chk["src"], chk["use_link_metric"])
        for node, exp in chk["expect"].items():
            assert node in res, (where, "missing", node)
            assert res[node]["metric"] == exp["metric"], (where, node, res[node], exp)
            assert sorted(res[node]["nextHops"]) == exp["nextHops"], (where, node, res[node], exp)
        if chk["exact_keys"]:
            assert sorted(res) == sorted(chk["expect"]), (where, sorted(res))
    elif t == "kth":
        paths = ad.kth(chk["src"], chk["dst"], chk["k"])
        assert len(paths) == chk["n_paths"], (where, paths)
        assert sorted(len(p) for p in paths) == sorted(chk["sizes"]), (where, paths)
        if "first_link_metric_from_src" in chk:
            assert _metric_from(dbs, paths[0][0], chk["src"]) == chk["first_link_metric_from_src"]
        if "path_metric" in chk:
            for p in paths:
                assert _path_metric(dbs, p, chk["src"]) == chk["path_metric"], (where, p)
        if "disjoint_with_k" in chk:
            seen = set()
            allp = list(paths)
            for k in chk["disjoint_with_k"]:
                allp += ad.kth(chk["src"], chk["dst"], k)
            for p in allp:
                for link in p:
                    key = tuple(link)
                    assert key not in seen, (where, "not edge-disjoint", key)
                    seen.add(key)
    elif t == "kth_first_hop_ifaces":
        paths = ad.kth(chk["src"], chk["dst"], chk["k"])
        src = chk["src"]
        ifaces = sorted(p[0][1] if p[0][0] == src else p[0][3] for p in paths)
        assert ifaces == sorted(chk["expect"]), (where, ifaces)
    elif t == "hops":
        assert ad.hops(chk["a"], chk["b"]) == chk["expect"], where
    elif t == "max_hops":
        assert ad.max_hops(chk["node"]) == chk["expect"], where
    elif t == "spf_runs_all_nodes":
        # getRouteMap over every node on a fresh LinkState (memo empty)
        fresh = ad.fresh()
        before = fresh.spf_runs()
        for n in sorted(dbs):
            fresh.spf(n, True)
        assert fresh.spf_runs() - before == chk["expect"], (where, fresh.spf_runs() - before)
    elif t == "ksp2_runs_all_pairs":
        # like getRouteMap for KSP2_ED_ECMP prefixes: per node, k=1 and k=2 to
        # every other node; memoised k=1 SPFs are already counted above
        nodes = sorted(dbs)
        fresh = ad.fresh()
        before = fresh.spf_runs()
        for s in nodes:
            for d in nodes:
                if s != d:
                    fresh.kth(s, d, 1)
                    fresh.kth(s, d, 2)
        assert fresh.spf_runs() - before == chk["expect"], (where, fresh.spf_runs() - before)
    elif t == "grid_manhattan":
        n = chk["n"]
        for s in range(n * n):
            res = ad.spf(str(s), True)
            assert len(res) == n * n, where
            for d in range(n * n):
                md = abs(s % n - d % n) + abs(s // n - d // n)
                assert res[str(d)]["metric"] == md, (where, s, d)
    elif t == "routes":
        labels = {n: db.nodeLabel for n, db in dbs.items()}
        for me, exp in chk["expect"].items():
            got = ad.routes(me, chk["lfa"], chk["v4"], labels)
            for key, rows in exp.items():
                assert got.get(key) == sorted(rows, key=str), (where, me, key, got.get(key), rows)
    elif t == "ksp2_routes":
        for me, exp in chk["expect"].items():
            got = ad.ksp2_routes(me, chk["v4"])
            for dst, rows in exp.items():
                assert got.get(dst) == rows, (where, me, dst, got.get(dst), rows)
    elif t == "ksp2_route_build_spf_runs":
        fresh = ad.fresh()
        before = fresh.spf_runs()
        for n in chk["nodes"]:
            fresh.ksp2_route_build(n)
        assert fresh.spf_runs() - before == chk["expect"], (where, fresh.spf_runs() - before)
    else:
        raise AssertionError(f"unknown check {t}")
