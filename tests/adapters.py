"""Adapters exposing the oracle and the product LinkState to tests/refcases.py."""

from __future__ import annotations

from typing import Dict, List, Optional

from helpers import link_key, spf_canonical


class _Replay:
    def __init__(self) -> None:
        self.history: list = []

    def fresh(self):
        other = type(self)()
        for op, arg in self.history:
            getattr(other, op)(arg)
        return other


class OracleAdapter(_Replay):
    def __init__(self) -> None:
        super().__init__()
        from oracle import OracleLinkState, spf_runs

        self.ls = OracleLinkState()
        self._runs = spf_runs

    def update(self, dbs) -> List[tuple]:
        self.history.append(("update", dbs))
        return self.ls.update(dbs)

    def update_packed(self, packed):
        self.history.append(("update_packed", packed))
        return self.ls.update_packed(packed)

    def delete(self, node) -> tuple:
        self.history.append(("delete", node))
        return self.ls.delete(node)

    def links(self, node):
        return [l[0] for l in self.ls.links(node)]

    def overloaded(self, node) -> bool:
        return self.ls.is_overloaded(node)

    def spf(self, src, ulm=True) -> Dict[str, dict]:
        return self.ls.spf(src, ulm)

    def kth(self, src, dst, k):
        return self.ls.kth_paths(src, dst, k)

    def hops(self, a, b) -> Optional[int]:
        return self.ls.metric_a_to_b(a, b, False)

    def max_hops(self, n) -> int:
        return self.ls.max_hops(n)

    def spf_runs(self) -> int:
        return self._runs()


class ProductAdapter(_Replay):
    device = 0

    def __init__(self) -> None:
        super().__init__()
        from openr_amd.link_state import LinkState

        self.ls = LinkState(device=self.device)

    @staticmethod
    def _chg(c) -> tuple:
        return (c.topologyChanged, c.linkAttributesChanged, c.nodeLabelChanged)

    def update(self, dbs):
        self.history.append(("update", dbs))
        return [self._chg(c) for c in self.ls.updateAdjacencyDatabases(dbs)]

    def update_packed(self, packed):
        self.history.append(("update_packed", packed))
        return [self._chg(c) for c in self.ls.updateAdjacencyDatabases(packed)]

    def delete(self, node):
        self.history.append(("delete", node))
        return self._chg(self.ls.deleteAdjacencyDatabase(node))

    def links(self, node):
        return [link_key(l) for l in self.ls.linksFromNode(node)]

    def overloaded(self, node):
        return self.ls.isNodeOverloaded(node)

    def spf(self, src, ulm=True):
        return spf_canonical(self.ls.getSpfResult(src, ulm))

    def kth(self, src, dst, k):
        return [[link_key(l) for l in p] for p in self.ls.getKthPaths(src, dst, k)]

    def hops(self, a, b):
        return self.ls.getHopsFromAToB(a, b)

    def max_hops(self, n):
        return self.ls.getMaxHopsToNode(n)

    def spf_runs(self):
        return self.ls.spfRuns()


class HostOnlyProductAdapter(ProductAdapter):
    """Product LinkState without a GPU: LSDB bookkeeping only."""

    device = -1
