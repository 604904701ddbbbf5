"""LinkState drop-in: the reference's ``openr::LinkState`` API over the MI355X engine.

Python mirror of ``openr/decision/LinkState.h:82-469`` (same method names,
argument meaning and error behaviour) backed by the C-ABI facade
``include/openr_linkstate.h``: LSDB bookkeeping on the host, every shortest
path batch on the GPU.  Parity tests drive this class exactly like the
reference's ``LinkStateTest.cpp`` / ``DecisionTest.cpp`` drive the C++ one.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from collections.abc import Mapping
from typing import Dict, Iterable, List, Optional, Sequence, Set, Tuple, Union

from . import _native as N
from .lsdb import K_DEFAULT_AREA, AdjacencyDatabase, PackedLsdb, pack

LinkStateMetric = int


@dataclass(frozen=True)
class LinkStateChange:
    """``LinkState::LinkStateChange`` (LinkState.h:306-325)."""

    topologyChanged: bool = False
    linkAttributesChanged: bool = False
    nodeLabelChanged: bool = False


class Link:
    """Snapshot of ``openr::Link`` (LinkState.h:82-175) taken at query time."""

    __slots__ = ("_n1", "_n2", "_if1", "_if2", "_m1", "_m2", "_l1", "_l2",
                 "_o1", "_o2", "_up", "hash", "_key", "_area", "_v4", "_v6")

    def __init__(self, ls: "LinkState", d: N.LsLinkDesc, link_id: int = -1) -> None:
        name = ls._name
        self._n1, self._n2 = name(d.node1), name(d.node2)
        self._if1, self._if2 = d.if1.decode(), d.if2.decode()
        self._m1, self._m2 = int(d.metric1), int(d.metric2)
        self._l1, self._l2 = int(d.adj_label1), int(d.adj_label2)
        self._o1, self._o2 = bool(d.overload1), bool(d.overload2)
        self._up = bool(d.is_up)
        self.hash = int(d.hash)
        self._key = tuple(sorted([(self._n1, self._if1), (self._n2, self._if2)]))
        self._area = ls.getArea()
        self._v4 = (bytes(d.nh_v4_1[:4]), bytes(d.nh_v4_2[:4]))
        self._v6 = (bytes(d.nh_v6_1[:16]), bytes(d.nh_v6_2[:16]))

    def _side(self, node: str) -> int:
        if node == self._n1:
            return 0
        if node == self._n2:
            return 1
        raise ValueError(node)  # std::invalid_argument in the reference

    def getArea(self) -> str:
        return self._area

    def getOtherNodeName(self, node: str) -> str:
        return self._n2 if self._side(node) == 0 else self._n1

    def firstNodeName(self) -> str:
        return self._key[0][0]

    def secondNodeName(self) -> str:
        return self._key[1][0]

    def getIfaceFromNode(self, node: str) -> str:
        return (self._if1, self._if2)[self._side(node)]

    def getMetricFromNode(self, node: str) -> int:
        return (self._m1, self._m2)[self._side(node)]

    def getAdjLabelFromNode(self, node: str) -> int:
        return (self._l1, self._l2)[self._side(node)]

    def getOverloadFromNode(self, node: str) -> bool:
        return (self._o1, self._o2)[self._side(node)]

    def getNhV4FromNode(self, node: str) -> bytes:
        return self._v4[self._side(node)]

    def getNhV6FromNode(self, node: str) -> bytes:
        return self._v6[self._side(node)]

    def isUp(self) -> bool:
        return self._up

    @property
    def orderedNames(self) -> Tuple[Tuple[str, str], Tuple[str, str]]:
        return self._key  # type: ignore[return-value]

    def __eq__(self, other: object) -> bool:
        return isinstance(other, Link) and self.hash == other.hash and self._key == other._key

    def __lt__(self, other: "Link") -> bool:  # Link::operator< (LinkState.cpp:347-353)
        if self.hash != other.hash:
            return self.hash < other.hash
        return self._key < other._key

    def __hash__(self) -> int:
        return self.hash

    def toString(self) -> str:
        return f"{self._area} - {self._n1}%{self._if1} <---> {self._n2}%{self._if2}"

    def directionalToString(self, fromNode: str) -> str:
        other = self.getOtherNodeName(fromNode)
        return (f"{self._area} - {fromNode}%{self.getIfaceFromNode(fromNode)} ---> "
                f"{other}%{self.getIfaceFromNode(other)}")

    def __repr__(self) -> str:
        return f"Link({self.toString()})"


@dataclass(frozen=True)
class PathLink:
    """``NodeSpfResult::PathLink`` (LinkState.h:207-213)."""

    link: Link
    prevNode: str


class NodeSpfResult:
    """``LinkState::NodeSpfResult`` (LinkState.h:203-257)."""

    __slots__ = ("_metric", "_nh", "_pl")

    def __init__(self, metric: int, nh: Set[str], pl) -> None:
        # pl: the list, or a callable building it on first use (pathLinks are
        # derived only for the callers that read them)
        self._metric, self._nh, self._pl = metric, nh, pl

    def metric(self) -> int:
        return self._metric

    def nextHops(self) -> Set[str]:
        return self._nh

    def pathLinks(self) -> List[PathLink]:
        if callable(self._pl):
            self._pl = self._pl()
        return self._pl

    def __repr__(self) -> str:
        return f"NodeSpfResult(metric={self._metric}, nextHops={sorted(self._nh)})"


SpfResult = Dict[str, NodeSpfResult]
Path = List[Link]


def _change(c: N.LsChange) -> LinkStateChange:
    return LinkStateChange(bool(c.topology_changed), bool(c.link_attributes_changed),
                           bool(c.node_label_changed))


class _LazySpfResult(Mapping):
    """SpfResult (unordered_map<string, NodeSpfResult>) backed by numpy
    copies of the C-ABI view; a NodeSpfResult is built when first read.
    Like the reference's ``SpfResult const&`` into the memo, it is valid until
    the next topology change: link ids are resolved lazily through the
    LinkState's link table, so reading an unmaterialised entry after the
    topology changed raises instead of naming the wrong links."""

    def __init__(self, ls: "LinkState", v: "N.LsSpfView", key=None) -> None:
        import numpy as np

        def arr(ptr, n, dt):
            return np.ctypeslib.as_array(ptr, (n,)).astype(dt) if n else np.zeros(0, dt)

        n = int(v.n)
        self._ls = ls
        self._gen = ls._gen
        self._key = key
        self._node = arr(v.node, n, np.uint32)
        self._metric = arr(v.metric, n, np.uint64)
        self._nh_ptr = arr(v.nh_ptr, n + 1, np.uint32)
        self._nh_node = arr(v.nh_node, int(self._nh_ptr[-1]) if n else 0, np.uint32)
        self._pl_ptr = None
        if v.pl_ptr:
            self._take_pl(v)
        self._index: Optional[Dict[str, int]] = None
        self._made: Dict[str, NodeSpfResult] = {}

    def _take_pl(self, v) -> None:
        import numpy as np

        n = len(self._node)
        self._pl_ptr = np.ctypeslib.as_array(v.pl_ptr, (n + 1,)).astype(np.uint32) if n else np.zeros(1, np.uint32)
        m = int(self._pl_ptr[-1]) if n else 0
        self._pl_link = np.ctypeslib.as_array(v.pl_link, (m,)).astype(np.uint32) if m else np.zeros(0, np.uint32)
        self._pl_prev = np.ctypeslib.as_array(v.pl_prev, (m,)).astype(np.uint32) if m else np.zeros(0, np.uint32)

    def _path_links(self, i: int) -> List[PathLink]:
        ls = self._ls
        if ls._gen != self._gen:
            raise RuntimeError("SpfResult read after a topology change: call getSpfResult again")
        if self._pl_ptr is None:  # the same memo entry, its pathLinks now (spf_runs unchanged)
            self._take_pl(ls._spf_view(*self._key))
        a, b = int(self._pl_ptr[i]), int(self._pl_ptr[i + 1])
        return [PathLink(ls._link(int(l)), ls._name(int(p)))
                for l, p in zip(self._pl_link[a:b], self._pl_prev[a:b])]

    def _idx(self) -> Dict[str, int]:
        if self._index is None:
            name = self._ls._name
            self._index = {name(int(x)): i for i, x in enumerate(self._node)}
        return self._index

    def __getitem__(self, key: str) -> NodeSpfResult:
        r = self._made.get(key)
        if r is None:
            ls = self._ls
            if ls._gen != self._gen:
                raise RuntimeError("SpfResult read after a topology change: call getSpfResult again")
            i = self._idx()[key]
            a, b = int(self._nh_ptr[i]), int(self._nh_ptr[i + 1])
            nh = {ls._name(int(x)) for x in self._nh_node[a:b]}
            r = self._made[key] = NodeSpfResult(int(self._metric[i]), nh, lambda i=i: self._path_links(i))
        return r

    def __iter__(self):
        return iter(self._idx())

    def __len__(self) -> int:
        return len(self._node)

    def __contains__(self, key: object) -> bool:
        return key in self._idx()


class LinkState(N.NativeHandle):
    """``openr::LinkState`` (LinkState.h:177-469) on the MI355X engine.

    ``device`` selects the GPU; ``device=-1`` builds a host-only state (LSDB
    bookkeeping and graph flatten, no shortest-path queries).  ``close()``
    (or a ``with`` block) releases the engine context it owns.
    """

    _LEVEL = 1
    _destroy = "ls_destroy"

    def __init__(self, area: str = K_DEFAULT_AREA, device: int = 0,
                 devices: Optional[Sequence[int]] = None) -> None:
        h = C.c_void_p()
        if devices:  # several GPUs behind one state (ls_create_multi)
            ids = (C.c_int * len(devices))(*[int(d) for d in devices])
            st = N.lib.ls_create_multi(area.encode(), ids, len(devices), C.byref(h))
        else:
            st = N.lib.ls_create(area.encode(), device, C.byref(h))
        N.raise_for(st, N.global_error())
        self._adopt(h)
        self._area = area
        self._names: List[Optional[str]] = []
        self._gen = 0
        self._spf_cache: Dict[Tuple[str, bool], SpfResult] = {}
        self._ksp_cache: Dict[Tuple[str, str, int], List[Path]] = {}
        self._link_cache: Dict[int, Link] = {}

    # -- helpers ---------------------------------------------------------------
    def _err(self, st: int) -> None:
        N.raise_for(st, (N.lib.ls_last_error(self._h) or b"").decode())

    def _name(self, i: int) -> str:
        while i >= len(self._names):
            self._names.append(None)
        s = self._names[i]
        if s is None:
            s = N.lib.ls_name(self._h, i).decode()
            self._names[i] = s
        return s

    def _topology(self, changes: Iterable[LinkStateChange]) -> None:
        if any(c.topologyChanged for c in changes):
            self._gen += 1
            self._spf_cache.clear()
            self._ksp_cache.clear()
            self._link_cache.clear()

    def _link(self, link_id: int) -> Link:
        lk = self._link_cache.get(link_id)
        if lk is None:
            d = N.LsLinkDesc()
            self._err(N.lib.ls_link_info(self._h, link_id, C.byref(d)))
            lk = Link(self, d, link_id)
            self._link_cache[link_id] = lk
        return lk

    # -- mutators (LinkState.h:327-337) -----------------------------------------
    def updateAdjacencyDatabase(self, adjacencyDb: AdjacencyDatabase, holdUpTtl: int = 0,
                                holdDownTtl: int = 0) -> LinkStateChange:
        return self.updateAdjacencyDatabases([adjacencyDb], holdUpTtl, holdDownTtl)[0]

    def updateAdjacencyDatabases(self, dbs: Union[PackedLsdb, Sequence[AdjacencyDatabase]],
                                 holdUpTtl: int = 0, holdDownTtl: int = 0
                                 ) -> List[LinkStateChange]:
        """Apply databases in order (one updateAdjacencyDatabase each)."""
        packed = dbs if isinstance(dbs, PackedLsdb) else pack(dbs)
        s = N.lsdb_struct(packed)
        out = (N.LsChange * max(1, len(packed)))()
        self._err(N.lib.ls_update_adjacency_databases(self._h, C.byref(s), holdUpTtl,
                                                      holdDownTtl, out))
        res = [_change(out[i]) for i in range(len(packed))]
        self._link_cache.clear()  # attributes may have changed
        self._topology(res)
        return res

    def processPublication(self, publication: bytes,
                           orderedFibNode: Optional[str] = None) -> LinkStateChange:
        """The link-state half of ``Decision::processPublication``
        (Decision.cpp:1709-1817) for this area: a serialized
        thrift::Publication (CompactProtocol); every ``"adj:"`` value is
        decoded and applied (in the reference's keyVals iteration order),
        every expired ``"adj:"`` key deletes its node's database.  With
        ``orderedFibNode`` (this node's name, enable_ordered_fib_programming)
        each database carries the hold-up / hold-down TTLs of
        Decision.cpp:1750-1758.  Returns the OR of the steps'
        LinkStateChanges; the counts of applied / deleted databases land in
        ``lastPublicationCounts``."""
        nu, nd, c = C.c_uint32(), C.c_uint32(), N.LsChange()
        st = N.lib.ls_apply_publication_ordered(
            self._h, publication, len(publication),
            orderedFibNode.encode() if orderedFibNode is not None else None, C.byref(nu),
            C.byref(nd), C.byref(c))
        N.raise_for(st, (N.lib.openr_wire_last_error() or b"").decode())
        self.lastPublicationCounts = (int(nu.value), int(nd.value))
        res = _change(c)
        self._link_cache.clear()
        self._topology([res])
        return res

    def deleteAdjacencyDatabase(self, nodeName: str) -> LinkStateChange:
        c = N.LsChange()
        self._err(N.lib.ls_delete_adjacency_database(self._h, nodeName.encode(), C.byref(c)))
        res = _change(c)
        self._link_cache.clear()
        self._topology([res])
        return res

    def decrementHolds(self) -> LinkStateChange:
        c = N.LsChange()
        self._err(N.lib.ls_decrement_holds(self._h, C.byref(c)))
        res = _change(c)
        self._link_cache.clear()
        self._topology([res])
        return res

    # -- const queries -----------------------------------------------------------
    def getArea(self) -> str:
        return self._area

    def hasHolds(self) -> bool:
        return bool(N.lib.ls_has_holds(self._h))

    def numLinks(self) -> int:
        return int(N.lib.ls_num_links(self._h))

    def numNodes(self) -> int:
        return int(N.lib.ls_num_nodes(self._h))

    def hasNode(self, nodeName: str) -> bool:
        return bool(N.lib.ls_has_node(self._h, nodeName.encode()))

    def isNodeOverloaded(self, nodeName: str) -> bool:
        return bool(N.lib.ls_is_node_overloaded(self._h, nodeName.encode()))

    def getAdjacencyDatabaseLabels(self) -> Dict[str, int]:
        """{node: nodeLabel} of every node with an adjacency database -- the
        part of getAdjacencyDatabases() (LinkState.h:357-359) SpfSolver reads."""
        cnt = C.c_uint32()
        self._err(N.lib.ls_adjacency_databases(self._h, None, None, 0, C.byref(cnt)))
        ids = (C.c_uint32 * max(1, cnt.value))()
        labels = (C.c_int32 * max(1, cnt.value))()
        self._err(N.lib.ls_adjacency_databases(self._h, ids, labels, cnt.value, C.byref(cnt)))
        return {self._name(ids[i]): int(labels[i]) for i in range(cnt.value)}

    def linksFromNode(self, nodeName: str) -> List[Link]:
        """Links of ``nodeName`` in the reference's LinkSet iteration order."""
        cnt = C.c_uint32()
        self._err(N.lib.ls_links_from_node(self._h, nodeName.encode(), None, 0, C.byref(cnt)))
        ids = (C.c_uint32 * max(1, cnt.value))()
        self._err(N.lib.ls_links_from_node(self._h, nodeName.encode(), ids, cnt.value,
                                           C.byref(cnt)))
        return [self._link(ids[i]) for i in range(cnt.value)]

    def spfRuns(self) -> int:
        """The reference's ``decision.spf_runs`` counter (LinkState.cpp:815)."""
        return int(N.lib.ls_spf_runs(self._h))

    # -- shortest paths ----------------------------------------------------------
    def getSpfResult(self, nodeName: str, useLinkMetric: bool = True) -> SpfResult:
        """``getSpfResult`` (LinkState.cpp:793-803): a read-only mapping node
        name -> NodeSpfResult over the C-ABI's result arrays (copied once);
        entries are materialised on access, pathLinks on the first
        ``pathLinks()`` of the result (ls_get_spf_metrics now, the same memo
        entry's pathLinks from ls_get_spf_result then: one spf_runs count)."""
        key = (nodeName, bool(useLinkMetric))
        hit = self._spf_cache.get(key)
        if hit is not None:
            return hit
        v = N.LsSpfView()  # metrics and next hops now, pathLinks when first read
        self._err(N.lib.ls_get_spf_metrics(self._h, nodeName.encode(), int(bool(useLinkMetric)),
                                           C.byref(v)))
        res = _LazySpfResult(self, v, key)
        self._spf_cache[key] = res
        return res

    def _spf_view(self, nodeName: str, useLinkMetric: bool = True) -> "N.LsSpfView":
        """The raw C-ABI result (ls_get_spf_result): arrays owned by the
        LinkState's memo, valid until the next topology change."""
        v = N.LsSpfView()
        self._err(N.lib.ls_get_spf_result(self._h, nodeName.encode(), int(bool(useLinkMetric)),
                                          C.byref(v)))
        return v

    def getKthPaths(self, src: str, dest: str, k: int) -> List[Path]:
        key = (src, dest, int(k))
        hit = self._ksp_cache.get(key)
        if hit is not None:
            return hit
        if k < 1:
            raise ValueError("getKthPaths: k must be >= 1")
        v = N.LsPathsView()
        self._err(N.lib.ls_get_kth_paths(self._h, src.encode(), dest.encode(), k, C.byref(v)))
        paths = [[self._link(v.link[j]) for j in range(v.path_ptr[p], v.path_ptr[p + 1])]
                 for p in range(v.n_paths)]
        self._ksp_cache[key] = paths
        return paths

    def prefetchKthPaths(self, src: str) -> None:
        """Fill the getKthPaths memo for (src, *, 1) and (src, *, 2) with one
        batched KSP2 launch (ls_prefetch_kth_paths)."""
        self._err(N.lib.ls_prefetch_kth_paths(self._h, src.encode()))

    def prefetchSpfResults(self, nodes: Sequence[str], useLinkMetric: bool = True) -> None:
        """Fill the getSpfResult memo for every node of `nodes` with one
        batched plan (ls_prefetch_spf_results); spfRuns() counts each when it
        is first read, as the reference's one-by-one calls would."""
        arr = (C.c_char_p * max(1, len(nodes)))(*[n.encode() for n in nodes])
        self._err(N.lib.ls_prefetch_spf_results(self._h, arr, len(nodes), int(bool(useLinkMetric))))

    def prefetchAllSources(self, useLinkMetric: bool = True) -> None:
        """getSpfResult for every node as one all-sources pass split over the
        state's GPUs (ls_prefetch_all_sources; needs ``devices=[...]``):
        results stay on their GPU and later getSpfResult(node) calls read
        node's share from it -- Decision::getDecisionRouteDb for every node
        (Decision.cpp:1480-1500)."""
        self._err(N.lib.ls_prefetch_all_sources(self._h, int(bool(useLinkMetric))))

    def allSourcesDigests(self):
        """Per-node digests (csr order) of the resident all-sources pass, on
        the owning GPUs (spf_mplan_digest); None when no pass is valid."""
        import numpy as np

        mp = N.lib.ls_all_sources_plan(self._h)
        if not mp:
            return None
        n = C.c_uint32()
        e = C.c_uint32()
        self._err(N.lib.ls_flatten(self._h, C.byref(n), C.byref(e)))
        out = np.zeros(max(1, n.value), np.uint64)
        st = N.lib.spf_mplan_digest(C.c_void_p(mp), N.ptr(out, C.c_uint64))
        N.raise_for(st, N.global_error())
        return out[: n.value]

    def linkValueHashes(self):
        """u64 value identity of every link id of the flattened graph (FNV-1a
        over its ordered key, bench.link_value_hash's definition), for the
        engine's route / KSP2 digests; cached until the topology changes."""
        import numpy as np

        lid = self._csr_link_ids()
        # keyed on the flattened graph's epoch: a link id freed and reused by
        # another link changes the structure, hence the epoch
        key = int(N.lib.ls_graph_epoch(self._h))
        if getattr(self, "_lh_key", None) == key and self._lh is not None:
            return self._lh
        lh = np.zeros(max(1, int(lid.max()) + 1 if len(lid) else 1), np.uint64)
        M, P = (1 << 64) - 1, 0x100000001b3
        for l in np.unique(lid):
            try:
                (a, b), (c, d) = self._link(int(l)).orderedNames
            except N.SpfError:  # a withdrawn link's dead slots: never a result
                continue
            f = 0xcbf29ce484222325
            for part in (a, b, c, d):
                for ch in part.encode():
                    f = ((f ^ ch) * P) & M
                f = ((f ^ 0x01) * P) & M
            f = ((f ^ (f >> 30)) * 0xbf58476d1ce4e5b9) & M
            f = ((f ^ (f >> 27)) * 0x94d049bb133111eb) & M
            lh[int(l)] = f ^ (f >> 31)
        self._lh, self._lh_key = lh, key
        return lh

    def allSourcesRouteDigests(self, set_ptr, set_nodes, lfa: bool, mes=None):
        """Route selections of every node (or the csr ids in `mes`) towards
        every destination set from the resident all-sources pass
        (spf_mplan_route_digests, needs prefetchAllSources()): per node one
        u64 digest, and the slowest member's kernel ms."""
        import numpy as np

        mp = N.lib.ls_all_sources_plan(self._h)
        if not mp:
            raise RuntimeError("allSourcesRouteDigests: no resident all-sources pass")
        n = self._csr_sizes()[0]
        mes = np.arange(n, dtype=np.uint32) if mes is None else np.ascontiguousarray(mes, np.uint32)
        sp = np.ascontiguousarray(set_ptr, np.uint32)
        sn = np.ascontiguousarray(set_nodes if len(set_nodes) else [0], np.uint32)
        lh = self.linkValueHashes()
        out = np.zeros(max(1, len(mes)), np.uint64)
        ms = C.c_double()
        st = N.lib.spf_mplan_route_digests(C.c_void_p(mp), N.ptr(mes), len(mes), N.ptr(sp), N.ptr(sn),
                                           len(sp) - 1, N.SPF_ROUTE_LFA if lfa else 0,
                                           N.ptr(lh, C.c_uint64), len(lh), N.ptr(out, C.c_uint64),
                                           C.byref(ms))
        N.raise_for(st, N.global_error())
        return out[: len(mes)], ms.value

    def allSourcesRouteRecords(self, set_ptr, set_nodes, lfa: bool, mes=None):
        """Every node's (or the csr ids in `mes`) route database materialised
        on its owning GPU from the resident all-sources pass
        (spf_mplan_route_records): returns (records over every node, the
        slowest member's kernel ms); read one node's with allSourcesRouteDb."""
        import numpy as np

        mp = N.lib.ls_all_sources_plan(self._h)
        if not mp:
            raise RuntimeError("allSourcesRouteRecords: no resident all-sources pass")
        n = self._csr_sizes()[0]
        mes = np.arange(n, dtype=np.uint32) if mes is None else np.ascontiguousarray(mes, np.uint32)
        sp = np.ascontiguousarray(set_ptr, np.uint32)
        sn = np.ascontiguousarray(set_nodes if len(set_nodes) else [0], np.uint32)
        tot, ms = C.c_uint64(), C.c_double()
        st = N.lib.spf_mplan_route_records(C.c_void_p(mp), N.ptr(mes), len(mes), N.ptr(sp), N.ptr(sn),
                                           len(sp) - 1, N.SPF_ROUTE_LFA if lfa else 0, C.byref(tot),
                                           C.byref(ms))
        N.raise_for(st, N.global_error())
        self._db_sets = len(sp) - 1
        return int(tot.value), ms.value

    def allSourcesRouteDb(self, t: int):
        """Node t's (index into the last allSourcesRouteRecords' node list)
        database: (headers [n_sets] u64 = offset | count << 32, records u64 =
        CSR edge | metric << 32)."""
        import numpy as np

        mp = N.lib.ls_all_sources_plan(self._h)
        if not mp:
            raise RuntimeError("allSourcesRouteDb: no resident all-sources pass")
        n = C.c_uint64()
        hdr = np.zeros(max(1, self._db_sets), np.uint64)
        N.raise_for(N.lib.spf_mplan_route_db(C.c_void_p(mp), int(t), N.ptr(hdr, C.c_uint64), None, 0,
                                             C.byref(n)), N.global_error())
        rec = np.zeros(max(1, n.value), np.uint64)
        N.raise_for(N.lib.spf_mplan_route_db(C.c_void_p(mp), int(t), None, N.ptr(rec, C.c_uint64),
                                             n.value, C.byref(n)), N.global_error())
        return hdr[: self._db_sets], rec[: n.value]

    def debugPhaseNs(self) -> Tuple[int, int, int, int]:
        """Cumulative getSpfResult cost (ns): plan build, GPU execute + copy
        back, pathLinks, host assembly (ls_debug_phase_ns)."""
        out = (C.c_uint64 * 4)()
        N.lib.ls_debug_phase_ns(self._h, out)
        return tuple(int(x) for x in out)  # type: ignore[return-value]

    def getMetricFromAToB(self, a: str, b: str, useLinkMetric: bool = True) -> Optional[int]:
        m = C.c_uint64()
        has = C.c_int()
        self._err(N.lib.ls_get_metric_a_to_b(self._h, a.encode(), b.encode(),
                                             int(bool(useLinkMetric)), C.byref(m), C.byref(has)))
        return int(m.value) if has.value else None

    def getHopsFromAToB(self, a: str, b: str) -> Optional[int]:
        return self.getMetricFromAToB(a, b, False)

    def getMaxHopsToNode(self, nodeName: str) -> int:
        m = C.c_uint64()
        self._err(N.lib.ls_get_max_hops_to_node(self._h, nodeName.encode(), C.byref(m)))
        return int(m.value)

    @staticmethod
    def pathAInPathB(a: Sequence, b: Sequence) -> bool:
        """``LinkState::pathAInPathB`` (LinkState.h:395-410) through the C-ABI
        (``ls_path_a_in_path_b``): a is a contiguous run of b.  Links compare
        by value, as the reference's ``*a.at(i) == *b.at(j)`` does
        (Link::operator==, LinkState.cpp:356-361: hash and orderedNames), so
        equal links of different LinkStates, snapshots and ``OwnedLink``s
        match.  Each distinct value gets one integer code for the C-ABI."""
        import numpy as np

        ids: Dict[object, int] = {}

        def enc(p):
            return np.array([ids.setdefault((int(l.hash), l.orderedNames), len(ids))
                             for l in p] or [0], np.uint32)

        ea, eb = enc(a), enc(b)
        return bool(N.lib.ls_path_a_in_path_b(N.ptr(ea), len(a), N.ptr(eb), len(b)))

    # -- batch access to the flattened graph ---------------------------------------
    def _csr_sizes(self):
        """(nodes, directed edges) of the flattened graph, without copying it."""
        n = C.c_uint32()
        e = C.c_uint32()
        self._err(N.lib.ls_flatten(self._h, C.byref(n), C.byref(e)))
        return n.value, e.value

    def _csr_link_ids(self):
        """The flattened graph's link id per CSR edge (no node names)."""
        import numpy as np

        _, e = self._csr_sizes()
        lid = np.zeros(max(1, e), np.uint32)
        self._err(N.lib.ls_graph_csr(self._h, None, None, None, N.ptr(lid), None))
        return lid[:e]

    def flatten(self):
        """(node names in id order, row_ptr, col, metric, link_id, overloaded)."""
        import numpy as np

        n = C.c_uint32()
        e = C.c_uint32()
        self._err(N.lib.ls_flatten(self._h, C.byref(n), C.byref(e)))
        ids = np.zeros(n.value, np.uint32)
        rp = np.zeros(n.value + 1, np.uint32)
        col = np.zeros(max(1, e.value), np.uint32)
        met = np.zeros(max(1, e.value), np.int32)
        lid = np.zeros(max(1, e.value), np.uint32)
        ovl = np.zeros(max(1, n.value), np.uint8)
        if n.value:
            self._err(N.lib.ls_graph_node_names(self._h, N.ptr(ids)))
        self._err(N.lib.ls_graph_csr(self._h, N.ptr(rp), N.ptr(col), N.ptr(met, C.c_int32),
                                     N.ptr(lid), N.ptr(ovl, C.c_uint8)))
        names = [self._name(int(i)) for i in ids]
        return names, rp, col[: e.value], met[: e.value], lid[: e.value], ovl[: n.value]

    def engine_handle(self) -> C.c_void_p:
        return C.c_void_p(N.lib.ls_engine(self._h))


class OwnedLink(N.NativeHandle):
    """A standalone ``openr::Link`` (LinkState.h:82-175) built from two
    adjacencies, as ``Link(area, n1, adj1, n2, adj2)`` (LinkState.cpp:127-186)
    -- the C-ABI ``ls_link_*`` object.  Side accessors raise ValueError for a
    node not on the link (std::invalid_argument in the reference)."""

    _destroy = "ls_link_destroy"

    def __init__(self, area: str, node1: str, adj1, node2: str, adj2) -> None:
        h = C.c_void_p()
        N.raise_for(N.lib.ls_link_create(
            area.encode(), node1.encode(), adj1.ifName.encode(), adj1.metric, adj1.adjLabel,
            int(adj1.isOverloaded), node2.encode(), adj2.ifName.encode(), adj2.metric,
            adj2.adjLabel, int(adj2.isOverloaded), C.byref(h)), "ls_link_create")
        self._adopt(h)
        # orderedNames_ = minmax((n1, if1), (n2, if2)) (LinkState.cpp:127-137)
        self._key = tuple(sorted([(node1, adj1.ifName), (node2, adj2.ifName)]))

    @property
    def orderedNames(self) -> Tuple[Tuple[str, str], Tuple[str, str]]:
        return self._key  # type: ignore[return-value]

    def _side(self, fn, node: str, out):
        if fn(self._h, node.encode(), C.byref(out)) != N.SPF_OK:
            raise ValueError(node)
        return out.value

    def getArea(self) -> str:
        return N.lib.ls_link_area(self._h).decode()

    @property
    def hash(self) -> int:
        return int(N.lib.ls_link_hash(self._h))

    def getOtherNodeName(self, node: str) -> str:
        return self._side(N.lib.ls_link_other_node, node, C.c_char_p()).decode()

    def getIfaceFromNode(self, node: str) -> str:
        return self._side(N.lib.ls_link_iface, node, C.c_char_p()).decode()

    def getMetricFromNode(self, node: str) -> int:
        return int(self._side(N.lib.ls_link_metric, node, C.c_uint64()))

    def getAdjLabelFromNode(self, node: str) -> int:
        return int(self._side(N.lib.ls_link_adj_label, node, C.c_int32()))

    def getOverloadFromNode(self, node: str) -> bool:
        return bool(self._side(N.lib.ls_link_overload, node, C.c_int()))

    def isUp(self) -> bool:
        return bool(N.lib.ls_link_is_up(self._h))

    def setMetricFromNode(self, node: str, metric: int, holdUpTtl: int, holdDownTtl: int) -> bool:
        ch = C.c_int()
        if N.lib.ls_link_set_metric(self._h, node.encode(), metric, holdUpTtl, holdDownTtl,
                                    C.byref(ch)) != N.SPF_OK:
            raise ValueError(node)
        return bool(ch.value)

    def setOverloadFromNode(self, node: str, overload: bool, holdUpTtl: int,
                            holdDownTtl: int) -> bool:
        ch = C.c_int()
        if N.lib.ls_link_set_overload(self._h, node.encode(), int(overload), holdUpTtl,
                                      holdDownTtl, C.byref(ch)) != N.SPF_OK:
            raise ValueError(node)
        return bool(ch.value)

    def __eq__(self, other: object) -> bool:
        return isinstance(other, OwnedLink) and bool(N.lib.ls_link_equal(self._h, other._h))

    def __lt__(self, other: "OwnedLink") -> bool:
        return bool(N.lib.ls_link_less(self._h, other._h))

    def __hash__(self) -> int:  # equal links have equal Link::hash
        return self.hash


class HoldableValue(N.NativeHandle):
    """``openr::HoldableValue<bool>`` / ``<LinkStateMetric>`` (LinkState.h:36-58,
    LinkState.cpp:54-125), the C-ABI ``ls_holdable_*`` object."""

    _destroy = "ls_holdable_destroy"

    def __init__(self, value) -> None:
        self._bool = isinstance(value, bool)
        self._adopt(C.c_void_p(N.lib.ls_holdable_create(int(self._bool), int(value))))

    def value(self):
        v = int(N.lib.ls_holdable_value(self._h))
        return bool(v) if self._bool else v

    def hasHold(self) -> bool:
        return bool(N.lib.ls_holdable_has_hold(self._h))

    def decrementTtl(self) -> bool:
        return bool(N.lib.ls_holdable_decrement_ttl(self._h))

    def updateValue(self, value, holdUpTtl: int, holdDownTtl: int) -> bool:
        return bool(N.lib.ls_holdable_update_value(self._h, int(value), holdUpTtl, holdDownTtl))
