"""SpfSolver drop-in: the route computation that consumes LinkState's SPF
results (reference ``openr/decision/Decision.cpp`` SpfSolver::SpfSolverImpl).

Covered, single area, over the MI355X engine:
  * ``buildRouteDb`` (:557-722): unicast routes for every prefix of the
    PrefixState (SP_ECMP, IP forwarding), node-label MPLS routes (POP for our
    own label, SWAP/PHP towards every other node, label collisions resolved
    as :605-617 does) and adjacency-label routes (PHP over each of our links);
  * ``createRouteForPrefix`` (:390-555): reachable advertisers, v4 sanity,
    openr (non-BGP) best-route selection = every advertiser, drained
    advertisers filtered (maybeFilterDrainedNodes :766-789), self-advertised
    prefixes skipped;
  * ``getMinCostNodes`` / ``getNextHopsWithMetric`` (with LFA) /
    ``getNextHopsThrift`` (:1082-1305): ONE batched call ``spf_routes``
    (include/openr_spf.h) for all prefixes and node labels of a route build --
    one SPF plan for me (+ every neighbour with LFA) and a next-hop selection
    kernel, one wavefront per destination set.

Not covered yet (raise NotImplementedError): multiple areas, BGP / best-route
selection by PrefixMetrics, SR_MPLS forwarding and KSP2_ED_ECMP prefixes
(SURVEY.md §8(f) rank 3).
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, FrozenSet, List, Optional, Sequence, Set, Tuple

import numpy as np

from . import _native as N
from .link_state import LinkState

MPLS_LABEL_MIN, MPLS_LABEL_MAX = 0, (1 << 20) - 1
Metric = int


def isMplsLabelValid(label: int) -> bool:
    """openr/common/Util.h isMplsLabelValid: 20-bit label space."""
    return MPLS_LABEL_MIN <= label <= MPLS_LABEL_MAX


@dataclass(frozen=True)
class MplsAction:
    """thrift::MplsAction (openr/if/Network.thrift)."""

    action: str  # "PUSH" | "SWAP" | "PHP" | "POP_AND_LOOKUP"
    swapLabel: Optional[int] = None
    pushLabels: Optional[Tuple[int, ...]] = None


@dataclass(frozen=True)
class NextHopThrift:
    """thrift::NextHopThrift (Network.thrift:65-86) as built by createNextHop
    (openr/common/Util.cpp:907-922): metric is an i32."""

    address: bytes
    ifName: Optional[str]
    metric: int
    mplsAction: Optional[MplsAction]
    area: Optional[str]
    neighborNodeName: Optional[str]


def createNextHop(addr: bytes, ifName: Optional[str], metric: int,
                  mplsAction: Optional[MplsAction] = None, area: Optional[str] = None,
                  neighborNodeName: Optional[str] = None) -> NextHopThrift:
    m = metric & 0xFFFFFFFF
    return NextHopThrift(bytes(addr), ifName, m - (1 << 32) if m >= 1 << 31 else m, mplsAction,
                         area, neighborNodeName)


@dataclass
class PrefixEntry:
    """The fields of thrift::PrefixEntry (Lsdb.thrift) route building reads."""

    prefix: str
    type: str = "LOOPBACK"
    forwardingType: str = "IP"
    forwardingAlgorithm: str = "SP_ECMP"
    prependLabel: Optional[int] = None

    @property
    def isV4(self) -> bool:
        return ":" not in self.prefix


class PrefixState:
    """prefix -> {(node, area): PrefixEntry} (openr/decision/PrefixState.h)."""

    def __init__(self) -> None:
        self._p: Dict[str, Dict[Tuple[str, str], PrefixEntry]] = {}

    def updatePrefix(self, node: str, area: str, entry: PrefixEntry) -> None:
        self._p.setdefault(entry.prefix, {})[(node, area)] = entry

    def deletePrefix(self, node: str, area: str, prefix: str) -> None:
        ent = self._p.get(prefix)
        if ent is not None:
            ent.pop((node, area), None)
            if not ent:
                del self._p[prefix]

    def prefixes(self) -> Dict[str, Dict[Tuple[str, str], PrefixEntry]]:
        return self._p


@dataclass
class RibUnicastEntry:
    prefix: str
    nexthops: Set[NextHopThrift]
    bestPrefixEntry: PrefixEntry
    bestArea: str
    doNotInstall: bool = False


@dataclass
class RibMplsEntry:
    label: int
    nexthops: Set[NextHopThrift]


@dataclass
class DecisionRouteDb:
    unicastRoutes: Dict[str, RibUnicastEntry] = field(default_factory=dict)
    mplsRoutes: Dict[int, RibMplsEntry] = field(default_factory=dict)

    def addUnicastRoute(self, r: RibUnicastEntry) -> None:
        self.unicastRoutes[r.prefix] = r

    def addMplsRoute(self, r: RibMplsEntry) -> None:
        self.mplsRoutes[r.label] = r


@dataclass
class _SetResult:
    min_metric: Optional[int]
    hops: List[Tuple[int, int]]  # (directed edge me -> neighbour, metric)


class SpfSolver:
    """``openr::SpfSolver`` (Decision.h) on the MI355X engine."""

    def __init__(self, myNodeName: str, enableV4: bool, computeLfaPaths: bool,
                 enableOrderedFib: bool = False, bgpDryRun: bool = False,
                 enableBestRouteSelection: bool = False) -> None:
        self.myNodeName = myNodeName
        self.enableV4 = enableV4
        self.computeLfaPaths = computeLfaPaths
        if enableBestRouteSelection:
            raise NotImplementedError("best route selection by PrefixMetrics")

    # -- batched next-hop selection (getMinCostNodes/..WithMetric/..Thrift) ----
    def _select(self, ls: LinkState, me: str, sets: Sequence[Sequence[str]]) -> List[_SetResult]:
        names, rp, col, met, lid, ovl = ls.flatten()
        id_of = {n: i for i, n in enumerate(names)}
        if me not in id_of or not sets:
            return [_SetResult(None, []) for _ in sets]
        ptr = np.zeros(len(sets) + 1, np.uint32)
        members: List[int] = []
        for i, s in enumerate(sets):
            members.extend(id_of[d] for d in s if d in id_of)
            ptr[i + 1] = len(members)
        nodes = np.asarray(members if members else [0], np.uint32)
        m = id_of[me]
        deg = max(1, int(rp[m + 1] - rp[m]))
        mins = np.zeros(len(sets), np.uint64)
        cnt = np.zeros(len(sets), np.uint32)
        edge = np.zeros(len(sets) * deg, np.uint32)
        metric = np.zeros(len(sets) * deg, np.uint64)
        st = N.lib.spf_routes(ls.engine_handle(), m, N.ptr(ptr), N.ptr(nodes), len(sets),
                              N.SPF_ROUTE_LFA if self.computeLfaPaths else 0,
                              N.ptr(mins, C.c_uint64), N.ptr(cnt), N.ptr(edge),
                              N.ptr(metric, C.c_uint64))
        if st != N.SPF_OK:
            N.raise_for(st, (N.lib.spf_last_error(ls.engine_handle()) or b"").decode())
        out = []
        for i in range(len(sets)):
            mm = int(mins[i])
            hops = [(int(edge[i * deg + t]), int(metric[i * deg + t])) for t in range(int(cnt[i]))]
            out.append(_SetResult(None if mm == (1 << 64) - 1 else mm, hops))
        self._lid = lid
        return out

    def _next_hops(self, ls: LinkState, me: str, area: str, res: _SetResult, isV4: bool,
                   dsts: Set[str], swapLabel: Optional[int]) -> Set[NextHopThrift]:
        """getNextHopsThrift (Decision.cpp:1198-1305) from the kernel's
        (link, metric) selection."""
        out: Set[NextHopThrift] = set()
        for e, metric in res.hops:
            link = ls._link(int(self._lid[e]))
            nb = link.getOtherNodeName(me)
            action = None
            if swapLabel is not None:
                also_dst = nb in dsts
                action = MplsAction("PHP") if also_dst else MplsAction("SWAP", swapLabel)
            addr = link.getNhV4FromNode(me) if isV4 else link.getNhV6FromNode(me)
            out.add(createNextHop(addr, link.getIfaceFromNode(me), metric, action,
                                  link.getArea(), nb))
        return out

    # -- buildRouteDb (Decision.cpp:557-722) ----------------------------------------
    def buildRouteDb(self, myNodeName: str, areaLinkStates: Dict[str, LinkState],
                     prefixState: PrefixState) -> Optional[DecisionRouteDb]:
        if len(areaLinkStates) != 1:
            raise NotImplementedError("multi-area route computation")
        (area, ls), = areaLinkStates.items()
        if not ls.hasNode(myNodeName):
            return None
        me = myNodeName
        db = DecisionRouteDb()
        mine = ls.getSpfResult(me)  # memoised: reachability for prefix filtering

        # ---- unicast: destination set per prefix (createRouteForPrefix) ----
        uni: List[Tuple[str, Dict[Tuple[str, str], PrefixEntry], List[str]]] = []
        for prefix, entries in prefixState.prefixes().items():
            ents = {na: e for na, e in entries.items() if na[1] == area and na[0] in mine}
            if not ents:
                continue  # no reachable advertiser
            isV4 = next(iter(ents.values())).isV4
            if isV4 and not self.enableV4:
                continue
            if any(e.type == "BGP" for e in ents.values()):
                raise NotImplementedError("BGP prefixes / metric-vector selection")
            if any(e.forwardingType != "IP" or e.forwardingAlgorithm != "SP_ECMP"
                   for e in ents.values()):
                raise NotImplementedError("SR_MPLS / KSP2_ED_ECMP forwarding")
            # openr routes: every advertiser is best; drop drained ones unless
            # all are (maybeFilterDrainedNodes)
            best = sorted(ents)
            undrained = [na for na in best if not ls.isNodeOverloaded(na[0])]
            best = undrained or best
            hasSelfPrepend = all(e.prependLabel is not None
                                 for na, e in ents.items() if na[0] == me)
            if any(na[0] == me for na in best) and not hasSelfPrepend:
                continue  # self-advertised
            uni.append((prefix, ents, [na[0] for na in best]))

        # ---- node labels (collisions: Decision.cpp:605-617) ----
        labels = ls.getAdjacencyDatabaseLabels()
        label_to_node: Dict[int, str] = {}
        for node, label in labels.items():
            if label == 0 or not isMplsLabelValid(label):
                continue
            prev = label_to_node.get(label)
            if prev is not None and prev < node:
                continue
            label_to_node[label] = node

        sets = [dsts for _, _, dsts in uni] + [[n] for n in label_to_node.values()]
        sel = self._select(ls, me, sets)

        for (prefix, ents, dsts), res in zip(uni, sel[: len(uni)]):
            if not res.hops:
                continue  # no route to prefix
            isV4 = next(iter(ents.values())).isV4
            bestNA = (sorted(dsts)[0], area)
            nhs = self._next_hops(ls, me, area, res, isV4, set(dsts), None)
            db.addUnicastRoute(RibUnicastEntry(prefix, nhs, ents[bestNA], area))

        for (label, node), res in zip(label_to_node.items(), sel[len(uni):]):
            if node == me:
                db.addMplsRoute(RibMplsEntry(label, {NextHopThrift(
                    bytes(16), None, 0, MplsAction("POP_AND_LOOKUP"), area, None)}))
                continue
            if not res.hops:
                continue  # no route to node label
            db.addMplsRoute(RibMplsEntry(label, self._next_hops(
                ls, me, area, res, False, {node}, label)))

        # ---- adjacency labels (Decision.cpp:682-707) ----
        for link in ls.linksFromNode(me):
            top = link.getAdjLabelFromNode(me)
            if top == 0 or not isMplsLabelValid(top):
                continue
            db.addMplsRoute(RibMplsEntry(top, {createNextHop(
                link.getNhV6FromNode(me), link.getIfaceFromNode(me),
                link.getMetricFromNode(me), MplsAction("PHP"), link.getArea(),
                link.getOtherNodeName(me))}))
        return db

    def getNextHops(self, ls: LinkState, me: str, dsts: Sequence[str], isV4: bool = False,
                    swapLabel: Optional[int] = None) -> Tuple[Optional[int], Set[NextHopThrift]]:
        """(min metric, next hops) of one destination set: getNextHopsWithMetric
        + getNextHopsThrift with perDestination = false."""
        res = self._select(ls, me, [list(dsts)])[0]
        area = ls.getArea()
        return res.min_metric, self._next_hops(ls, me, area, res, isV4, set(dsts), swapLabel)

    def getNextHopsBatch(self, ls: LinkState, me: str, sets: Sequence[Sequence[str]],
                         isV4: bool = False) -> List[Tuple[Optional[int], Set[NextHopThrift]]]:
        res = self._select(ls, me, sets)
        area = ls.getArea()
        return [(r.min_metric, self._next_hops(ls, me, area, r, isV4, set(s), None))
                for r, s in zip(res, sets)]
