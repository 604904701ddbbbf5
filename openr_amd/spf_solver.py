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

  * SR_MPLS forwarding (selectBestPathsSpf with perDestination, :829-893 and
    the push-label branch of getNextHopsThrift :1260-1290) over the memoised
    SPF results of me (and, with LFA, of every neighbour);
  * KSP2_ED_ECMP (selectBestPathsKsp2 :895-1018):
    k = 1 / k = 2 edge-disjoint paths to every advertiser from ONE batched
    KSP2 launch (LinkState.prefetchKthPaths -> ls_prefetch_kth_paths), the
    anycast filter LinkState.pathAInPathB, label stacks with PHP and prepend
    labels;
  * addBestPaths (:1020-1080): min-nexthop threshold, static next hops of a
    self-advertised prefix with a prepend label.

Not covered yet (raise NotImplementedError): multiple areas, BGP / best-route
selection by PrefixMetrics.
"""

from __future__ import annotations

import ctypes as C
from collections import deque
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
    minNexthop: Optional[int] = None

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


# enum values of OpenrConfig.thrift:77-85 (getPrefixForwardingTypeAndAlgorithm
# takes the minimum over the best entries)
_FWD_TYPE = {"IP": 0, "SR_MPLS": 1}
_FWD_ALGO = {"SP_ECMP": 0, "KSP2_ED_ECMP": 1}


def getPrefixForwardingTypeAndAlgorithm(entries: Dict[Tuple[str, str], "PrefixEntry"],
                                        best: Set[Tuple[str, str]]) -> Tuple[str, str]:
    """openr/common/Util.cpp:617-643."""
    if not entries:
        return "IP", "SP_ECMP"
    t, a = 1, 1
    for na, e in entries.items():
        if na not in best:
            continue
        t = min(t, _FWD_TYPE[e.forwardingType])
        a = min(a, _FWD_ALGO[e.forwardingAlgorithm])
        if t == 0 and a == 0:
            break
    return ("IP", "SR_MPLS")[t], ("SP_ECMP", "KSP2_ED_ECMP")[a]


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
        self.bgpDryRun = bgpDryRun
        self.staticMplsRoutes: Dict[int, List[NextHopThrift]] = {}
        if enableBestRouteSelection:
            raise NotImplementedError("best route selection by PrefixMetrics")

    def updateStaticMplsRoutes(self, routesToUpdate: Dict[int, List[NextHopThrift]],
                               routesToDelete: Sequence[int] = ()) -> None:
        """SpfSolver::updateStaticMplsRoutes (Decision.cpp): label -> next hops."""
        for label, nhs in routesToUpdate.items():
            self.staticMplsRoutes[label] = list(nhs)
        for label in routesToDelete:
            self.staticMplsRoutes.pop(label, None)

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

    # -- SR_MPLS SP_ECMP: getNextHopsWithMetric / getNextHopsThrift with
    #    perDestination = true (Decision.cpp:829-893, 1107-1305) --------------------
    def _srSpfNextHops(self, ls: LinkState, me: str, area: str, best: List[Tuple[str, str]],
                       ents: Dict[Tuple[str, str], PrefixEntry], isV4: bool,
                       labels: Dict[str, int]) -> Set[NextHopThrift]:
        dsts = list(best)
        if any(na[0] == me for na in best):  # :848-857
            for na, e in ents.items():
                if na[0] == me and e.prependLabel is not None:
                    if na in dsts:
                        dsts.remove(na)
                    break
        dstSet = set(dsts)
        mine = ls.getSpfResult(me)
        shortest, minCost = (1 << 64) - 1, set()
        for d, _ in sorted(dsts):  # getMinCostNodes (:1082-1105)
            if d not in mine:
                continue
            m = mine[d].metric()
            if shortest >= m:
                if shortest > m:
                    shortest, minCost = m, set()
                minCost.add(d)
        nextHopNodes: Dict[Tuple[str, str], int] = {}
        for d in minCost:
            for nh in mine[d].nextHops():
                nextHopNodes[(nh, d)] = shortest - ls.getMetricFromAToB(me, nh)
        if self.computeLfaPaths and minCost:
            # me + every neighbour in one batched plan (Decision.cpp:1158-1165)
            ls.prefetchSpfResults([me] + [l.getOtherNodeName(me) for l in ls.linksFromNode(me)
                                          if l.isUp()])
            for link in ls.linksFromNode(me):
                if not link.isUp():
                    continue
                nb = link.getOtherNodeName(me)
                fromNb = ls.getSpfResult(nb)
                nbToHere = fromNb[me].metric()
                for d, a in sorted(dsts):
                    if a != area or d not in fromNb:
                        continue
                    dn = fromNb[d].metric()
                    if dn < shortest + nbToHere:  # RFC 5286 (:1180)
                        key = (nb, d)
                        if key not in nextHopNodes or nextHopNodes[key] > dn:
                            nextHopNodes[key] = dn
        out: Set[NextHopThrift] = set()
        if not nextHopNodes:
            return out
        for link in ls.linksFromNode(me):
            nb = link.getOtherNodeName(me)
            for d, a in sorted(dsts):
                if a != area:
                    continue
                via = nextHopNodes.get((nb, d))
                if via is None or not link.isUp():
                    continue
                if (nb, area) in dstSet and nb != d:
                    continue
                over = link.getMetricFromNode(me) + via
                if not self.computeLfaPaths and over != shortest:
                    continue
                push: List[int] = []
                pe = ents[(d, area)]
                if pe.prependLabel is not None:
                    push.append(pe.prependLabel)
                    if not isMplsLabelValid(push[-1]):
                        continue
                if d != nb:
                    push.append(labels.get(d, 0))
                    if not isMplsLabelValid(push[-1]):
                        continue
                action = MplsAction("PUSH", None, tuple(push)) if push else None
                addr = link.getNhV4FromNode(me) if isV4 else link.getNhV6FromNode(me)
                out.add(createNextHop(addr, link.getIfaceFromNode(me), over, action,
                                      link.getArea(), nb))
        return out

    # -- KSP2_ED_ECMP: selectBestPathsKsp2 (Decision.cpp:895-1018) -------------------
    def _ksp2NextHops(self, ls: LinkState, me: str, area: str, best: List[Tuple[str, str]],
                      ents: Dict[Tuple[str, str], PrefixEntry], isV4: bool,
                      labels: Dict[str, int]) -> Set[NextHopThrift]:
        paths = []
        for node, a in sorted(best):
            if node == me and a == area:
                continue
            paths.extend(ls.getKthPaths(me, node, 1))
        first = len(paths)
        for node, a in sorted(best):
            if a != area:
                continue
            for sec in ls.getKthPaths(me, node, 2):
                # anycast: drop a second path that contains a shortest one
                if not any(LinkState.pathAInPathB(paths[i], sec) for i in range(first)):
                    paths.append(sec)
        out: Set[NextHopThrift] = set()
        for path in paths:
            cost, stack, nxt = 0, deque(), me
            for link in path:
                cost += link.getMetricFromNode(nxt)
                nxt = link.getOtherNodeName(nxt)
                stack.appendleft(labels.get(nxt, 0))
            stack.pop()  # the first hop's label: PHP
            pe = ents[(nxt, area)]
            if pe.prependLabel is not None:
                stack.appendleft(pe.prependLabel)  # bottom of the stack
            head = path[0]
            action = MplsAction("PUSH", None, tuple(stack)) if stack else None
            addr = head.getNhV4FromNode(me) if isV4 else head.getNhV6FromNode(me)
            out.add(createNextHop(addr, head.getIfaceFromNode(me), cost, action, head.getArea(),
                                  head.getOtherNodeName(me)))
        return out

    # -- addBestPaths (Decision.cpp:1020-1080) ---------------------------------------
    def _addBestPaths(self, me: str, prefix: str, best: List[Tuple[str, str]],
                      bestNA: Tuple[str, str], ents: Dict[Tuple[str, str], PrefixEntry],
                      nhs: Set[NextHopThrift]) -> Optional[RibUnicastEntry]:
        need = None
        for na in best:  # getMinNextHopThreshold: the largest minNexthop
            m = ents[na].minNexthop
            if m is not None and (need is None or m > need):
                need = m
        if need is not None and need > len(nhs):
            return None  # min-nexthop requirement not met
        if any(na[0] == me for na in best):
            prepend = next((e.prependLabel for na, e in ents.items()
                            if na[0] == me and e.prependLabel is not None), None)
            assert prepend is not None, "self route must carry a prepend label"
            nhs = set(nhs)
            for nh in self.staticMplsRoutes.get(prepend, []):
                nhs.add(createNextHop(nh.address, None, 0, None))
        return RibUnicastEntry(prefix, nhs, ents[bestNA], bestNA[1])

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
        labels = ls.getAdjacencyDatabaseLabels()
        uni: List[Tuple[str, Dict[Tuple[str, str], PrefixEntry], List[str], Tuple[str, str]]] = []
        sr: List[Tuple[str, Dict[Tuple[str, str], PrefixEntry], List[Tuple[str, str]],
                       Tuple[str, str], str]] = []
        for prefix, entries in prefixState.prefixes().items():
            ents = {na: e for na, e in entries.items() if na[1] == area and na[0] in mine}
            if not ents:
                continue  # no reachable advertiser
            isV4 = next(iter(ents.values())).isV4
            if isV4 and not self.enableV4:
                continue
            if any(e.type == "BGP" for e in ents.values()):
                raise NotImplementedError("BGP prefixes / metric-vector selection")
            # openr routes: every advertiser is best (selectBestRoutes), the
            # best node-area the first of them; drop drained ones unless all
            # are (maybeFilterDrainedNodes :766-789 -- which keeps the
            # unfiltered bestNodeArea)
            allNA = sorted(ents)
            bestNA = allNA[0]
            best = [na for na in allNA if not ls.isNodeOverloaded(na[0])] or allNA
            hasSelfPrepend = all(e.prependLabel is not None
                                 for na, e in ents.items() if na[0] == me)
            if any(na[0] == me for na in best) and not hasSelfPrepend:
                continue  # self-advertised
            ftype, falgo = getPrefixForwardingTypeAndAlgorithm(ents, set(best))
            if falgo == "SP_ECMP" and ftype == "IP":
                uni.append((prefix, ents, [na[0] for na in best], bestNA))
            else:
                sr.append((prefix, ents, best, bestNA, falgo))

        # ---- node labels (collisions: Decision.cpp:605-617) ----
        label_to_node: Dict[int, str] = {}
        for node, label in labels.items():
            if label == 0 or not isMplsLabelValid(label):
                continue
            prev = label_to_node.get(label)
            if prev is not None and prev < node:
                continue
            label_to_node[label] = node

        sets = [dsts for _, _, dsts, _ in uni] + [[n] for n in label_to_node.values()]
        sel = self._select(ls, me, sets)

        for (prefix, ents, dsts, bestNA), res in zip(uni, sel[: len(uni)]):
            if not res.hops:
                continue  # no route to prefix
            isV4 = next(iter(ents.values())).isV4
            nhs = self._next_hops(ls, me, area, res, isV4, set(dsts), None)
            r = self._addBestPaths(me, prefix, [(d, area) for d in dsts], bestNA, ents, nhs)
            if r is not None:
                db.addUnicastRoute(r)

        # ---- SR_MPLS prefixes: per-destination SP_ECMP or KSP2_ED_ECMP ----
        if any(falgo == "KSP2_ED_ECMP" for *_, falgo in sr):
            ls.prefetchKthPaths(me)  # one batched KSP2 launch for every advertiser
        for prefix, ents, best, bestNA, falgo in sr:
            isV4 = next(iter(ents.values())).isV4
            if falgo == "KSP2_ED_ECMP":
                if any(ents[na].forwardingType != "SR_MPLS" for na in best):
                    continue  # incompatible forwarding type (Decision.cpp:905-913)
                nhs = self._ksp2NextHops(ls, me, area, best, ents, isV4, labels)
            else:
                nhs = self._srSpfNextHops(ls, me, area, best, ents, isV4, labels)
            if not nhs:
                continue  # no route to prefix
            r = self._addBestPaths(me, prefix, best, bestNA, ents, nhs)
            if r is not None:
                db.addUnicastRoute(r)

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
