"""Synthetic link-state topologies (workload generators for tests and bench).

* :func:`grid` -- the reference benchmark's n x n grid,
  ``openr/decision/tests/RoutingBenchmarkUtils.cpp:161-240`` (names ``"r*n+c"``,
  ifName ``if_<me>_<nbr>``, metric 1, neighbour order right, left, up, down).
* :func:`decision_test_grid` -- ``DecisionTest.cpp:4206-4256``'s grid
  (ifNames ``0/1``..``0/4``, other neighbour order).
* :func:`fabric` -- the reference DC fabric, ``RoutingBenchmarkUtils.cpp:247-400``
  (8 planes x 36 SSW, pods of 8 FSW + 48 RSW).  ``full=False`` reproduces the
  reference generator exactly, including its per-pod ``emplace`` quirk
  (``createSswsAdjacencies`` keeps only pod 0's adjacency per SSW,
  ``:261-271``); ``full=True`` wires every SSW to its plane's FSW in every pod.
* :func:`wan` -- ring + seeded random chords, per-direction metrics U[1,1000].
* :func:`barabasi_albert` -- scale-free graph, m links per new node, metrics U[1,16].

Every generator returns a :class:`Topology` holding a packed LSDB
(``openr_amd.lsdb.PackedLsdb``) plus the plain edge arrays.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from .lsdb import PackedLsdb, pack_fast

K_SSW, K_FSW, K_RSW = 1, 2, 3  # RoutingBenchmarkUtils.h markers
K_SSW_PER_PLANE, K_FSW_PER_POD, K_RSW_PER_POD = 36, 8, 48


@dataclass
class Topology:
    name: str
    nodes: List[str]
    adj_src: np.ndarray  # adjacency k advertised by nodes[adj_src[k]]
    adj_dst: np.ndarray
    metric: np.ndarray
    lsdb: PackedLsdb

    @property
    def n_nodes(self) -> int:
        return len(self.nodes)

    @property
    def n_adjacencies(self) -> int:
        return len(self.adj_src)


def _build(name, nodes, src, dst, metric, if_fmt=None, ifs=None, oifs=None,
           adj_label=None, node_overloaded=None, node_label=None) -> Topology:
    src = np.asarray(src, np.int64)
    dst = np.asarray(dst, np.int64)
    if ifs is None:
        ifs = [if_fmt(nodes[a], nodes[b]) for a, b in zip(src.tolist(), dst.tolist())]
        oifs = [if_fmt(nodes[b], nodes[a]) for a, b in zip(src.tolist(), dst.tolist())]
    packed = pack_fast(nodes, src, dst, ifs, oifs, metric, node_overloaded=node_overloaded,
                       adj_label=adj_label, node_label=node_label)
    return Topology(name, list(nodes), src, dst, np.asarray(metric, np.int32), packed)


def grid(n: int) -> Topology:
    """RoutingBenchmarkUtils.cpp:161-240 (createGridAdjacencys order: c+1, c-1, r-1, r+1)."""
    nodes = [str(i) for i in range(n * n)]
    src, dst = [], []
    for r in range(n):
        for c in range(n):
            me = r * n + c
            for rr, cc in ((r, c + 1), (r, c - 1), (r - 1, c), (r + 1, c)):
                if 0 <= rr < n and 0 <= cc < n:
                    src.append(me)
                    dst.append(rr * n + cc)
    dst_a = np.asarray(dst)
    return _build(f"grid{n}", nodes, src, dst, np.ones(len(src), np.int32),
                  if_fmt=lambda a, b: f"if_{a}_{b}", adj_label=100001 + dst_a)


def decision_test_grid(n: int) -> Topology:
    """DecisionTest.cpp:4206-4256 (addAdj order: j+1 "0/1", i-1 "0/2", j-1 "0/3", i+1 "0/4")."""
    nodes = [str(i) for i in range(n * n)]
    src, dst, ifs, oifs = [], [], [], []
    for i in range(n):
        for j in range(n):
            me = i * n + j
            for ii, jj, a, b in ((i, j + 1, "0/1", "0/3"), (i - 1, j, "0/2", "0/4"),
                                 (i, j - 1, "0/3", "0/1"), (i + 1, j, "0/4", "0/2")):
                if 0 <= ii < n and 0 <= jj < n:
                    src.append(me)
                    dst.append(ii * n + jj)
                    ifs.append(a)
                    oifs.append(b)
    return _build(f"dtgrid{n}", nodes, src, dst, np.ones(len(src), np.int32), ifs=ifs,
                  oifs=oifs, adj_label=100001 + np.asarray(dst),
                  node_label=np.arange(1, n * n + 1))  # createAdjDb(name, adjs, node + 1)


def fabric(num_sws: int = 10000, full: bool = True,
           ssw_per_plane: int = K_SSW_PER_PLANE, fsw_per_pod: int = K_FSW_PER_POD,
           rsw_per_pod: int = K_RSW_PER_POD) -> Topology:
    """RoutingBenchmarkUtils.cpp:247-400, 574-630 (BM_DecisionFabric sizing)."""
    planes = fsw_per_pod
    pods = (num_sws - planes * ssw_per_plane) // (fsw_per_pod + rsw_per_pod)
    nodes: List[str] = []
    index = {}

    def nid(marker, pod, sw):
        key = (marker, pod, sw)
        if key not in index:
            index[key] = len(nodes)
            nodes.append(f"{marker}-{pod}-{sw}")
        return index[key]

    src, dst, label = [], [], []

    def adj(me, marker, pod, sw):
        src.append(me)
        dst.append(nid(marker, pod, sw))
        label.append(marker * 100000 + pod * 100 + sw)  # getId()

    for plane in range(planes):
        for i in range(ssw_per_plane):
            me = nid(K_SSW, plane, i)
            for pod in (range(pods) if full else range(1)):
                adj(me, K_FSW, pod, plane)
    for pod in range(pods):
        for j in range(fsw_per_pod):
            me = nid(K_FSW, pod, j)
            for i in range(ssw_per_plane):
                adj(me, K_SSW, j, i)
            for k in range(rsw_per_pod):
                adj(me, K_RSW, pod, k)
    for pod in range(pods):
        for k in range(rsw_per_pod):
            me = nid(K_RSW, pod, k)
            for j in range(fsw_per_pod):
                adj(me, K_FSW, pod, j)
    return _build(("fabric_full" if full else "fabric_ref") + str(num_sws), nodes, src, dst,
                  np.ones(len(src), np.int32), if_fmt=lambda a, b: f"if_{a}_{b}",
                  adj_label=np.asarray(label))


def fabric_rtt(seed: int = 7, num_sws: int = 10000) -> Topology:
    """fabric_full wiring with per-direction metrics max(rtt/100, 1), the
    RTT-derived metric of LinkMonitor.cpp:44-47; rtt in microseconds drawn
    per adjacency (seeded): intra-pod 40-400 us, pod-to-spine 200-3000 us."""
    topo = fabric(num_sws, full=True)
    rng = np.random.default_rng(seed)
    src, dst = topo.adj_src, topo.adj_dst
    spine = np.array([n.startswith("1-") for n in topo.nodes])
    far = spine[src] | spine[dst]
    rtt = np.where(far, rng.integers(200, 3001, len(src)), rng.integers(40, 401, len(src)))
    metric = np.maximum(rtt // 100, 1).astype(np.int32)
    topo.lsdb.adjs["metric"] = metric
    topo.metric = metric
    topo.name = "fabric_rtt"
    return topo


def _undirected_to_adj(nodes, links, metric_fwd, metric_rev, name):
    links = np.asarray(links, np.int64)
    src = np.concatenate([links[:, 0], links[:, 1]])
    dst = np.concatenate([links[:, 1], links[:, 0]])
    met = np.concatenate([metric_fwd, metric_rev]).astype(np.int32)
    return _build(name, nodes, src, dst, met, if_fmt=lambda a, b: f"if_{a}_{b}")


def wan(n: int = 2000, chords: int = 1000, seed: int = 1, max_metric: int = 1000) -> Topology:
    """Ring of n nodes + `chords` distinct random chords; per-direction metrics
    U[1, max_metric] (numpy PCG64, seeded)."""
    rng = np.random.default_rng(seed)
    nodes = [f"w{i}" for i in range(n)]
    seen = set()
    links = []
    for i in range(n):
        a, b = i, (i + 1) % n
        seen.add((min(a, b), max(a, b)))
        links.append((a, b))
    while len(links) < n + chords:
        a, b = (int(x) for x in rng.integers(0, n, 2))
        if a == b:
            continue
        key = (min(a, b), max(a, b))
        if key in seen:
            continue
        seen.add(key)
        links.append((a, b))
    m = len(links)
    fwd = rng.integers(1, max_metric + 1, m)
    rev = rng.integers(1, max_metric + 1, m)
    return _undirected_to_adj(nodes, links, fwd, rev, f"wan{n}")


def barabasi_albert(n: int = 250_000, m: int = 4, seed: int = 1,
                    max_metric: int = 16) -> Topology:
    """Preferential attachment: each new node links to m distinct earlier nodes
    chosen proportionally to degree (repeated-endpoint list method)."""
    rng = np.random.default_rng(seed)
    nodes = [str(i) for i in range(n)]
    links = []
    targets = list(range(m))
    repeated: List[int] = []
    for v in range(m, n):
        for t in set(targets):
            links.append((v, t))
        repeated.extend(targets)
        repeated.extend([v] * m)
        chosen = set()
        while len(chosen) < m:
            chosen.add(repeated[int(rng.integers(0, len(repeated)))])
        targets = list(chosen)
    k = len(links)
    fwd = rng.integers(1, max_metric + 1, k)
    rev = rng.integers(1, max_metric + 1, k)
    return _undirected_to_adj(nodes, links, fwd, rev, f"ba{n}")


def clique_with_tail(k: int, depth: int) -> Topology:
    """A k-clique with a path of depth - 1 nodes hanging off clique node 0,
    unit metrics: the graph's diameter (deepest BFS level over all sources)
    is exactly `depth` (k >= 2, depth >= 1)."""
    nodes = [f"c{i:02d}" for i in range(k)] + [f"t{i:03d}" for i in range(depth - 1)]
    links = [(a, b) for a in range(k) for b in range(a + 1, k)]
    prev = 0
    for i in range(depth - 1):
        links.append((prev, k + i))
        prev = k + i
    ones = np.ones(len(links), np.int64)
    return _undirected_to_adj(nodes, links, ones, ones, f"clique{k}_tail{depth}")


def random_graph(n: int, n_links: int, seed: int, max_metric: int = 10,
                 parallel_frac: float = 0.0, overload_frac: float = 0.0,
                 link_overload_frac: float = 0.0) -> Topology:
    """Small random multigraph for parity fuzzing: optional parallel links,
    drained nodes and drained links, per-direction metrics U[1, max_metric]."""
    rng = np.random.default_rng(seed)
    nodes = [f"n{i:03d}" if i % 3 else f"{i}" for i in range(n)]
    links = []
    while len(links) < n_links:
        a, b = (int(x) for x in rng.integers(0, n, 2))
        if a == b:
            continue
        links.append((a, b))
        if parallel_frac and rng.random() < parallel_frac:
            links.append((a, b))
    links = np.asarray(links, np.int64)
    k = len(links)
    fwd = rng.integers(1, max_metric + 1, k)
    rev = rng.integers(1, max_metric + 1, k)
    src = np.concatenate([links[:, 0], links[:, 1]])
    dst = np.concatenate([links[:, 1], links[:, 0]])
    met = np.concatenate([fwd, rev]).astype(np.int32)
    # parallel links need distinct interface names: number them per (a, b)
    counter = {}
    ifs, oifs = [], []
    for i in range(k):
        a, b = int(links[i, 0]), int(links[i, 1])
        key = (min(a, b), max(a, b))  # one numbering per unordered pair
        c = counter.get(key, 0)
        counter[key] = c + 1
        ifs.append(f"{nodes[a]}/{nodes[b]}/{c}")
        oifs.append(f"{nodes[b]}/{nodes[a]}/{c}")
    ifs_all = ifs + oifs
    oifs_all = oifs + ifs
    node_ovl = (rng.random(n) < overload_frac).astype(np.int32) if overload_frac else None
    topo = _build(f"rand{n}_{seed}", nodes, src, dst, met, ifs=ifs_all, oifs=oifs_all,
                  node_overloaded=node_ovl)
    if link_overload_frac:
        drain = rng.random(len(topo.lsdb.adjs)) < link_overload_frac
        topo.lsdb.adjs["is_overloaded"] = drain.astype(np.int32)
    return topo
