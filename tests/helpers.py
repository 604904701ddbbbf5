"""Shared test helpers: fixture builders that mirror the reference's test utils."""

from __future__ import annotations

from typing import Dict, List, Sequence, Tuple, Union

from openr_amd.lsdb import AdjacencyDatabase, create_adj_db, create_adjacency

# libstdc++ _Prime_rehash_policy::_M_next_bkt fast path (hashtable_c++0x.cc)
_FAST_BKT = [2, 2, 2, 3, 5, 5, 7, 7, 11, 11, 11, 11, 13, 13]


def libstdcxx_int_map_order(keys: Sequence[int]) -> List[int]:
    """Iteration order of ``std::unordered_map<int, T>`` built from an
    initializer list holding ``keys`` in this order (libstdc++, identity
    std::hash<int>, max_load_factor 1).  Exact for fewer than 14 keys, where
    the constructor's bucket count (_M_next_bkt fast path) never rehashes."""
    n = len(keys)
    if n >= len(_FAST_BKT):
        raise ValueError("emulation covers maps with < 14 keys")
    nb = _FAST_BKT[n]
    order: List[int] = []
    for k in keys:
        b = k % nb
        idx = next((i for i, x in enumerate(order) if x % nb == b), None)
        # a node goes first in its bucket's run; a new bucket's run goes first
        order.insert(0 if idx is None else idx, k)
    return order


def get_link_state_dbs(
    adj_map: Dict[int, Sequence[Union[int, Tuple[int, int]]]]
) -> List[AdjacencyDatabase]:
    """Adjacency databases in the order ``getLinkState`` applies them
    (reference openr/decision/tests/DecisionTestUtils.cpp:16-44): integer node
    names, ifName ``node/adj/k`` (k-th parallel adjacency), label
    ``(node << 16) + adj``, fe80::/192.168 addresses from the neighbour id."""
    dbs = []
    for node in libstdcxx_int_map_order(list(adj_map.keys())):
        assert node < (1 << 16)
        adjs = []
        num_parallel: Dict[int, int] = {}
        for entry in adj_map[node]:
            adj, weight = (entry, 1) if isinstance(entry, int) else entry
            k = num_parallel.get(adj, 0)
            num_parallel[adj] = k + 1
            bottom, top = adj & 0xFF, (adj & 0xFF00) >> 8
            adjs.append(create_adjacency(
                str(adj), f"{node}/{adj}/{k}", f"{adj}/{node}/{k}",
                f"fe80::{top:02x}{bottom:02x}", f"192.168.{top}.{bottom}", weight,
                (node << 16) + adj))
        dbs.append(create_adj_db(str(node), adjs, node))
    return dbs


def link_key(link) -> list:
    """Canonical [n1, if1, n2, if2] (ordered names) of a product Link."""
    (a, b), (c, d) = link.orderedNames
    return [a, b, c, d]


def spf_canonical(res) -> dict:
    """Product SpfResult -> the oracle's JSON shape."""
    return {
        node: {
            "metric": r.metric(),
            "nextHops": sorted(r.nextHops()),
            "pathLinks": [[link_key(pl.link), pl.prevNode] for pl in r.pathLinks()],
        }
        for node, r in sorted(res.items())
    }


def planar_rows(ks, dist, mats, pitch):
    """Oracle dense results (dist [m, n] u64, mats[i] bool [>= k_i, n]) in the
    engine's plan layout: dist rows u32 padded to `pitch` (unreachable =
    0xFFFFFFFF, padding 0) and next-hop bitmaps, k_i rows of pitch/32 words
    per source, concatenated in source order."""
    import numpy as np

    m, n = dist.shape
    d32 = np.zeros((m, pitch), np.uint32)
    d32[:, :n] = np.where(dist == np.iinfo(np.uint64).max, 0xFFFFFFFF, dist).astype(np.uint32)
    rows = []
    for i in range(m):
        for j in range(int(ks[i])):
            row = np.zeros(pitch, bool)
            row[:n] = mats[i][j]
            rows.append(np.packbits(row, bitorder="little").view(np.uint32))
    nh = np.concatenate(rows) if rows else np.zeros(0, np.uint32)
    return d32, nh


def _mix64(z):
    """splitmix64's finaliser over a uint64 array (wrapping arithmetic)."""
    import numpy as np

    z = np.asarray(z, np.uint64)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


def route_db_digest(hdr, rec, link_id, link_hash) -> int:
    """One node's materialised route database (spf_mplan_route_records:
    headers offset | count << 32, records CSR edge | metric << 32) reduced
    with spf_mplan_route_digests' formula keyed by the smallest next-hop
    metric (oracle route_digests(kept_min=True)): per set p with next hops,
    mix(mix(K (p + 1) + least) + sum mix(link_hash[link] + metric) + p),
    summed over p.  (Without LFA, least == the shortest distance and this is
    the digest kernel's value.)  Also checks each route's next hops are in
    link order."""
    import numpy as np

    hdr = np.asarray(hdr, np.uint64)
    rec = np.asarray(rec, np.uint64)
    off = (hdr & np.uint64(0xFFFFFFFF)).astype(np.int64)
    cnt = (hdr >> np.uint64(32)).astype(np.int64)
    edge = (rec & np.uint64(0xFFFFFFFF)).astype(np.int64)
    met = rec >> np.uint64(32)
    lh = np.asarray(link_hash, np.uint64)
    per = _mix64(lh[np.asarray(link_id, np.int64)[edge]] + met) if len(rec) else np.zeros(0, np.uint64)
    nz = np.nonzero(cnt)[0]
    if len(nz) == 0:
        return 0
    c = cnt[nz]
    seg = np.concatenate([[0], np.cumsum(c)[:-1]])
    idx = np.repeat(off[nz], c) + (np.arange(int(c.sum())) - np.repeat(seg, c))
    assert idx.max() < len(rec), "a route's records run past the node's region"
    e = edge[idx]
    inner = np.ones(len(idx), bool)
    inner[seg] = False
    assert np.all(np.diff(e)[inner[1:]] > 0), "next hops not in link order"
    with np.errstate(over="ignore"):
        sums = np.add.reduceat(per[idx], seg, dtype=np.uint64)
        shortest = np.minimum.reduceat(met[idx], seg)
        p = nz.astype(np.uint64)
        h = _mix64(_mix64(np.uint64(0x9e3779b97f4a7c15) * (p + np.uint64(1)) + shortest) + sums + p)
        total = h.sum(dtype=np.uint64)
    return int(total)
