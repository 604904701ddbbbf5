"""Link-state database (LSDB) input types and their packed wire layout.

Python mirrors of the reference's thrift input schema for the SPF path
(reference ``openr/if/Lsdb.thrift:71-129``):

* :class:`Adjacency`          -- ``thrift::Adjacency``
* :class:`AdjacencyDatabase`  -- ``thrift::AdjacencyDatabase``

and of the fixture helpers in ``openr/common/Util.cpp:727-793``
(:func:`create_adjacency`, :func:`create_thrift_adjacency`,
:func:`create_adj_db`).

Across the C-ABI an LSDB travels *packed* (``include/openr_lsdb.h``): one
byte blob holding every string, a table of fixed-size database records and a
table of fixed-size adjacency records.  :func:`pack` builds that layout with
numpy so 10k-node fabrics (≈230k adjacencies) pack in well under a second.
"""

from __future__ import annotations

import ipaddress
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence

import numpy as np

K_DEFAULT_AREA = "0"  # openr/if/KvStore.thrift:18
K_DEFAULT_ADJ_WEIGHT = 1  # Constants::kDefaultAdjWeight

# -- packed record layouts (must match include/openr_lsdb.h) -----------------
DB_DTYPE = np.dtype(
    [
        ("name_off", "<u4"), ("name_len", "<u4"),
        ("area_off", "<u4"), ("area_len", "<u4"),
        ("is_overloaded", "<i4"), ("node_label", "<i4"),
        ("adj_begin", "<u4"), ("adj_count", "<u4"),
    ]
)
ADJ_DTYPE = np.dtype(
    [
        ("other_off", "<u4"), ("other_len", "<u4"),
        ("if_off", "<u4"), ("if_len", "<u4"),
        ("oif_off", "<u4"), ("oif_len", "<u4"),
        ("metric", "<i4"), ("adj_label", "<i4"),
        ("is_overloaded", "<i4"), ("rtt", "<i4"),
        ("timestamp", "<i8"), ("weight", "<i8"),
        ("nh_v6", "u1", (16,)), ("nh_v4", "u1", (4,)), ("pad", "u1", (4,)),
    ]
)
assert DB_DTYPE.itemsize == 32 and ADJ_DTYPE.itemsize == 80


def _addr_bytes(addr: str | bytes, width: int) -> bytes:
    if isinstance(addr, (bytes, bytearray)):
        b = bytes(addr)
    elif not addr:
        b = b""
    else:
        b = ipaddress.ip_address(addr).packed
    return b[:width].ljust(width, b"\0")


@dataclass
class Adjacency:
    """``thrift::Adjacency`` (Lsdb.thrift:71-105)."""

    otherNodeName: str
    ifName: str
    nextHopV6: bytes = b""
    nextHopV4: bytes = b""
    metric: int = 1
    adjLabel: int = 0
    isOverloaded: bool = False
    rtt: int = 0
    timestamp: int = 0
    weight: int = K_DEFAULT_ADJ_WEIGHT
    otherIfName: str = ""


@dataclass
class AdjacencyDatabase:
    """``thrift::AdjacencyDatabase`` (Lsdb.thrift:109-129)."""

    thisNodeName: str
    isOverloaded: bool = False
    adjacencies: List[Adjacency] = field(default_factory=list)
    nodeLabel: int = 0
    area: str = K_DEFAULT_AREA


def create_thrift_adjacency(
    nodeName: str,
    ifName: str,
    nextHopV6: str,
    nextHopV4: str,
    metric: int,
    adjLabel: int,
    isOverloaded: bool,
    rtt: int,
    timestamp: int,
    weight: int,
    remoteIfName: str,
) -> Adjacency:
    """Mirror of ``createThriftAdjacency`` (openr/common/Util.cpp:727-751)."""
    return Adjacency(
        otherNodeName=nodeName,
        ifName=ifName,
        nextHopV6=_addr_bytes(nextHopV6, 16),
        nextHopV4=_addr_bytes(nextHopV4, 4),
        metric=metric,
        adjLabel=adjLabel,
        isOverloaded=isOverloaded,
        rtt=rtt,
        timestamp=timestamp,
        weight=weight,
        otherIfName=remoteIfName,
    )


def create_adjacency(
    nodeName: str,
    ifName: str,
    remoteIfName: str,
    nextHopV6: str,
    nextHopV4: str,
    metric: int,
    adjLabel: int,
    weight: int = K_DEFAULT_ADJ_WEIGHT,
) -> Adjacency:
    """Mirror of ``createAdjacency`` (openr/common/Util.cpp:753-776).

    The reference stamps ``timestamp`` with wall-clock seconds; it takes no
    part in SPF, so a constant is used to keep fixtures reproducible.
    """
    return create_thrift_adjacency(
        nodeName, ifName, nextHopV6, nextHopV4, metric, adjLabel, False,
        metric * 100, 0, weight, remoteIfName,
    )


def create_adj_db(
    nodeName: str,
    adjs: Sequence[Adjacency],
    nodeLabel: int,
    overLoadBit: bool = False,
    area: str = K_DEFAULT_AREA,
) -> AdjacencyDatabase:
    """Mirror of ``createAdjDb`` (openr/common/Util.cpp:778-793)."""
    return AdjacencyDatabase(
        thisNodeName=nodeName,
        isOverloaded=overLoadBit,
        adjacencies=list(adjs),
        nodeLabel=nodeLabel,
        area=area,
    )


class _Blob:
    def __init__(self) -> None:
        self._parts: List[bytes] = []
        self._len = 0
        self._memo: dict = {}

    def add(self, s: str) -> tuple:
        hit = self._memo.get(s)
        if hit is not None:
            return hit
        b = s.encode()
        ref = (self._len, len(b))
        self._parts.append(b)
        self._len += len(b)
        self._memo[s] = ref
        return ref

    def bytes(self) -> bytes:
        return b"".join(self._parts) + b"\0"


@dataclass
class PackedLsdb:
    """The packed LSDB layout of ``include/openr_lsdb.h``."""

    blob: bytes
    dbs: np.ndarray  # DB_DTYPE
    adjs: np.ndarray  # ADJ_DTYPE

    def __len__(self) -> int:
        return len(self.dbs)

    def slice(self, i: int, j: int) -> "PackedLsdb":
        """Databases [i, j) (adjacency indices stay global)."""
        return PackedLsdb(self.blob, self.dbs[i:j], self.adjs)


def pack(dbs: Iterable[AdjacencyDatabase]) -> PackedLsdb:
    """Pack adjacency databases into the C-ABI layout."""
    dbs = list(dbs)
    blob = _Blob()
    n_adj = sum(len(d.adjacencies) for d in dbs)
    drec = np.zeros(len(dbs), DB_DTYPE)
    arec = np.zeros(n_adj, ADJ_DTYPE)
    k = 0
    for i, d in enumerate(dbs):
        no, nl = blob.add(d.thisNodeName)
        ao, al = blob.add(d.area)
        drec[i] = (no, nl, ao, al, int(d.isOverloaded), d.nodeLabel, k,
                   len(d.adjacencies))
        for a in d.adjacencies:
            oo, ol = blob.add(a.otherNodeName)
            io, il = blob.add(a.ifName)
            po, pl = blob.add(a.otherIfName)
            r = arec[k]
            r["other_off"], r["other_len"] = oo, ol
            r["if_off"], r["if_len"] = io, il
            r["oif_off"], r["oif_len"] = po, pl
            r["metric"] = a.metric
            r["adj_label"] = a.adjLabel
            r["is_overloaded"] = int(a.isOverloaded)
            r["rtt"] = a.rtt
            r["timestamp"] = a.timestamp
            r["weight"] = a.weight
            r["nh_v6"] = np.frombuffer(_addr_bytes(a.nextHopV6, 16), np.uint8)
            r["nh_v4"] = np.frombuffer(_addr_bytes(a.nextHopV4, 4), np.uint8)
            k += 1
    return PackedLsdb(blob.bytes(), drec, arec)


def pack_fast(
    node_names: Sequence[str],
    adj_src: np.ndarray,
    adj_dst: np.ndarray,
    if_names: Sequence[str],
    other_if_names: Sequence[str],
    metric: np.ndarray,
    node_overloaded: Optional[np.ndarray] = None,
    adj_label: Optional[np.ndarray] = None,
    node_label: Optional[np.ndarray] = None,
    area: str = K_DEFAULT_AREA,
    db_order: Optional[np.ndarray] = None,
) -> PackedLsdb:
    """Vectorised packer for large synthetic topologies.

    ``adj_src[k] -> adj_dst[k]`` is adjacency k, advertised by node
    ``adj_src[k]`` (adjacencies of one node keep their relative order).
    ``db_order`` gives the order in which node databases are emitted
    (default: node index order).
    """
    n = len(node_names)
    adj_src = np.asarray(adj_src, np.int64)
    adj_dst = np.asarray(adj_dst, np.int64)
    m = len(adj_src)
    order = np.argsort(adj_src, kind="stable")
    blob = _Blob()
    name_ref = np.array([blob.add(s) for s in node_names], np.uint32).reshape(n, 2)
    if_ref = np.array([blob.add(s) for s in if_names], np.uint32).reshape(m, 2)
    oif_ref = np.array([blob.add(s) for s in other_if_names], np.uint32).reshape(m, 2)
    area_ref = blob.add(area)
    arec = np.zeros(m, ADJ_DTYPE)
    arec["other_off"] = name_ref[adj_dst[order], 0]
    arec["other_len"] = name_ref[adj_dst[order], 1]
    arec["if_off"] = if_ref[order, 0]
    arec["if_len"] = if_ref[order, 1]
    arec["oif_off"] = oif_ref[order, 0]
    arec["oif_len"] = oif_ref[order, 1]
    arec["metric"] = np.asarray(metric, np.int32)[order]
    if adj_label is not None:
        arec["adj_label"] = np.asarray(adj_label, np.int32)[order]
    arec["rtt"] = arec["metric"] * 100
    arec["weight"] = 1
    counts = np.bincount(adj_src, minlength=n)
    begins = np.concatenate([[0], np.cumsum(counts)[:-1]])
    drec = np.zeros(n, DB_DTYPE)
    drec["name_off"] = name_ref[:, 0]
    drec["name_len"] = name_ref[:, 1]
    drec["area_off"], drec["area_len"] = area_ref
    if node_overloaded is not None:
        drec["is_overloaded"] = np.asarray(node_overloaded, np.int32)
    drec["node_label"] = (
        np.asarray(node_label, np.int32) if node_label is not None
        else np.arange(1, n + 1, dtype=np.int32)
    )
    drec["adj_begin"] = begins
    drec["adj_count"] = counts
    if db_order is not None:
        drec = drec[np.asarray(db_order)]
    return PackedLsdb(blob.bytes(), drec, arec)
