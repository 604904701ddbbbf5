"""LSDB wire ingest: thrift CompactProtocol adjacency databases and KvStore
publications, decoded by libopenr_spf.so (include/openr_wire.h,
csrc/lsdb_wire.cpp).

Mirrors what the reference's Decision does with a publication
(openr/decision/Decision.cpp:1709-1817): ``"adj:"`` values are read with
``readThriftObjStr<thrift::AdjacencyDatabase>(value, CompactSerializer)``
(:1743-1745), their area set to the publication's, expired ``"adj:"`` keys
delete the node's database.  ``LinkState.processPublication`` applies one.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List

import numpy as np

from . import _native as N
from .lsdb import ADJ_DTYPE, DB_DTYPE, Adjacency, AdjacencyDatabase, PackedLsdb


@dataclass
class DecodedPublication:
    """The link-state part of one thrift::Publication."""

    area: str
    adjacencyDbs: List[AdjacencyDatabase] = field(default_factory=list)
    expiredNodes: List[str] = field(default_factory=list)
    skipped: int = 0  # "adj:" values that failed to decode (logged and skipped)
    packed: PackedLsdb | None = None


def _err(status: int) -> None:
    N.raise_for(status, (N.lib.openr_wire_last_error() or b"").decode())


def _packed(h) -> PackedLsdb:
    v = N.lib.openr_wire_view(h).contents
    n_db = int(v.n_dbs)
    dbs = np.ctypeslib.as_array(C.cast(v.dbs, C.POINTER(C.c_uint8)), (n_db * DB_DTYPE.itemsize,)
                                ).view(DB_DTYPE).copy() if n_db else np.zeros(0, DB_DTYPE)
    n_adj = int(dbs["adj_begin"][-1] + dbs["adj_count"][-1]) if n_db else 0
    adjs = np.ctypeslib.as_array(C.cast(v.adjs, C.POINTER(C.c_uint8)), (n_adj * ADJ_DTYPE.itemsize,)
                                 ).view(ADJ_DTYPE).copy() if n_adj else np.zeros(0, ADJ_DTYPE)
    blob_len = 0
    for name in ("name", "area"):
        if n_db:
            blob_len = max(blob_len, int((dbs[f"{name}_off"] + dbs[f"{name}_len"]).max()))
    for name in ("other", "if", "oif"):
        if n_adj:
            blob_len = max(blob_len, int((adjs[f"{name}_off"] + adjs[f"{name}_len"]).max()))
    # the blob pointer itself (the c_char_p field would copy up to a NUL)
    blob_ptr = C.c_void_p.from_buffer(v, N.OpenrLsdb.blob.offset).value
    blob = C.string_at(blob_ptr, blob_len) if blob_len else b""
    return PackedLsdb(blob + b"\0", dbs, adjs)


def unpack(p: PackedLsdb) -> List[AdjacencyDatabase]:
    """PackedLsdb -> AdjacencyDatabase objects."""
    s = lambda off, ln: p.blob[int(off): int(off) + int(ln)].decode("utf-8", "surrogateescape")  # noqa: E731
    out = []
    for d in p.dbs:
        adjs = []
        for a in p.adjs[int(d["adj_begin"]): int(d["adj_begin"] + d["adj_count"])]:
            adjs.append(Adjacency(
                otherNodeName=s(a["other_off"], a["other_len"]), ifName=s(a["if_off"], a["if_len"]),
                nextHopV6=bytes(a["nh_v6"]), nextHopV4=bytes(a["nh_v4"]), metric=int(a["metric"]),
                adjLabel=int(a["adj_label"]), isOverloaded=bool(a["is_overloaded"]),
                rtt=int(a["rtt"]), timestamp=int(a["timestamp"]), weight=int(a["weight"]),
                otherIfName=s(a["oif_off"], a["oif_len"])))
        out.append(AdjacencyDatabase(
            thisNodeName=s(d["name_off"], d["name_len"]), isOverloaded=bool(d["is_overloaded"]),
            adjacencies=adjs, nodeLabel=int(d["node_label"]), area=s(d["area_off"], d["area_len"])))
    return out


def decode_adjacency_database(buf: bytes) -> AdjacencyDatabase:
    """``readThriftObjStr<thrift::AdjacencyDatabase>`` (CompactSerializer)."""
    h = C.c_void_p()
    _err(N.lib.openr_wire_decode_adjdb(buf, len(buf), C.byref(h)))
    try:
        return unpack(_packed(h))[0]
    finally:
        N.lib.openr_wire_free(h)


def decode_publication(buf: bytes) -> DecodedPublication:
    """The link-state half of ``Decision::processPublication``'s parsing."""
    h = C.c_void_p()
    _err(N.lib.openr_wire_decode_publication(buf, len(buf), C.byref(h)))
    try:
        packed = _packed(h)
        return DecodedPublication(
            area=N.lib.openr_wire_area(h).decode(),
            adjacencyDbs=unpack(packed),
            expiredNodes=[N.lib.openr_wire_expired(h, i).decode()
                          for i in range(N.lib.openr_wire_n_expired(h))],
            skipped=int(N.lib.openr_wire_n_skipped(h)),
            packed=packed)
    finally:
        N.lib.openr_wire_free(h)
