"""Test infrastructure: a thrift CompactProtocol *encoder* for the LSDB
structs, restated from the published protocol specification (Apache Thrift
`doc/specs/thrift-compact-protocol.md`; fbthrift's CompactProtocol, which the
reference's CompactSerializer uses, writes the same bytes for these types).
fbthrift is not in this image, so bytes produced by the reference's own
serializer are not available: the wire decoder's parity is pinned to the
specification (known-answer vectors in test_wire.py), not to fbthrift output.

Field order follows the IDL declaration order, as thrift generators emit it:
Adjacency writes 1, 2, 3, 5, 4, 6..11 (Lsdb.thrift:71-105) and Value 1, 3, 2,
4, 5, 6 (KvStore.thrift:21-41), so the long field-header form (negative id
delta) is exercised.
"""

from __future__ import annotations

import struct
from typing import Iterable, List, Optional, Sequence, Tuple

BOOL_TRUE, BOOL_FALSE, BYTE, I16, I32, I64, DOUBLE, BINARY, LIST, SET, MAP, STRUCT = range(1, 13)


def varint(n: int) -> bytes:
    assert n >= 0
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def zigzag(n: int, bits: int = 64) -> int:
    return ((n << 1) ^ (n >> (bits - 1))) & ((1 << bits) - 1)


class Writer:
    def __init__(self) -> None:
        self.buf = bytearray()
        self._last: List[int] = [0]

    # ---- structs
    def struct_begin(self) -> None:
        self._last.append(0)

    def struct_end(self) -> None:
        self.buf.append(0)
        self._last.pop()

    def field(self, fid: int, ftype: int) -> None:
        delta = fid - self._last[-1]
        if 0 < delta <= 15:
            self.buf.append((delta << 4) | ftype)
        else:
            self.buf.append(ftype)
            self.buf += varint(zigzag(fid, 16))
        self._last[-1] = fid

    # ---- scalars
    def i32(self, v: int) -> None:
        self.buf += varint(zigzag(v, 32))

    def i64(self, v: int) -> None:
        self.buf += varint(zigzag(v, 64))

    def binary(self, b: bytes | str) -> None:
        if isinstance(b, str):
            b = b.encode()
        self.buf += varint(len(b)) + b

    def double(self, v: float) -> None:
        self.buf += struct.pack("<d", v)

    # ---- fields
    def f_bool(self, fid: int, v: bool) -> None:
        self.field(fid, BOOL_TRUE if v else BOOL_FALSE)

    def f_i32(self, fid: int, v: int) -> None:
        self.field(fid, I32)
        self.i32(v)

    def f_i64(self, fid: int, v: int) -> None:
        self.field(fid, I64)
        self.i64(v)

    def f_binary(self, fid: int, v: bytes | str) -> None:
        self.field(fid, BINARY)
        self.binary(v)

    def list_begin(self, etype: int, n: int) -> None:
        if n < 15:
            self.buf.append((n << 4) | etype)
        else:
            self.buf.append(0xF0 | etype)
            self.buf += varint(n)

    def map_begin(self, ktype: int, vtype: int, n: int) -> None:
        self.buf += varint(n)
        if n:
            self.buf.append((ktype << 4) | vtype)

    def bytes(self) -> bytes:
        return bytes(self.buf)


def _unknown_fields(w: Writer, fid: int) -> None:
    """A field a newer schema might add: a list<string>, a double, a map and a
    nested struct under one id each (the decoder must skip them)."""
    w.field(fid, LIST)
    w.list_begin(BINARY, 2)
    w.binary("x")
    w.binary("yz")
    w.field(fid + 1, DOUBLE)
    w.double(2.5)
    w.field(fid + 2, MAP)
    w.map_begin(BINARY, I64, 1)
    w.binary("k")
    w.i64(-7)
    w.field(fid + 3, STRUCT)
    w.struct_begin()
    w.f_bool(1, True)
    w.f_i32(2, 5)
    w.field(3, LIST)
    w.list_begin(BOOL_TRUE, 3)
    w.buf += bytes([1, 2, 1])
    w.struct_end()


def _address(w: Writer, fid: int, addr: bytes) -> None:
    w.field(fid, STRUCT)
    w.struct_begin()
    w.f_binary(1, addr)
    w.struct_end()


def write_adjacency(w: Writer, a, omit_defaults: bool = False, unknown: bool = False) -> None:
    """thrift::Adjacency (Lsdb.thrift:71-105), IDL field order."""
    w.struct_begin()
    w.f_binary(1, a.otherNodeName)
    w.f_binary(2, a.ifName)
    _address(w, 3, bytes(a.nextHopV6))
    _address(w, 5, bytes(a.nextHopV4))
    w.f_i32(4, a.metric)
    if not (omit_defaults and a.adjLabel == 0):
        w.f_i32(6, a.adjLabel)
    if not (omit_defaults and not a.isOverloaded):
        w.f_bool(7, a.isOverloaded)
    w.f_i32(8, a.rtt)
    w.f_i64(9, a.timestamp)
    if not (omit_defaults and a.weight == 1):
        w.f_i64(10, a.weight)
    if not (omit_defaults and a.otherIfName == ""):
        w.f_binary(11, a.otherIfName)
    if unknown:
        _unknown_fields(w, 40)
    w.struct_end()


def encode_adjacency_database(db, omit_defaults: bool = False, unknown: bool = False,
                              perf_events: bool = False) -> bytes:
    """thrift::AdjacencyDatabase (Lsdb.thrift:109-129) as CompactSerializer
    writes it."""
    w = Writer()
    w.struct_begin()
    w.f_binary(1, db.thisNodeName)
    if not (omit_defaults and not db.isOverloaded):
        w.f_bool(2, db.isOverloaded)
    w.field(3, LIST)
    w.list_begin(STRUCT, len(db.adjacencies))
    for a in db.adjacencies:
        write_adjacency(w, a, omit_defaults, unknown)
    w.f_i32(4, db.nodeLabel)
    if perf_events:  # 5: optional PerfEvents {1: list<PerfEvent>}
        w.field(5, STRUCT)
        w.struct_begin()
        w.field(1, LIST)
        w.list_begin(STRUCT, 1)
        w.struct_begin()
        w.f_binary(1, db.thisNodeName)
        w.f_binary(2, "ADJ_DB_UPDATED")
        w.f_i64(3, 1600000000000)
        w.struct_end()
        w.struct_end()
    if not (omit_defaults and db.area == ""):
        w.f_binary(6, db.area)
    if unknown:
        _unknown_fields(w, 20)
    w.struct_end()
    return w.bytes()


def encode_value(version: int, originator: str, value: Optional[bytes], ttl: int = 3600000,
                 ttl_version: int = 0, hash_: Optional[int] = None) -> bytes:
    """thrift::Value (KvStore.thrift:21-41), field order 1, 3, 2, 4, 5, 6."""
    w = Writer()
    _write_value(w, version, originator, value, ttl, ttl_version, hash_)
    return w.bytes()


def _write_value(w: Writer, version, originator, value, ttl, ttl_version, hash_) -> None:
    w.struct_begin()
    w.f_i64(1, version)
    w.f_binary(3, originator)
    if value is not None:
        w.f_binary(2, value)
    w.f_i64(4, ttl)
    w.f_i64(5, ttl_version)
    if hash_ is not None:
        w.f_i64(6, hash_)
    w.struct_end()


def encode_publication(key_vals: Sequence[Tuple[str, Optional[bytes]]],
                       expired: Iterable[str] = (), area: Optional[str] = "0",
                       node_ids: Sequence[str] = (), flood_root: Optional[str] = None,
                       area_first: bool = False) -> bytes:
    """thrift::Publication (KvStore.thrift:226-247).  key_vals: (key, value
    bytes or None for a TTL-only update)."""
    w = Writer()
    w.struct_begin()
    if area_first and area is not None:  # not IDL order: the decoder must not care
        w.f_binary(7, area)
    w.field(2, MAP)
    w.map_begin(BINARY, STRUCT, len(key_vals))
    for i, (k, v) in enumerate(key_vals):
        w.binary(k)
        _write_value(w, i + 1, "orig", v, 3600000, 0 if v is not None else 1, None)
    exp = list(expired)
    w.field(3, LIST)
    w.list_begin(BINARY, len(exp))
    for k in exp:
        w.binary(k)
    if node_ids:
        w.field(4, LIST)
        w.list_begin(BINARY, len(node_ids))
        for n in node_ids:
            w.binary(n)
    if flood_root is not None:
        w.f_binary(6, flood_root)
    if not area_first and area is not None:
        w.f_binary(7, area)
    w.struct_end()
    return w.bytes()
