"""LSDB wire ingest (include/openr_wire.h, csrc/lsdb_wire.cpp): thrift
CompactProtocol adjacency databases and KvStore publications, decoded on the
host -- no device needed.

Parity: fbthrift is not in this image, so no byte string produced by the
reference's CompactSerializer is available.  The decoder is pinned to the
protocol specification instead: hand-assembled known-answer vectors (each
byte annotated), plus round trips through tests/thrift_compact.py, an
independent encoder restated from the spec.  The semantics of a publication
(which keys are link state, TTL-only updates, expired keys, the node-name
check, area) follow Decision::processPublication (Decision.cpp:1709-1817).
"""

import numpy as np
import pytest

from openr_amd import _native as N
from openr_amd import topology as T
from openr_amd.link_state import LinkState
from openr_amd.lsdb import Adjacency, AdjacencyDatabase, pack
from openr_amd.wire import decode_adjacency_database, decode_publication
from thrift_compact import encode_adjacency_database, encode_publication


def test_known_answer_adjacency_database():
    """thrift::AdjacencyDatabase{thisNodeName="a", isOverloaded=true,
    adjacencies=[Adjacency{otherNodeName="b", ifName="i1", metric=-3,
    otherIfName="i2"}], nodeLabel=300}, assembled by hand from the spec."""
    buf = bytes([
        0x18, 0x01, ord("a"),          # field 1 (delta 1), binary, len 1, "a"
        0x11,                          # field 2 (delta 1), bool true
        0x19, 0x1C,                    # field 3 (delta 1), list: 1 element of struct
        0x18, 0x01, ord("b"),          #   Adjacency.1 otherNodeName "b"
        0x18, 0x02, ord("i"), ord("1"),  # .2 ifName "i1"
        0x25, 0x05,                    #   .4 (delta 2) i32 zigzag(-3) = 5
        0x75, 0xA0, 0x9C, 0x01,        #   .11 (delta 7) as an i32: a foreign type, skipped
        0x00,                          #   end Adjacency
        0x15, 0xD8, 0x04,              # field 4 (delta 1), i32 zigzag(300) = 600
        0x00,                          # end
    ])
    db = decode_adjacency_database(buf)
    assert db.thisNodeName == "a" and db.isOverloaded and db.nodeLabel == 300
    assert db.area == ""  # no declared default (Lsdb.thrift:128)
    (a,) = db.adjacencies
    assert (a.otherNodeName, a.ifName, a.metric) == ("b", "i1", -3)
    # field 11 arrived with a foreign type (i32, not string): skipped, default kept
    assert a.otherIfName == "" and a.weight == 1 and a.adjLabel == 0 and not a.isOverloaded


def test_known_answer_long_field_header_and_varints():
    """Field ids going backwards use the long header form (type byte +
    zigzag i16 id); a 200-byte name needs a two-byte length varint; an i64
    weight of 2**40 a six-byte varint."""
    name = "n" * 200
    buf = bytearray()
    buf += bytes([0x08, 0x02]) + bytes([0xC8, 0x01]) + name.encode()  # field 1 long form, len 200
    buf += bytes([0x09, 0x06, 0x1C])  # field 3 long form (zigzag 3 = 6): list of 1 struct
    buf += bytes([0x58, 0x00])  # Adjacency.5 as an empty binary: a foreign type, skipped
    buf += bytes([0x0C, 0x06])  # Adjacency.3 (long form, backwards) struct BinaryAddress
    buf += bytes([0x18, 0x10]) + bytes(range(16)) + bytes([0x00])  # addr = 00..0f
    buf += bytes([0x06, 0x14]) + bytes([0x80, 0x80, 0x80, 0x80, 0x80, 0x40])  # .10 long form, i64 zigzag(2**40)
    buf += bytes([0x00])  # end Adjacency
    buf += bytes([0x00])  # end
    db = decode_adjacency_database(bytes(buf))
    assert db.thisNodeName == name
    (a,) = db.adjacencies
    assert a.nextHopV6 == bytes(range(16)) and a.weight == 2 ** 40 and a.nextHopV4 == bytes(4)


def _random_db(rng, name, n_adj):
    adjs = []
    for k in range(n_adj):
        adjs.append(Adjacency(
            otherNodeName=f"node-{int(rng.integers(1e6))}", ifName=f"if_{k}_{'x' * int(rng.integers(0, 150))}",
            nextHopV6=rng.integers(0, 256, 16, dtype=np.uint8).tobytes(),
            nextHopV4=rng.integers(0, 256, 4, dtype=np.uint8).tobytes(),
            metric=int(rng.integers(-2 ** 31, 2 ** 31)), adjLabel=int(rng.integers(-5, 1 << 20)),
            isOverloaded=bool(rng.integers(2)), rtt=int(rng.integers(-100, 10 ** 6)),
            timestamp=int(rng.integers(-2 ** 62, 2 ** 62)), weight=int(rng.integers(-3, 2 ** 40)),
            otherIfName=f"rif_{k}" if rng.integers(2) else ""))
    return AdjacencyDatabase(thisNodeName=name, isOverloaded=bool(rng.integers(2)), adjacencies=adjs,
                             nodeLabel=int(rng.integers(-2 ** 31, 2 ** 31)),
                             area=["0", "spine", "a" * 40][int(rng.integers(3))])


@pytest.mark.parametrize("omit_defaults", [False, True])
@pytest.mark.parametrize("unknown", [False, True])
def test_round_trip_random_databases(omit_defaults, unknown):
    rng = np.random.default_rng(7 + 2 * omit_defaults + unknown)
    for n_adj in (0, 1, 14, 15, 16, 40, 300):  # list headers: short, 15 = long form
        db = _random_db(rng, f"r{n_adj}", n_adj)
        buf = encode_adjacency_database(db, omit_defaults=omit_defaults, unknown=unknown,
                                        perf_events=bool(n_adj % 2))
        assert decode_adjacency_database(buf) == db


def test_truncated_and_corrupted_input_fails_cleanly():
    rng = np.random.default_rng(3)
    buf = encode_adjacency_database(_random_db(rng, "t", 6), unknown=True)
    for cut in range(len(buf)):  # every proper prefix is malformed
        with pytest.raises(N.SpfError):
            decode_adjacency_database(buf[:cut])
    for _ in range(300):  # random byte flips: decode or refuse, never crash
        b = bytearray(buf)
        for _ in range(int(rng.integers(1, 4))):
            b[int(rng.integers(len(b)))] = int(rng.integers(256))
        try:
            decode_adjacency_database(bytes(b))
        except N.SpfError:
            pass
    with pytest.raises(N.SpfError):  # nesting beyond the skip depth limit
        decode_adjacency_database(bytes([0x1C] * 100 + [0] * 101))


def test_publication_semantics():
    """Decision.cpp:1726-1817: "adj:" values decode (area := publication's),
    TTL-only updates and non-adj keys are ignored, expired "adj:" keys name
    nodes, an undecodable value is skipped and counted."""
    rng = np.random.default_rng(11)
    d1, d2 = _random_db(rng, "n1", 3), _random_db(rng, "n2", 2)
    pub = encode_publication(
        [("adj:n1", encode_adjacency_database(d1)),
         ("prefix:n1", b"\x00"),
         ("adj:n3", None),  # TTL refresh: no value
         ("adj:n2:extra", encode_adjacency_database(d2)),  # node = 2nd ':'-token
         ("adj:bad", b"\x19\xff"),  # malformed
         ("fibTime:n1", b"123")],
        expired=["adj:gone", "prefix:gone", "adj:"], area="spine", node_ids=["x"],
        flood_root="r")
    p = decode_publication(pub)
    assert p.area == "spine" and p.skipped == 1
    # keyVals iteration order of the reference (see the order test below)
    got = {d.thisNodeName: d for d in p.adjacencyDbs}
    assert sorted(got) == ["n1", "n2"]
    for name, want in (("n1", d1), ("n2", d2)):
        want.area = "spine"
        assert got[name] == want
    assert p.expiredNodes == ["gone", ""]
    # area before the key-values (non-IDL order) and the IDL default area
    assert decode_publication(encode_publication([("adj:n1", encode_adjacency_database(d1))],
                                                 area="x", area_first=True)).adjacencyDbs[0].area == "x"
    assert decode_publication(encode_publication([], area=None)).area == "0"


def test_publication_name_mismatch_and_empty_area_are_refused():
    db = _random_db(np.random.default_rng(1), "other", 1)
    with pytest.raises(N.SpfError, match="carries the database"):
        decode_publication(encode_publication([("adj:n1", encode_adjacency_database(db))]))
    with pytest.raises(N.SpfError, match="empty area"):
        decode_publication(encode_publication([], area=""))


def _same_graph(a, b):
    ga, gb = a.flatten(), b.flatten()
    assert ga[0] == gb[0]  # node names in id order
    for x, y in zip(ga[1:], gb[1:]):  # row_ptr, col, metric, link_id, overloaded
        assert np.array_equal(x, y)


def test_link_state_from_publications_equals_direct_updates():
    """Host-only LinkState (device -1): the fabric's LSDB fed as KvStore
    publications builds the same links, overload bits and CSR as
    updateAdjacencyDatabases; expired keys delete like deleteAdjacencyDatabase."""
    topo = T.fabric(1000, full=False)
    from openr_amd.wire import unpack

    from oracle import keyvals_order

    dbs = unpack(topo.lsdb)
    direct = LinkState(device=-1)
    wire = LinkState(device=-1)
    chunks = [dbs[i:i + 97] for i in range(0, len(dbs), 97)]
    for ch in chunks:  # each publication in the reference's keyVals order
        direct.updateAdjacencyDatabases(
            [ch[i] for i in keyvals_order([f"adj:{d.thisNodeName}" for d in ch])])
    for ch in chunks:
        pub = encode_publication([(f"adj:{d.thisNodeName}", encode_adjacency_database(d)) for d in ch])
        c = wire.processPublication(pub)
        assert c.topologyChanged
        assert wire.lastPublicationCounts == (len(ch), 0)
    assert wire.numLinks() == direct.numLinks() and wire.numNodes() == direct.numNodes()
    _same_graph(wire, direct)
    # expire two nodes' databases
    gone = [dbs[0].thisNodeName, dbs[5].thisNodeName]
    c = wire.processPublication(encode_publication([], expired=[f"adj:{g}" for g in gone]))
    assert c.topologyChanged and wire.lastPublicationCounts == (0, 2)
    for g in gone:
        direct.deleteAdjacencyDatabase(g)
    assert wire.numLinks() == direct.numLinks()
    _same_graph(wire, direct)
    # a publication of another area is refused
    with pytest.raises(N.SpfError, match="area"):
        wire.processPublication(encode_publication([], area="other"))


def test_publication_databases_follow_reference_keyvals_order():
    """Databases come out in the iteration order of the reference's
    keyVals container (std::unordered_map<std::string, Value>,
    KvStore.thrift:43-44, Decision.cpp:1726), not in wire order; TTL-only and
    non-adj keys take part in the container but yield no database."""
    from oracle import keyvals_order

    rng = np.random.default_rng(11)
    for n in (1, 2, 5, 13, 14, 40, 97):
        names = [f"node{int(x)}" for x in rng.choice(10 ** 6, n, replace=False)]
        kv = []
        for i, nm in enumerate(names):
            db = AdjacencyDatabase(thisNodeName=nm, adjacencies=[], nodeLabel=i, area="0")
            kv.append((f"adj:{nm}", encode_adjacency_database(db)))
            if i % 3 == 0:
                kv.append((f"prefix:{nm}", b"x"))
            if i % 4 == 1:
                kv.append((f"adj:ttl{nm}", None))
        pub = decode_publication(encode_publication(kv))
        want = [kv[i][0][4:] for i in keyvals_order([k for k, _ in kv])
                if kv[i][0].startswith("adj:") and kv[i][1] is not None]
        assert [d.thisNodeName for d in pub.adjacencyDbs] == want
