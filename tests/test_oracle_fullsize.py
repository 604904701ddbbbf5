"""Pins the oracle machinery behind the full-size digests (CPU only):

* the integer-CSR restatement of runSpf (oracle/spf_oracle.cpp ``IntSpf``)
  equals the string-keyed restatement source for source, including drained
  nodes, drained links, parallel links and zero-metric plateaus (where the
  next-hop sets depend on the (metric, name) pop order);
* its what-if digests equal ``orc_ls_whatif_digests`` (runSpf / runSpfFast);
* the digest of the engine's planar output layout and of KSP2 pair/pool
  records, fed the oracle's own results, equals the oracle's direct digests,
  so a digest match on the GPU box means the outputs match;
* the committed fixtures load without pickle and describe the graphs the
  seeded generators build today.
"""

import ast
import sys
from pathlib import Path

import numpy as np
import pytest

from helpers import link_key
from oracle import (NameTable, OracleLinkState, digest_ksp2, digest_planar, keyvals_order,
                    ksp2_digests, link_keyhash, source_digests, whatif_digests,
                    whatif_digests_int)
from openr_amd import topology as T
from openr_amd.link_state import LinkState

GOLDEN = Path(__file__).resolve().parent / "golden"


def setup(topo):
    ls = LinkState(device=-1)
    ls.updateAdjacencyDatabases(topo.lsdb)
    names, rp, col, met, lid, ovl = ls.flatten()
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    return ls, names, orc, NameTable(names), (rp, col, met, lid, ovl)


def _zero_metrics(topo, frac, seed):
    rng = np.random.default_rng(seed)
    m = topo.lsdb.adjs["metric"]
    m[rng.random(len(m)) < frac] = 0
    return topo


GRAPHS = [
    ("grid8", lambda: T.grid(8)),
    ("fabric_ref1000", lambda: T.fabric(1000, full=False)),
    ("wan120", lambda: T.wan(120, 60, seed=2)),
] + [
    (f"rand{s}", (lambda s: lambda: T.random_graph(
        60, 150, 40 + s, max_metric=6, parallel_frac=0.25, overload_frac=0.1,
        link_overload_frac=0.05))(s))
    for s in range(4)
] + [
    (f"zero{s}", (lambda s: lambda: _zero_metrics(T.random_graph(
        50, 120, 60 + s, max_metric=3, parallel_frac=0.2, overload_frac=0.1), 0.3, s))(s))
    for s in range(3)
]


@pytest.mark.parametrize("name,make", GRAPHS, ids=[g[0] for g in GRAPHS])
@pytest.mark.parametrize("ulm", [True, False], ids=["metric", "hops"])
def test_int_restatement_equals_runspf(name, make, ulm):
    ls, names, orc, table, _ = setup(make())
    srcs = np.arange(len(names), dtype=np.uint32)
    a = source_digests(orc, table, srcs, ulm=ulm)
    b = source_digests(orc, table, srcs, ulm=ulm, int_path=True)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("name,make", GRAPHS[3:], ids=[g[0] for g in GRAPHS[3:]])
def test_int_whatif_equals_runspf(name, make):
    ls, names, orc, table, csr = setup(make())
    links = np.unique(csr[3])
    fails = [(ls._link(int(l))._n1, ls._link(int(l))._if1) for l in links]
    for s in (names[0], names[len(names) // 2]):
        base, want = whatif_digests(orc, table, s, fails, fast=False)
        base2, got = whatif_digests_int(orc, table, s, fails, threads=3)
        assert base == base2
        assert [tuple(int(x) for x in d) for d in got] == want


def _planar(names, csr, dist, mats):
    """Oracle dense results rendered in the engine's planar layout."""
    rp, col = csr[0], csr[1]
    n = len(names)
    pitch = (n + 63) // 64 * 64
    ks, offs, rows, off = [], [], [], 0
    for i in range(n):
        k = len(set(int(c) for c in col[rp[i]:rp[i + 1]]) - {i})  # (dead slots: self-loops)
        ks.append(k)
        offs.append(off)
        for j in range(k):
            row = np.zeros(pitch, bool)
            row[:n] = mats[i][j]
            rows.append(np.packbits(row, bitorder="little").view(np.uint32))
        off += k * pitch // 32
    d32 = np.where(dist == np.iinfo(np.uint64).max, 0xFFFFFFFF, dist).astype(np.uint32)
    nh = np.concatenate(rows) if rows else np.zeros(1, np.uint32)
    return d32, nh, np.array(offs, np.uint64), np.array(ks, np.uint32), pitch


@pytest.mark.parametrize("name,make", GRAPHS[:6], ids=[g[0] for g in GRAPHS[:6]])
def test_planar_digest_equals_oracle_digest(name, make):
    ls, names, orc, table, csr = setup(make())
    srcs = list(range(len(names)))
    dist, mats = orc.dense(names, srcs)
    d32, nh, offs, ks, pitch = _planar(names, csr, dist, mats)
    assert np.array_equal(digest_planar(d32, nh, offs, ks, pitch),
                          source_digests(orc, table, srcs))
    # a single flipped next-hop bit or distance changes the digest
    nh2 = nh.copy()
    nz = np.nonzero(nh2)[0]
    nh2[nz[len(nz) // 2]] ^= 1 << int(np.nonzero(
        np.unpackbits(nh2[nz[len(nz) // 2]:nz[len(nz) // 2] + 1].view(np.uint8),
                      bitorder="little"))[0][0])
    assert not np.array_equal(digest_planar(d32, nh2, offs, ks, pitch),
                              source_digests(orc, table, srcs))


@pytest.mark.parametrize("name,make", [GRAPHS[2], GRAPHS[3], GRAPHS[5]],
                         ids=[GRAPHS[2][0], GRAPHS[3][0], GRAPHS[5][0]])
def test_ksp2_digest_of_records_equals_oracle_digest(name, make):
    ls, names, orc, table, csr = setup(make())
    n = len(names)
    lid = csr[3]
    key_of = {tuple(link_key(ls._link(int(l)))): int(l) for l in np.unique(lid)}
    lh = np.zeros(int(lid.max()) + 1, np.uint64)
    for k, l in key_of.items():
        lh[l] = link_keyhash(k)
    srcs = list(range(0, n, 3))
    pairs = np.zeros((len(srcs) * n, 4), np.uint32)
    pool = []
    for i, s in enumerate(srcs):
        for d in range(n):
            for k in (1, 2):
                paths = orc.kth_paths(names[s], names[d], k)
                pairs[i * n + d, 2 + k - 1] = len(paths)
                pairs[i * n + d, k - 1] = len(pool) if paths else 0xFFFFFFFF
                for q, p in enumerate(paths):
                    last = q == len(paths) - 1
                    nxt = 0xFFFFFFFF if last else len(pool) + 2 + len(p)
                    pool += [len(p), nxt] + [key_of[tuple(x)] for x in p]
    got, gp = digest_ksp2(pairs, np.array(pool, np.uint32), len(srcs), n, lh, with_pairs=True)
    want, wp = ksp2_digests(orc, table, srcs, pairs=True)
    assert np.array_equal(gp, wp)
    assert np.array_equal(got, want)


def test_keyvals_order_is_a_permutation():
    keys = [f"adj:n{i}" for i in range(57)]
    order = keyvals_order(keys)
    assert sorted(order) == list(range(57)) and order != list(range(57))
    assert keyvals_order(["adj:a", "adj:a"]) == [0]  # duplicate key: first wins


def _load(name):
    z = np.load(GOLDEN / f"fullsize_{name}.npz")
    return ast.literal_eval(str(z["meta"])), z


@pytest.mark.parametrize("name", ["fabric_full", "fabric_ref", "grid100", "fabric_rtt",
                                  "wan2k_spf", "wan2k_ksp2", "ba250k_whatif", "ba250k_spf"])
def test_golden_fixtures_are_complete(name):
    meta, z = _load(name)
    assert meta["name"] == name
    if name in ("fabric_full", "fabric_ref", "grid100", "fabric_rtt", "wan2k_spf"):
        assert np.array_equal(z["srcs"], np.arange(meta["n_nodes"]))  # every source
        assert len(z["digest"]) == meta["n_nodes"]
    elif name == "wan2k_ksp2":
        assert len(z["srcs"]) >= 64 and z["pair_digest"].shape == (8, meta["n_nodes"])
    elif name == "ba250k_whatif":
        assert len(z["links"]) >= 10_000 and len(z["big_links"]) >= 159
        assert np.isin(z["big_links"], z["links"]).all()
        assert (z["n_nh_changed"] > 0).sum() > 1000  # hot failures are in the sample


@pytest.mark.parametrize("name", ["fabric_full", "grid100", "fabric_rtt", "wan2k_spf"])
def test_golden_fixtures_match_todays_generators(name):
    sys.path.insert(0, str(GOLDEN))
    from make_fullsize_digests import WORKLOADS, csr_digest

    meta, _ = _load(name)
    topo = WORKLOADS[name]()
    ls = LinkState(device=-1)
    ls.updateAdjacencyDatabases(topo.lsdb)
    _, rp, col, met, lid, ovl = ls.flatten()
    assert csr_digest(rp, col, met, lid, ovl) == meta["csr_digest"]
