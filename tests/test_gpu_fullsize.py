"""Full-size parity on the MI355X against the oracle's committed digests
(tests/golden/fullsize_*.npz, made by tests/golden/make_fullsize_digests.py
with oracle/spf_oracle.cpp in the build container).

Every output the engine produces for these workloads is reduced with the same
hash the oracle used (oracle.digest_planar / digest_ksp2 over the engine's
output layout) and compared source by source, failure by failure:

* all-sources SPF + ECMP, every source: fabric_full / fabric_ref / grid100
  (BASELINE configs 2-3), fabric_rtt (RTT-style weighted metrics),
  wan2k_spf (weighted WAN);
* KSP2 (config 4): 256 sources x all 2000 destinations, per-pair digests
  for 8 of them;
* what-if (config 5): ~16.5k single-link failures of the 250k-node graph,
  including the 3000 shortest-path-tree links with the largest subtrees,
  and every one of the ~80k failures of a 20k-node graph of the same family;
* large-graph SPF + next hops (N2): 64 sources of the 250k-node graph.
"""

import ast
from pathlib import Path

import numpy as np
import pytest

from helpers import link_key
from oracle import digest_ksp2, digest_planar, link_keyhash
from openr_amd import topology as T
from openr_amd.engine import SpfEngine
from openr_amd.link_state import LinkState

pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).resolve().parent / "golden"
sys_path_golden = str(GOLDEN)


def golden(name):
    z = np.load(GOLDEN / f"fullsize_{name}.npz")  # allow_pickle=False (default)
    meta = ast.literal_eval(str(z["meta"]))
    return meta, {k: z[k] for k in z.files if k != "meta"}


def _make(name):
    import sys

    sys.path.insert(0, sys_path_golden)
    from make_fullsize_digests import WORKLOADS, csr_digest

    topo = WORKLOADS[name]()
    ls = LinkState(device=-1)
    ls.updateAdjacencyDatabases(topo.lsdb)
    names, rp, col, met, lid, ovl = ls.flatten()
    return ls, names, (rp, col, met, lid, ovl), csr_digest(rp, col, met, lid, ovl)


def _engine(csr):
    eng = SpfEngine(0)
    eng.load(*csr)
    return eng


def _report(got, want, what, labels):
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (f"{what}: {len(bad)} of {len(want)} differ from the oracle, "
                           f"first: {[labels[i] for i in bad[:5]]}")


@pytest.mark.parametrize("name", ["fabric_full", "fabric_ref", "grid100", "fabric_rtt",
                                  "wan2k_spf"])
def test_all_sources_every_source_matches_oracle(name):
    meta, g = golden(name)
    ls, names, csr, cd = _make(name)
    assert cd == meta["csr_digest"] and len(names) == meta["n_nodes"]
    with _engine(csr) as eng:
        srcs = g["srcs"]
        plan = eng.plan(srcs)
        res = plan.execute_host()
        got = digest_planar(res.dist, res.nh, res.nh_off, res.words, res.pitch)
    _report(got, g["digest"], f"{name} per-source digests", [names[int(s)] for s in srcs])


def test_ksp2_wan2k_256_sources_all_destinations_match_oracle():
    meta, g = golden("wan2k_ksp2")
    ls, names, csr, cd = _make("wan2k_ksp2")
    assert cd == meta["csr_digest"]
    lid = csr[3]
    lh = np.zeros(int(lid.max()) + 1, np.uint64)
    for l in np.unique(lid):
        lh[int(l)] = link_keyhash(link_key(ls._link(int(l))))
    srcs = g["srcs"]
    with _engine(csr) as eng:
        res = eng.ksp2(srcs)
    got, pairs = digest_ksp2(res.pairs, res.pool, len(srcs), len(names), lh, with_pairs=True)
    want_pairs = g["pair_digest"]
    for i in range(want_pairs.shape[0]):
        _report(pairs[i], want_pairs[i], f"KSP2 pairs of source {names[int(srcs[i])]}", names)
    _report(got, g["digest"], "KSP2 per-source digests", [names[int(s)] for s in srcs])


def test_whatif_ba250k_16k_failures_match_oracle():
    meta, g = golden("ba250k_whatif")
    ls, names, csr, cd = _make("ba250k_whatif")
    assert cd == meta["csr_digest"]
    links = g["links"]
    with _engine(csr) as eng:
        got_links, got, base = eng.whatif(names.index(meta["src"]), links)
    assert np.array_equal(got_links, links)
    assert (int(base["n_dist_changed"]), int(base["n_nh_changed"]), int(base["hash"])) == \
        tuple(int(x) for x in g["base"])
    for f in ("n_dist_changed", "n_nh_changed", "hash"):
        _report(got[f], g[f], f"what-if {f}", [int(l) for l in links])
    # the sample reaches the large repairs (workgroup teams)
    assert int(g["n_nh_changed"].max()) > 50_000


@pytest.mark.parametrize("wavecap", [None, "128"], ids=["default", "wavecap128"])
def test_whatif_ba20k_every_failure_matches_oracle(wavecap, monkeypatch):
    """Config 5's repair machinery where the oracle covers every failure: all
    ~80k single-link failures of a 20k-node Barabasi-Albert graph from "0"
    (cold, wave-team, group-team and overflow repairs), on the default path
    and with the wave teams' |D| cap lowered so more repairs overflow to the
    workgroup teams."""
    if wavecap:
        monkeypatch.setenv("SPF_WHATIF_WAVECAP", wavecap)
    meta, g = golden("ba20k_whatif_all")
    ls, names, csr, cd = _make("ba20k_whatif_all")
    assert cd == meta["csr_digest"]
    links = g["links"]
    with _engine(csr) as eng:
        got_links, got, base = eng.whatif(names.index(meta["src"]))
    assert np.array_equal(np.sort(got_links), links)
    order = np.argsort(got_links)
    assert (int(base["n_dist_changed"]), int(base["n_nh_changed"]), int(base["hash"])) == \
        tuple(int(x) for x in g["base"])
    for f in ("n_dist_changed", "n_nh_changed", "hash"):
        _report(got[f][order], g[f], f"what-if {f}", [int(l) for l in links])
    # the graph reaches repairs past a wave team's cap (workgroup teams)
    assert int(g["n_nh_changed"].max()) > 1024


@pytest.mark.parametrize("big", ["1", "0"], ids=["big_kernel", "exact_kernel"])
def test_large_graph_spf_ecmp_ba250k_matches_oracle(big, monkeypatch):
    """N2: batched SPF + ECMP next hops beyond the LDS-resident kernels, on
    spf_big_kernel (the default) and on the exact kernel (SPF_BIG=0; 16 of
    the sources, it is the slow envelope)."""
    monkeypatch.setenv("SPF_BIG", big)
    meta, g = golden("ba250k_spf")
    ls, names, csr, cd = _make("ba250k_spf")
    assert cd == meta["csr_digest"]
    n = len(g["srcs"]) if big == "1" else 16
    srcs = g["srcs"][:n]
    with _engine(csr) as eng:
        p = eng.plan(srcs)
        assert p.kernels()[0] == ("spf_big_kernel" if big == "1" else "exact_spf_kernel")
        p.close()
        res = eng.solve(srcs)
        got = digest_planar(res.dist, res.nh, res.nh_off, res.words, res.pitch)
    _report(got, g["digest"][:n], "ba250k per-source digests", [names[int(s)] for s in srcs])


def test_ksp2_wan2k_every_source_engine_digest_matches_oracle():
    """Config 4's whole output -- getKthPaths(s, d, 1|2) for all 4M pairs --
    reduced on the GPU (spf_ksp2_digest, the reduction bench.py's wan_ksp2
    line checks) against the oracle's digests of every source
    (fullsize_wan2k_ksp2_all.npz), and the GPU reduction equals the oracle's
    reduction (digest_ksp2) of the same output on the 256-source fixture."""
    import sys

    from openr_amd.hiprt import DeviceArray

    sys.path.insert(0, str(GOLDEN.parent.parent))
    from bench import link_value_hash

    meta, g = golden("wan2k_ksp2_all")
    ls, names, csr, cd = _make("wan2k_ksp2_all")
    assert cd == meta["csr_digest"]
    lid = csr[3]
    lh = np.zeros(int(lid.max()) + 1, np.uint64)
    for l in np.unique(lid):
        (a, b), (c, d) = ls._link(int(l)).orderedNames
        lh[int(l)] = link_value_hash(a, b, c, d)
        assert int(lh[int(l)]) == link_keyhash(link_key(ls._link(int(l))))
    srcs = g["srcs"]
    n = len(names)
    with _engine(csr) as eng:
        p = eng.ksp2_plan(srcs)
        pairs = DeviceArray(len(srcs) * n * 4, np.uint32)
        cnt = DeviceArray(4, np.uint64, zero=True)
        words = 1 << 20
        pool = DeviceArray(words, np.uint32)
        p.execute(pairs.ptr, pool.ptr, words, cnt.ptr)
        eng.check()
        used = int(cnt.numpy()[0])
        if used > words:  # size the pool and run again
            pool.free()
            words = used + used // 4 + (1 << 20)  # grab slack varies run to run
            pool = DeviceArray(words, np.uint32)
            p.execute(pairs.ptr, pool.ptr, words, cnt.ptr)
            eng.check()
            used = int(cnt.numpy()[0])
        assert not (int(cnt.numpy()[2]) & 1)
        d_lh = DeviceArray(len(lh), np.uint64)
        d_lh.upload(lh)
        dg = DeviceArray(len(srcs), np.uint64, zero=True)
        p.digest(pairs.ptr, pool.ptr, d_lh.ptr, dg.ptr)
        eng.check()
        got = dg.numpy()
        # the GPU reduction equals the oracle's reduction of the same output
        sub = np.arange(0, len(srcs), 97)
        host = digest_ksp2(pairs.numpy().view(np.uint32).reshape(-1, 4)[
            (sub[:, None] * n + np.arange(n)[None, :]).ravel()], pool.numpy()[:used], len(sub), n, lh)
        assert np.array_equal(host, got[sub])
        p.close()
        for b in (pairs, cnt, pool, d_lh, dg):
            b.free()
    _report(got, g["digest"], "KSP2 per-source digests (every source)", [names[int(s)] for s in srcs])
