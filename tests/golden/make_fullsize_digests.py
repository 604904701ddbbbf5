#!/usr/bin/env python3
"""Generate the full-size parity digests (VERDICT r01 "next round" #1,
SURVEY.md §8(c)(iii)-(vi)) with the CPU oracle, in this container.

    python tests/golden/make_fullsize_digests.py [--only NAME ...] [--threads T]

Each fixture is ``tests/golden/fullsize_<name>.npz`` holding the oracle's
64-bit digests (oracle/spf_oracle.cpp, "Full-size parity digests"):

* ``fabric_full`` / ``fabric_ref`` / ``grid100`` -- BASELINE configs 2-3: one
  digest of runSpf(src) (distances + next-hop sets, LinkState.cpp:808-882)
  for EVERY source; the string-keyed restatement (``runSpf``).
* ``fabric_rtt`` -- the fabric with RTT-style per-direction metrics
  (LinkMonitor.cpp:44-47, max(rtt/100, 1)), every source, weighted SPF; the
  integer-CSR restatement (pinned to runSpf by tests/test_oracle_fullsize.py).
* ``wan2k_spf`` -- the config-4 WAN graph, every source, weighted SPF.
* ``wan2k_ksp2`` -- config 4: getKthPaths(s, d, 1) and (s, d, 2)
  (LinkState.cpp:762-791) for 256 sources x every destination, per-source
  digests plus per-pair digests of 8 of them.
* ``wan2k_ksp2_all`` -- the same for EVERY source (4M pairs, per-source
  digests): bench.py's wan_ksp2 line checks its whole output against it.
* ``ba250k_whatif`` -- config 5: runSpf("0", true, {l}) digests for ~16k
  single-link failures: uniform random links, random tight links and the
  3000 shortest-path-tree links with the largest subtrees (every failure
  whose affected region can exceed a GPU wave team; the affected nodes of a
  tree link's failure lie in its subtree).
* ``ba20k_whatif_all`` -- config 5's repair machinery at a scale the oracle
  covers whole: runSpf("0", true, {l}) digests for EVERY link of a 20k-node
  Barabasi-Albert graph (m = 4, ~80k links; wave-team, group-team and
  overflow repairs all occur).
* ``ba250k_spf`` -- the large-graph regime (N2): 64 sampled sources of the
  config-5 graph, weighted SPF + next hops, integer restatement.

Inputs are regenerated from the seeded generators in openr_amd/topology.py
(the same calls bench.py makes); the fixture stores the parameters, node
count and a digest of the flattened CSR so a generator change is caught.
"""

from __future__ import annotations

import argparse
import hashlib
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from oracle import (NameTable, OracleLinkState, ksp2_digests, source_digests,  # noqa: E402
                    whatif_digests_int)
from openr_amd import topology as T  # noqa: E402
from openr_amd.link_state import LinkState  # noqa: E402


fabric_rtt = T.fabric_rtt  # openr_amd/topology.py (same seeded generator)


WORKLOADS = {
    "fabric_full": lambda: T.fabric(10000, full=True),
    "fabric_ref": lambda: T.fabric(10000, full=False),
    "grid100": lambda: T.grid(100),
    "fabric_rtt": fabric_rtt,
    "wan2k_spf": lambda: T.wan(2000, 1000, seed=1),
    "wan2k_ksp2": lambda: T.wan(2000, 1000, seed=1),
    "wan2k_ksp2_all": lambda: T.wan(2000, 1000, seed=1),
    "ba250k_whatif": lambda: T.barabasi_albert(250_000, 4, seed=1),
    "ba250k_spf": lambda: T.barabasi_albert(250_000, 4, seed=1),
    "ba20k_whatif_all": lambda: T.barabasi_albert(20_000, 4, seed=7),
}


def csr_digest(rp, col, met, lid, ovl) -> str:
    h = hashlib.sha256()
    for a in (rp, col, met, lid, ovl):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:16]


def setup(topo):
    ls = LinkState(device=-1)
    ls.updateAdjacencyDatabases(topo.lsdb)
    names, rp, col, met, lid, ovl = ls.flatten()
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    return ls, names, orc, NameTable(names), (rp, col, met, lid, ovl)


def ba_failures(ls, names, csr, rng):
    """Failure links (product link ids) for the what-if fixture."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import dijkstra

    rp, col, met, lid, ovl = csr
    n = len(names)
    src = names.index("0")
    A = sp.csr_matrix((met.astype(np.float64), col, rp), shape=(n, n))
    dist, pred = dijkstra(A, indices=src, return_predecessors=True)
    tail = np.repeat(np.arange(n), np.diff(rp))
    tight = dist[tail] + met == dist[col]
    # subtree sizes of scipy's shortest-path tree, deepest first
    order = np.argsort(-dist)
    size = np.ones(n, np.int64)
    for v in order:
        p = pred[v]
        if p >= 0:
            size[p] += size[v]
    # the tree link into v: an edge pred[v] -> v (lowest link id among parallels)
    tree_e = {}
    for e in np.nonzero(tight)[0]:
        a, b = int(tail[e]), int(col[e])
        if pred[b] == a and (b not in tree_e or lid[e] < lid[tree_e[b]]):
            tree_e[b] = e
    heads = sorted(tree_e, key=lambda v: -size[v])[:3000]
    big = {int(lid[tree_e[v]]) for v in heads}
    all_links = np.unique(lid)
    tight_links = np.unique(lid[tight])
    pick = set(int(x) for x in rng.choice(all_links, 12000, replace=False))
    pick |= set(int(x) for x in rng.choice(tight_links, 1500, replace=False))
    pick |= big
    return np.array(sorted(pick), np.uint32), np.array(sorted(big), np.uint32)


def make(name: str, threads: int) -> None:
    t0 = time.time()
    topo = WORKLOADS[name]()
    ls, names, orc, table, csr = setup(topo)
    n = len(names)
    meta = dict(name=name, topology=topo.name, n_nodes=n, n_edges=len(csr[1]),
                csr_digest=csr_digest(*csr))
    rng = np.random.default_rng(2024)
    out = {}
    if name in ("fabric_full", "fabric_ref", "grid100"):
        srcs = np.arange(n, dtype=np.uint32)
        out["srcs"] = srcs
        out["digest"] = source_digests(orc, table, srcs, threads=threads)
        meta["oracle"] = "runSpf (string-keyed restatement)"
    elif name in ("fabric_rtt", "wan2k_spf"):
        srcs = np.arange(n, dtype=np.uint32)
        out["srcs"] = srcs
        out["digest"] = source_digests(orc, table, srcs, int_path=True, threads=threads)
        # the string restatement on a sample, as a cross-check at generation time
        samp = np.sort(rng.choice(n, 24, replace=False)).astype(np.uint32)
        ref = source_digests(orc, table, samp, threads=threads)
        assert np.array_equal(ref, out["digest"][samp]), "int restatement != runSpf"
        meta["oracle"] = "integer-CSR restatement (cross-checked against runSpf on 24 sources)"
    elif name == "ba250k_spf":
        srcs = np.sort(rng.choice(n, 64, replace=False)).astype(np.uint32)
        srcs[0] = names.index("0")
        srcs = np.unique(srcs)
        out["srcs"] = srcs
        out["digest"] = source_digests(orc, table, srcs, int_path=True, threads=threads)
        meta["oracle"] = "integer-CSR restatement"
    elif name == "wan2k_ksp2":
        srcs = np.sort(rng.choice(n, 256, replace=False)).astype(np.uint32)
        out["srcs"] = srcs
        d, pairs = ksp2_digests(orc, table, srcs[:8], pairs=True, threads=threads)
        rest = ksp2_digests(orc, table, srcs[8:], threads=threads)
        out["digest"] = np.concatenate([d, rest])
        out["pair_digest"] = pairs  # [8, n]
        meta["oracle"] = "getKthPaths k=1,2 (trace + runSpf with ignore set)"
    elif name == "wan2k_ksp2_all":
        # every source (config 4's whole workload, 4M pairs): what bench.py's
        # wan_ksp2 line checks in-bench
        srcs = np.arange(n, dtype=np.uint32)
        out["srcs"] = srcs
        out["digest"] = ksp2_digests(orc, table, srcs, threads=threads)
        meta["oracle"] = "getKthPaths k=1,2 (trace + runSpf with ignore set), every source"
    elif name == "ba20k_whatif_all":
        links = np.unique(csr[3]).astype(np.uint32)
        fails = [(ls._link(int(l))._n1, ls._link(int(l))._if1) for l in links]
        base, dig = whatif_digests_int(orc, table, "0", fails, threads=threads)
        out["links"] = links
        out["n_dist_changed"] = dig["n_dist_changed"]
        out["n_nh_changed"] = dig["n_nh_changed"]
        out["hash"] = dig["hash"]
        out["base"] = np.array(base, np.uint64)
        meta["oracle"] = "integer-CSR restatement of runSpf(src, true, {link}), every link"
        meta["src"] = "0"
    elif name == "ba250k_whatif":
        links, big = ba_failures(ls, names, csr, rng)
        fails = [(ls._link(int(l))._n1, ls._link(int(l))._if1) for l in links]
        base, dig = whatif_digests_int(orc, table, "0", fails, threads=threads)
        out["links"] = links
        out["big_links"] = big
        out["n_dist_changed"] = dig["n_dist_changed"]
        out["n_nh_changed"] = dig["n_nh_changed"]
        out["hash"] = dig["hash"]
        out["base"] = np.array(base, np.uint64)
        meta["oracle"] = "integer-CSR restatement of runSpf(src, true, {link})"
        meta["src"] = "0"
    meta["seconds"] = round(time.time() - t0, 1)
    meta["threads"] = threads
    np.savez_compressed(HERE / f"fullsize_{name}.npz", meta=np.array(repr(meta)), **out)
    print(f"{name}: {meta}", flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    for name in args.only or list(WORKLOADS):
        make(name, args.threads)


if __name__ == "__main__":
    main()
