"""Per-node getSpfResult latency on fabric_full: answered from the resident
all-sources pass (LinkState.prefetchAllSources, then getSpfResult(node) reads
node's row, bitmaps and pathLinks from the owning GPU) vs the plan path (no
resident pass: one single-source plan per node).  Both sides are compared on
every sampled node (metrics, next hops, pathLinks).  Prints one JSON line.

    python tools/facade_resident_latency.py [--nodes 400]
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

from openr_amd import topology as T  # noqa: E402
from openr_amd.link_state import LinkState  # noqa: E402


def view(r):
    """A result as plain data (metric, sorted next hops, sorted pathLinks) per node."""
    return {node: (e.metric(), sorted(e.nextHops()),
                   sorted(pl.link.directionalToString(pl.prevNode) for pl in e.pathLinks()))
            for node, e in r.items()}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=400)
    args = ap.parse_args()
    topo = T.fabric(10000, full=True)
    names = list(topo.nodes)
    rng = np.random.default_rng(7)
    sample = [names[int(i)] for i in rng.choice(len(names), args.nodes, replace=False)]

    res = LinkState(devices=[0])
    one = LinkState()
    for ls in (res, one):
        ls.updateAdjacencyDatabases(topo.lsdb)
    one.getSpfResult(sample[-1])  # build the plan path's engine state once
    t0 = time.perf_counter()
    res.prefetchAllSources()
    t_pass = time.perf_counter() - t0

    lat = {"resident": [], "plan": []}
    got = {}
    for name, ls in (("resident", res), ("plan", one)):
        for node in sample:
            t0 = time.perf_counter()
            r = ls.getSpfResult(node)
            len(r)  # the copied arrays are in place; entries stay lazy
            lat[name].append(time.perf_counter() - t0)
            if node in sample[:40]:
                got.setdefault(node, []).append(view(r))
    mism = [n for n, (a, b) in got.items() if a != b]
    us = {k: {"median_us": 1e6 * float(np.median(v)), "p90_us": 1e6 * float(np.percentile(v, 90)),
              "mean_us": 1e6 * float(np.mean(v))} for k, v in lat.items()}
    print(json.dumps({"workload": "fabric_full, getSpfResult(node) per node",
                      "nodes_timed": len(sample), "all_sources_pass_ms": 1e3 * t_pass,
                      "latency": us, "compared_nodes": len(got), "mismatches": mism}))


if __name__ == "__main__":
    main()
