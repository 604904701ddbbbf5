#!/usr/bin/env python3
"""Large-graph (N2) timing probe on the config-5 graph (BA 250k nodes):

* spf_sssp (cooperative frontier SSSP, distances only) for one source;
* a batched plan of 1 and of 64 sources (distance kernel + next hops),
  HIP-event kernel times from spf_plan_timing.

    python tools/n2_probe.py [--sources 64]
"""

from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from openr_amd import hiprt  # noqa: E402
from openr_amd import topology as T  # noqa: E402
from openr_amd.engine import SpfEngine, close_all  # noqa: E402
from openr_amd.link_state import LinkState  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sources", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    topo = T.barabasi_albert(250_000, 4, seed=1)
    ls = LinkState(device=-1)
    ls.updateAdjacencyDatabases(topo.lsdb)
    names, rp, col, met, lid, ovl = ls.flatten()
    eng = SpfEngine(0)
    eng.load(rp, col, met, lid, ovl)
    n = len(names)
    src0 = names.index("0")
    t = time.perf_counter()
    for _ in range(args.reps):
        eng.sssp(src0)
    print(f"spf_sssp(src '0'): {(time.perf_counter() - t) / args.reps * 1e3:.2f} ms host", flush=True)
    rng = np.random.default_rng(5)
    for srcs in ([src0], np.unique(rng.choice(n, args.sources, replace=False)).astype(np.uint32)):
        p = eng.plan(srcs)
        print(f"plan n_src={p.n_src} kernel={p.kernels()} nh_words={p.nh_words}", flush=True)
        D = hiprt.DeviceArray(p.n_src * eng.pitch, np.uint32)
        H = hiprt.DeviceArray(max(1, p.nh_words), np.uint32)
        p.execute(D.ptr, H.ptr)
        hiprt.synchronize()
        p.enable_timing(args.reps)
        t = time.perf_counter()
        for _ in range(args.reps):
            p.execute(D.ptr, H.ptr)
        hiprt.synchronize()
        host = (time.perf_counter() - t) / args.reps * 1e3
        a, b, k = p.timing()
        print(f"  execute {host:.1f} ms host; dist kernel {a / max(k, 1):.2f} ms, "
              f"next hops {b / max(k, 1):.2f} ms ({k} executes)", flush=True)
        D.free()
        H.free()
    close_all()


if __name__ == "__main__":
    main()
