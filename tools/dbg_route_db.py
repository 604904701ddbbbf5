"""Diagnose spf_mplan_route_records against spf_mplan_routes (one me at a
time) on a graph: prints the first routes whose records differ."""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, "tests")
from openr_amd import _native as N  # noqa: E402
from openr_amd import topology as T  # noqa: E402
from openr_amd.link_state import LinkState  # noqa: E402

lfa = "--sp" not in sys.argv
topo = T.fabric(1000, full=True)
with LinkState(devices=[0]) as ls:
    ls.updateAdjacencyDatabases(topo.lsdb)
    ls.prefetchAllSources()
    names, rp = ls.flatten()[:2]
    n = len(names)
    rng = np.random.default_rng(n)
    sets = [[v] for v in range(n)]
    for _ in range(40):
        sets.append(sorted(int(x) for x in rng.choice(n, int(rng.integers(2, 5)), replace=False)))
    ptr = np.zeros(len(sets) + 1, np.uint32)
    ptr[1:] = np.cumsum([len(s) for s in sets])
    nodes = np.concatenate([np.asarray(s, np.uint32) for s in sets])
    total, ms = ls.allSourcesRouteRecords(ptr, nodes, lfa)
    print("records", total, "ms", ms)
    mp = N.lib.ls_all_sources_plan(ls._h)
    bad = 0
    for me in range(n):
        hdr, rec = ls.allSourcesRouteDb(me)
        deg = int(rp[me + 1] - rp[me])
        S = len(sets)
        mn = np.zeros(S, np.uint64)
        cnt = np.zeros(S, np.uint32)
        edge = np.zeros(max(1, S * deg), np.uint32)
        met = np.zeros(max(1, S * deg), np.uint64)
        st = N.lib.spf_mplan_routes(C.c_void_p(mp), me, N.ptr(ptr), N.ptr(nodes), S, 1 if lfa else 0,
                                    N.ptr(mn, C.c_uint64), N.ptr(cnt), N.ptr(edge), N.ptr(met, C.c_uint64))
        assert st == 0, st
        for p in range(S):
            o, c = int(hdr[p] & 0xFFFFFFFF), int(hdr[p] >> 32)
            want = [(int(edge[p * deg + k]), int(met[p * deg + k])) for k in range(int(cnt[p]))]
            got = [(int(r & 0xFFFFFFFF), int(r >> 32)) for r in rec[o:o + c]]
            if got != want:
                bad += 1
                if bad <= 8:
                    print(f"me {me} deg {deg} set {p} off {o} cnt {c}: got {got} want {want}")
    print("bad routes", bad)
