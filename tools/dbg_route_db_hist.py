"""Next hops per route of every node's materialised database on fabric_full
(spf_mplan_route_records headers): how many routes exceed the LDS staging
(kRsKeep = 16) and how many records they hold, by node degree class."""
import ctypes as C
import sys

import numpy as np

from openr_amd import _native as N
from openr_amd import topology as T
from openr_amd.link_state import LinkState

topo = T.fabric(10000, full=True)
with LinkState(devices=[0]) as ls:
    ls.updateAdjacencyDatabases(topo.lsdb)
    ls.prefetchAllSources()
    names, rp = ls.flatten()[:2]
    n = len(names)
    ptr = np.arange(n + 1, dtype=np.uint32)
    nodes = np.arange(n, dtype=np.uint32)
    total, ms = ls.allSourcesRouteRecords(ptr, nodes, True)
    print("records", total, "kernel ms", ms)
    mp = N.lib.ls_all_sources_plan(ls._h)
    deg = np.diff(rp.astype(np.int64))
    hdr = np.zeros(n, np.uint64)
    cnt_n = C.c_uint64()
    stats = {}
    for me in range(n):
        N.raise_for(N.lib.spf_mplan_route_db(C.c_void_p(mp), me, N.ptr(hdr, C.c_uint64), None, 0,
                                             C.byref(cnt_n)), "db")
        c = (hdr >> np.uint64(32)).astype(np.int64)
        key = int(deg[me])
        s = stats.setdefault(key, [0, 0, 0, 0, 0])
        s[0] += 1
        s[1] += int(c.sum())
        s[2] += int((c > 16).sum())
        s[3] += int(c[c > 16].sum())
        s[4] = max(s[4], int(c.max()))
    print("deg: nodes, records, routes>16, their records, max nh")
    for k in sorted(stats):
        print(k, stats[k])
