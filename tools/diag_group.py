"""Diagnostic: a rank share of fabric_full (locality layout) solved in several
modes (SPF_SLICED_GROUP, SPF_SDIRECT, SPF_MSBFS_TEAM); each mode's rows of
a few sources compared with a small non-team plan of those sources."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from openr_amd import topology as T
from openr_amd.engine import SpfEngine, graph_from_lsdb
from openr_amd.sharding import AllSourcesLayout

world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
rank = int(sys.argv[2]) if len(sys.argv) > 2 else 1
names, rp, col, met, lid, ovl = graph_from_lsdb(T.fabric(10000, full=True).lsdb)
eng = SpfEngine(0); eng.load(rp, col, met, lid, ovl)
nbrs = [eng.neighbors(s) for s in range(len(names))]
k = np.array([len(x) for x in nbrs], np.int64)
lay = AllSourcesLayout(k, eng.pitch, world, nbrs=nbrs)
srcs = [int(x) for x in lay.srcs[rank]]
probe = [332, 350, 367, 410, 411, 1000, 5000, 9000]
probe = [s for s in probe if s in set(srcs)]
os.environ["SPF_MSBFS_TEAM"] = "0"
ref = eng.solve(probe)
del os.environ["SPF_MSBFS_TEAM"]
for env in ({}, {"SPF_SLICED_GROUP": "0"}, {"SPF_SDIRECT": "0"}, {"SPF_SDIRECT": "0", "SPF_SLICED_GROUP": "0"},
            {"SPF_MSBFS_TEAM": "0"}):
    for key in ("SPF_SLICED_GROUP", "SPF_SDIRECT", "SPF_MSBFS_TEAM"):
        os.environ.pop(key, None)
    os.environ.update(env)
    p = eng.plan(srcs)
    res = eng.solve(srcs)
    msg = []
    for q, s in enumerate(probe):
        i = srcs.index(s)
        dd = np.array_equal(res.dist[i], ref.dist[q])
        x, y = res.nh_matrix(i), ref.nh_matrix(q)
        nd = int((x != y).sum())
        if not dd or nd:
            j, v = np.nonzero(x != y)
            msg.append(f"{s}: dist {'ok' if dd else 'BAD'} nh diffs {nd} nbr {sorted(set(j.tolist()))[:5]} dst {v[:4].tolist()}")
    print(env, p.kernels(), p.row_mode(), "OK" if not msg else msg)
