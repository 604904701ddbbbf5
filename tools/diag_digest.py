"""Diagnostic: tests/test_gpu_sharded.py's bench-layout case for one
workload/world, per rank and per engine mode (env), against the golden
digests; prints the differing sources."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
from openr_amd.engine import SpfEngine
from openr_amd.sharding import AllSourcesLayout
from test_gpu_fullsize import _make, golden
from test_gpu_sharded import _run_rank

name = sys.argv[1] if len(sys.argv) > 1 else "fabric_full"
world = int(sys.argv[2]) if len(sys.argv) > 2 else 2
meta, g = golden(name)
ls, names, csr, cd = _make(name)
want = np.zeros(len(names), np.uint64)
want[g["srcs"].astype(np.int64)] = g["digest"]
for env in ({}, {"SPF_SLICED_GROUP": "0"}, {"SPF_SDIRECT": "0"}, {"SPF_MSBFS_TEAM": "0"},
            {"SPF_NARROW": "1"}, {"SPF_NARROW": "0"}):
    for key in ("SPF_SLICED_GROUP", "SPF_SDIRECT", "SPF_MSBFS_TEAM", "SPF_NARROW"):
        os.environ.pop(key, None)
    os.environ.update(env)
    eng = SpfEngine(0); eng.load(*csr)
    nbrs = [eng.neighbors(s) for s in range(len(names))]
    k = np.array([len(x) for x in nbrs], np.int64)
    lay = AllSourcesLayout(k, eng.pitch, world, nbrs=nbrs)
    for r in range(world):
        srcs = [int(x) for x in lay.srcs[r]]
        p = eng.plan(srcs)
        got = _run_rank(eng, srcs)
        bad = np.nonzero(got != want[srcs])[0]
        print(env, "rank", r, p.kernels(), p.row_mode(), "bad", len(bad),
              [(srcs[i], names[srcs[i]], len(nbrs[srcs[i]]), i) for i in bad[:4]], flush=True)
        p.close()
    eng.close()
