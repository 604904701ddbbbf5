"""Sweeps per workgroup of mssp_kernel on a weighted all-sources pass
(diagnostic; SPF_STAMPS makes the kernel count them)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SPF_STAMPS"] = "0"
import numpy as np
import bench
from openr_amd import hiprt
from openr_amd.engine import SpfEngine, graph_from_lsdb, close_all

w = sys.argv[1] if len(sys.argv) > 1 else "fabric_rtt"
topo, _ = bench.make_topology(w)
names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
hiprt.set_device(0)
dev = bench.Dev(0, 1)
eng = SpfEngine(0)
eng.load(rp, col, met, lid, ovl)
n = len(names)
plan = eng.plan(list(range(n)))
print("kernels", plan.kernels())
d = dev.buf(n * eng.pitch)
nh = dev.buf(max(1, plan.nh_words))
plan.execute(d.ptr, nh.ptr)
dev.sync()
st = eng.debug_stamps().astype(np.int64).ravel()
print("sweeps total", st[0], "max", st[1], "workgroups", st[2], "mean", st[0] / max(st[2], 1))
n_sl = (n + 63) // 64
print("slices swept", st[3], "of", st[0] * n_sl, "slice visits:", round(st[3] / max(1, st[0] * n_sl), 3))
print("slices swept per sweep", st[4:16].tolist())
print("nodes decreased per sweep", st[16:28].tolist())
print("metric range", met.min(), met.max(), "mean", met.mean())
plan.close()
close_all()
