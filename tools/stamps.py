"""Print the BFS kernel's per-phase cycle breakdown (workgroup 0) on fabric_full."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SPF_STAMPS"] = "1"
import numpy as np
import torch
from openr_amd import topology as T
from openr_amd.engine import SpfEngine, graph_from_lsdb
topo = T.fabric(10000, full=True) if (len(sys.argv) < 2 or sys.argv[1] == "fabric") else T.grid(100)
names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
eng = SpfEngine(0); eng.load(rp, col, met, lid, ovl)
plan = eng.plan(list(range(len(names))))
d = torch.empty(len(names) * eng.pitch, dtype=torch.int32, device="cuda")
h = torch.empty(max(1, plan.nh_words), dtype=torch.int32, device="cuda")
for _ in range(3):
    plan.execute_torch(d, h)
torch.cuda.synchronize()
st = eng.debug_stamps().astype(np.int64)
dt = np.diff(st)
print("stamps:", len(st), "total cycles", int(st[-1] - st[0]))
print("init", int(st[1] - st[0]))
lv = st[2:-2]
prev = st[1]
for L in range(len(lv) // 3):
    A, B, Cc = lv[3 * L: 3 * L + 3]
    print(f"level {L}: F-write(prev)+stores {A - prev:8d}  pull {B - A:8d}  barrier-wait {Cc - B:8d}")
    prev = Cc
print("last F-write/flag", int(st[-2] - prev), " tail (unreachable+padding)", int(st[-1] - st[-2]))
