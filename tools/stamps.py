"""Per-phase cycle breakdown of the BFS kernel (workgroup 0, every wave).

Diagnostic only: SPF_STAMPS=<workgroup> makes msbfs_kernel log s_memtime at
each phase boundary of that workgroup (default 0).  Prints, per level, the min/max over the 16 waves of the store phase,
pull phase and barrier wait, and which wave is the slowest.
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SPF_STAMPS", "0")  # the workgroup logged
import numpy as np
import torch
from openr_amd import topology as T
from openr_amd.engine import SpfEngine, graph_from_lsdb

which = sys.argv[1] if len(sys.argv) > 1 else "fabric"
topo = T.fabric(10000, full=True) if which == "fabric" else T.grid(100)
names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
eng = SpfEngine(0); eng.load(rp, col, met, lid, ovl)
plan = eng.plan(list(range(len(names))))
d = torch.empty(len(names) * eng.pitch, dtype=torch.int32, device="cuda")
h = torch.empty(max(1, plan.nh_words), dtype=torch.int32, device="cuda")
for _ in range(3):
    plan.execute_torch(d, h)
torch.cuda.synchronize()
raw = eng.debug_stamps().astype(np.int64)
waves = [raw[w, 1:1 + raw[w, 0]] for w in range(16) if raw[w, 0] > 0]
n = min(len(x) for x in waves)
st = np.stack([x[:n] for x in waves])  # [W, n]
t0 = st[:, 0].min()
print(f"{which}: {st.shape[0]} waves, {n} stamps, total cycles {int(st[:, -1].max() - t0)}")
# consecutive stamp intervals (min..max over the waves, slowest wave):
# single-buffered kernel: init | per level: stores, pull, barrier | tail;
# double-buffered: init | per level: pull+stores, barrier | tail
for k in range(1, n):
    d = st[:, k] - st[:, k - 1]
    print(f"interval {k:3d}: {int(d.min()):8d}..{int(d.max()):8d} (w{int(d.argmax()):2d})")
