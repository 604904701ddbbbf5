"""Diagnostics: one cooperative launch (spf_sssp on a graph
beyond the LDS kernels -> gsssp_coop_kernel) and exit, no torch.  Run under
`rocprofv3 --kernel-trace` to see whether the exit-time fault follows the
cooperative launch alone.  COOP_PROBE=plain runs a non-cooperative plan
instead (the control)."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from openr_amd import topology as T  # noqa: E402
from openr_amd.engine import SpfEngine, close_all, graph_from_lsdb  # noqa: E402

big = os.environ.get("COOP_PROBE", "coop") == "coop"
topo = T.wan(60000, 20000, seed=3) if big else T.wan(2000, 1000, seed=3)
names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
eng = SpfEngine(0)
eng.load(rp, col, met, lid, ovl)
d = eng.sssp(0)
print("probe", "coop" if big else "plain", len(names), int((d != 0xFFFFFFFF).sum()), flush=True)
close_all()
