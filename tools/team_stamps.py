"""Per-level phase breakdown of msbfs_team_kernel for one rank's share of an
all-sources pass (diagnostic).  SPF_STAMPS=<block> makes the kernel log
s_memtime at each phase boundary of that block (every wave's lane 0).

    python tools/team_stamps.py [--workload fabric_full] [--world 8] [--rank 1] [--block 0]

Per level the intervals are: sweep | wait for the member's waves | finalize
| team barrier | frontier copy (LDS) -- min..max over the 16 waves."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="fabric_full")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=1)
    ap.add_argument("--block", type=int, default=0)
    args = ap.parse_args()
    os.environ["SPF_STAMPS"] = str(args.block)
    import numpy as np
    import bench
    from openr_amd import hiprt
    from openr_amd.engine import SpfEngine, graph_from_lsdb, close_all
    from openr_amd.sharding import AllSourcesLayout

    topo, _ = bench.make_topology(args.workload)
    names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
    hiprt.set_device(0)
    dev = bench.Dev(0, 1)
    eng = SpfEngine(0)
    eng.load(rp, col, met, lid, ovl)
    n = len(names)
    nbrs = [eng.neighbors(s) for s in range(n)]
    k = np.array([len(x) for x in nbrs], np.int64)
    layout = AllSourcesLayout(k, eng.pitch, args.world, nbrs=nbrs)
    srcs = layout.srcs[args.rank]
    plan = eng.plan(srcs)
    print("kernels", plan.kernels(), "sources", len(srcs))
    d = dev.buf(max(1, len(srcs) * eng.pitch))
    nh = dev.buf(max(1, plan.nh_words))
    for _ in range(3):
        plan.execute(d.ptr, nh.ptr)
    dev.sync()
    raw = eng.debug_stamps().astype(np.int64).reshape(16, 64)
    waves = [raw[w, 1:1 + raw[w, 0]] for w in range(16) if raw[w, 0] > 0]
    m = min(len(x) for x in waves)
    st = np.stack([x[:m] for x in waves])
    t0 = st[:, 0].min()
    print(f"{len(waves)} waves, {m} stamps, total {int(st[:, -1].max() - t0)} cycles (100 MHz s_memtime? see guide)")
    for i in range(1, m):
        dd = st[:, i] - st[:, i - 1]
        print(f"interval {i:3d}: {int(dd.min()):8d}..{int(dd.max()):8d} (w{int(dd.argmax()):2d})")
    tl = eng.debug_timeline().astype(np.int64)
    live = tl[:, 1] > 0
    if live.any():
        t0 = tl[live, 0].min()
        st, en = (tl[live, 0] - t0) * 10, (tl[live, 1] - t0) * 10  # ns
        print(f"timeline: {int(live.sum())} blocks, start {st.min()}..{st.max()} ns, "
              f"end min {en.min()} p50 {int(np.median(en))} p90 {int(np.percentile(en, 90))} max {en.max()} ns")
        order = np.argsort(en)[::-1][:8]
        print("latest blocks:", [(int(np.flatnonzero(live)[i]), int(en[i])) for i in order])
    plan.close()
    close_all()


if __name__ == "__main__":
    main()
