#!/usr/bin/env python3
"""Emulated multi-GPU all-sources pass on ONE GPU: for world = 1, 2, 4, 8
build every rank's plan over its block of sources (sharding.AllSourcesLayout,
exactly what rank r runs in bench.py's sharded-resident mode), time each
rank's execute alone with HIP events, and verify the per-source digests of
all ranks together against the oracle's committed digests.

rank_ms is the whole execute timed like a bench step (back-to-back executes,
one sync); rank_kernel_ms the execute's kernels by HIP events.
The projected strong-scaling efficiency at world N is t(1) / (N * max_r t_r):
every rank of a real N-GPU run executes the same plan on its own GPU with no
data-path collective, so the slowest rank sets the step time (xGMI is not on
the path).  Output: one JSON line per world size.

    python tools/emulate_ranks.py [--workload fabric_full] [--worlds 1,2,4,8]
"""
from __future__ import annotations

import argparse
import ast
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="fabric_full")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()

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
    gold = ROOT / "tests" / "golden" / f"fullsize_{args.workload}.npz"
    want = None
    if gold.exists():
        z = np.load(gold)
        meta = ast.literal_eval(str(z["meta"]))
        if meta["n_nodes"] == n:
            want = dict(zip(z["srcs"].tolist(), z["digest"].tolist()))
    t1 = None
    for world in [int(x) for x in args.worlds.split(",")]:
        layout = AllSourcesLayout(k, eng.pitch, world, nbrs=nbrs)
        per_rank, phases, digests, wall, wall_nt = [], [], {}, [], []
        for r in range(world):
            srcs = layout.srcs[r]
            plan = eng.plan(srcs)
            d = dev.buf(max(1, len(srcs) * eng.pitch))
            nh = dev.buf(max(1, plan.nh_words))
            dg = dev.buf(max(1, len(srcs)), np.int64)
            for _ in range(2):
                plan.execute(d.ptr, nh.ptr)
            plan.enable_timing(args.steps)
            for _ in range(args.steps):
                plan.execute(d.ptr, nh.ptr)
            ms, cnt = plan.timing_phases()
            # the whole execute as the bench's step sees it (memsets, every
            # launch, the row gather of non-direct plans): back-to-back
            # executes, one sync
            dev.sync()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                plan.execute(d.ptr, nh.ptr)
            dev.sync()
            wall.append((time.perf_counter() - t0) * 1e3 / args.steps)
            # the same without timing events (a fresh plan: no event records)
            plan_nt = eng.plan(srcs)
            for _ in range(2):
                plan_nt.execute(d.ptr, nh.ptr)
            dev.sync()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                plan_nt.execute(d.ptr, nh.ptr)
            dev.sync()
            wall_nt.append((time.perf_counter() - t0) * 1e3 / args.steps)
            plan_nt.close()
            plan.digest(d.ptr, nh.ptr, dg.ptr)
            dev.sync()
            got = dg.numpy()[: len(srcs)].view(np.uint64)
            digests.update(zip(srcs.tolist(), got.tolist()))
            per_rank.append(sum(ms) / max(cnt, 1))
            phases.append([round(x / max(cnt, 1), 4) for x in ms])
            plan.close()
            for b in (d, nh, dg):
                b.free()
            dev.bufs = []
        t = max(wall)
        if world == 1:
            t1 = t
        bad = None
        if want is not None:
            bad = sum(1 for s, v in digests.items() if want.get(s) != v)
        print(json.dumps({
            "workload": args.workload, "world": world, "sources": n,
            "rank_ms": [round(x, 4) for x in wall], "rank_ms_no_events": [round(x, 4) for x in wall_nt], "rank_kernel_ms": [round(x, 4) for x in per_rank],
            "rank_phase_ms": phases, "partition": layout.partition, "closure": layout.closure,
            "rank_sources": [len(s) for s in layout.srcs],
            "step_ms": round(t, 4),
            "projected_efficiency": None if t1 is None else round(t1 / (world * t), 3),
            "digest_mismatches_vs_oracle": bad}), flush=True)
    eng.check()
    close_all()


if __name__ == "__main__":
    main()
