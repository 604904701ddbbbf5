#!/usr/bin/env python3
"""Headline benchmark: all-sources SPF + ECMP next-hop sets on the 10k-node DC
fabric (BASELINE.json configs[2]; metric "all-sources SPF solves/sec + GTEPS,
10k-node fabric, 1/2/4/8 MI355X").

Default workload (fabric_full): a step = one all-sources pass, every node of
the fabric solved as a source (distances + ECMP next-hop bitsets, bit-exact
with the reference's LinkState::runSpf, openr/decision/LinkState.cpp:808-882).
With --gpus N under torchrun (one process per GPU, the driver's launch) the
sources are split over the N ranks (sharding.AllSourcesLayout: the locality
partition on fabrics, contiguous id blocks on grids; the rule of the engine's
spf_partition_sources), every rank's distance rows and next-hop bitmaps stay
RESIDENT in its own HBM (no collective inside the step), and after the timed
steps rank 0 gathers per-source digests (RCCL) and checks every source
against the oracle (strong scaling: the work per step is fixed).
--results gather (labelled extra) gathers the rows and bitmaps to rank 0
inside the step instead; --scaling weak gives rank r its own LSDB snapshot
(rack switch r drained, BM_DecisionFabric's per-iteration perturbation,
RoutingBenchmarkUtils.cpp:406-447).  Without torchrun, --gpus N (or
--devices 0,1,..., repeats allowed) runs the same split from ONE process
through the multi-device context spf_mctx (Open/R's Decision is one process,
Decision.cpp:1484).

Other BASELINE configs (--workload):
  grid100    configs[1]: all-sources SPF + ECMP on grid 100x100 (as above)
  fabric_ref the reference generator's fabric (per-pod emplace quirk kept)
  fabric_rtt fabric_full wiring with RTT-derived metrics: the weighted path
  wan_ksp2   configs[3]: getKthPaths(s, d, 1) and (s, d, 2) for ALL pairs of the
             2000-node WAN graph; sources sharded over ranks (strong scaling),
             every rank's paths gathered to rank 0 with RCCL inside the step.
  ba_whatif  configs[4]: SPF of one source re-run for every single-link failure
             of a 250k-node / 1M-link scale-free graph, per-failure digests;
             failures sharded over ranks, digests gathered with RCCL.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload fabric_full]
    python bench.py --devices 0,0,0,0 [--graphs]      (one process, 4 members)
    torchrun --nproc-per-node N bench.py --gpus N ...
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "all-sources SPF solves/sec + GTEPS, 10k-node fabric, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)


def cpu_model() -> str:
    try:
        return next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                    if l.startswith("model name"))
    except Exception:  # noqa: BLE001
        return "unknown"


def oracle():
    sys.path.insert(0, str(ROOT / "tests"))
    from oracle import OracleLinkState  # CPU baseline leg only

    return OracleLinkState


class Buf:
    """A device buffer: `ptr` for the C-ABI, `t` the torch tensor on
    multi-rank runs (collectives), numpy() a host copy."""

    def __init__(self, dev, n: int, dtype, zero: bool) -> None:
        self.n, self.dtype = int(n), np.dtype(dtype)
        if dev.torch is not None:
            tt = {np.dtype(np.int32): dev.torch.int32, np.dtype(np.int64): dev.torch.int64}[self.dtype]
            mk = dev.torch.zeros if zero else dev.torch.empty
            self.t = mk(max(1, self.n), dtype=tt, device=dev.device)
            self.ptr = self.t.data_ptr()
            self.h = None
        else:
            from openr_amd.hiprt import DeviceArray

            self.t = None
            self.h = DeviceArray(self.n, self.dtype, zero=zero)
            self.ptr = self.h.ptr

    def numpy(self) -> np.ndarray:
        return self.t.cpu().numpy() if self.t is not None else self.h.numpy()

    def free(self) -> None:
        if self.h is not None:
            self.h.free()
        self.t = None


class Dev:
    """Device plumbing.  One rank: openr_amd.hiprt (the HIP runtime
    libopenr_spf.so links, no torch in the process).  Several ranks: torch,
    for torch.distributed over RCCL; kernels go on torch's current stream."""

    def __init__(self, local: int, world: int) -> None:
        self.index, self.world = local, world
        self.bufs = []
        if world > 1:
            import torch

            torch.cuda.set_device(local)
            self.torch, self.device = torch, torch.device("cuda", local)
        else:
            from openr_amd import hiprt

            hiprt.set_device(local)
            self.torch, self.device, self.hip = None, None, hiprt

    def buf(self, n: int, dtype=np.int32, zero: bool = False) -> Buf:
        b = Buf(self, n, dtype, zero)
        self.bufs.append(b)
        return b

    def stream(self) -> int:
        """hipStream_t for the engine's execute calls (0 = the engine's own)."""
        return self.torch.cuda.current_stream(self.device).cuda_stream if self.torch else 0

    def sync(self) -> None:
        if self.torch:
            self.torch.cuda.synchronize(self.device)
        else:
            self.hip.synchronize()

    def close(self) -> None:
        for b in self.bufs:
            b.free()
        self.bufs = []


_FNV_P = 0x100000001b3
_M64 = (1 << 64) - 1


def link_value_hash(a: str, b: str, c: str, d: str) -> int:
    """A link's value identity for digests: FNV-1a over its ordered key
    (node, ifname, node, ifname), each part closed by a 0x01 byte, then
    splitmix64's finaliser -- the hash the committed KSP2 fixtures use, so
    engine digests (spf_ksp2_digest) compare with them."""
    f = 0xcbf29ce484222325
    for part in (a, b, c, d):
        for ch in part.encode():
            f = ((f ^ ch) * _FNV_P) & _M64
        f = ((f ^ 0x01) * _FNV_P) & _M64
    f = ((f ^ (f >> 30)) * 0xbf58476d1ce4e5b9) & _M64
    f = ((f ^ (f >> 27)) * 0x94d049bb133111eb) & _M64
    return f ^ (f >> 31)


def make_topology(name: str):
    """The all-sources workloads' synthetic topologies: (Topology, description)."""
    from openr_amd import topology as T

    if name == "fabric_full":
        return T.fabric(10000, full=True), \
            "fabric_full numOfSws=10000 (RoutingBenchmarkUtils.cpp:247-400, every pod wired)"
    if name == "fabric_ref":
        return T.fabric(10000, full=False), \
            "fabric_ref numOfSws=10000 (reference generator incl. per-pod emplace quirk)"
    if name == "fabric_rtt":
        return T.fabric_rtt(), ("fabric_full wiring, per-direction metrics max(rtt/100,1) from "
                                "seeded RTTs (LinkMonitor.cpp:44-47), weighted SPF")
    if name == "grid100":
        return T.grid(100), "grid 100x100 (RoutingBenchmarkUtils.cpp:161-240)"
    raise ValueError(name)


class AllSources:
    """configs[1]/[2]: one all-sources SPF + ECMP pass per step.

    strong scaling (default), results resident (default): one LSDB, its
    sources split over the ranks balanced by next-hop work, grouped so each
    rank's closure stays small (sharding.AllSourcesLayout: contiguous id
    blocks or the locality partition); every rank writes its sources' distance
    rows and next-hop bitmaps into buffers that stay in its HBM -- the
    sharded result the facade serves getSpfResult(node) from on the owning
    rank (Decision::getDecisionRouteDb per node, Decision.cpp:1480-1500).  No
    data-path collective inside the step; after the timed steps every rank
    digests its rows on the GPU (spf_plan_digest) and rank 0 gathers the
    digests (RCCL) and checks every source against the oracle's committed
    digests.  --results gather (labelled extra) instead gathers every rank's
    rows and bitmaps to rank 0 inside the step.  --scaling weak: rank r
    solves its own LSDB snapshot (rack switch r drained, BM_DecisionFabric's
    per-iteration perturbation, RoutingBenchmarkUtils.cpp:406-447)."""

    unit = "solves/s"

    def __init__(self, name: str, rank: int, world: int, dev, eng_cls, graph_from_lsdb,
                 scaling: str = "strong", results: str = "resident"):
        from openr_amd.sharding import AllSourcesLayout, snapshot_for_rank

        topo, self.desc = make_topology(name)
        self.name = name
        self.scaling = scaling
        if scaling == "weak":  # rank r's snapshot: one node drained
            topo.lsdb = snapshot_for_rank(topo.lsdb, rank)
        self.topo = topo
        names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
        self.n, self.e = len(names), len(col)
        eng = eng_cls(dev.index)
        eng.load(rp, col, met, lid, ovl)
        self.eng, self.rank, self.world, self.dev = eng, rank, world, dev
        nbrs = [eng.neighbors(s) for s in range(self.n)]
        k = np.array([len(x) for x in nbrs], np.int64)
        self.k = k
        pitch = eng.pitch
        split = scaling == "strong"
        gather = split and world > 1 and results == "gather"
        self.results = "gather" if gather else ("resident" if split else "per-rank snapshot")
        # the gathered distance rows: the plans' u8 rows when every rank's
        # are lossless (checked once below), a quarter of the u32 bytes
        layout = AllSourcesLayout(k, pitch, world if split else 1, nbrs=nbrs)
        srcs = layout.srcs[rank if split else 0]
        self.srcs = srcs
        self.plan = eng.plan(srcs)
        self.dist_bytes = 4
        if gather and self.plan.row_mode() != "u32" and self._narrow_lossless(dev, len(srcs), pitch):
            self.dist_bytes = 1
            layout = AllSourcesLayout(k, pitch, world, dist_bytes=1, nbrs=nbrs)
        self.layout = layout
        assert np.array_equal(self.plan.nh_off, self.layout.plan_nh_off(rank if split else 0))
        cap = self.layout.cap
        self.dist_words = self.layout.dist_words[rank if split else 0]
        # u8 rows on the wire: the plan's u32 rows go to a scratch buffer
        self.d32 = dev.buf(max(1, len(srcs) * pitch)) if self.dist_bytes == 1 else None
        self.nbuf = 2 if gather else 1
        self.send = [dev.buf(max(1, cap), zero=True) for _ in range(self.nbuf)]
        self.recv = ([dev.torch.zeros((world, max(1, cap)), dtype=dev.torch.int32,
                                      device=dev.device)
                      for _ in range(self.nbuf)] if gather and rank == 0 else None)
        self.works = [None] * self.nbuf
        self.gather = gather
        self.i = 0
        self.units = len(srcs)
        self.gather_bytes = 4 * sum(self.layout.words) if gather else 0
        self.wire = ("u8 distance rows (lossless: every distance < 254) + next-hop bitmaps"
                     if self.dist_bytes == 1 else "u32 distance rows + next-hop bitmaps")
        # SURVEY.md §8(d) per-solve figure (one CSR sweep charged per solve)
        n, e = self.n, self.e
        self.graph_bytes = 4 * (n + 1) + 8 * e + n  # row_ptr, col + metric, drain bits
        self.survey_bytes = int(len(srcs) * (self.graph_bytes + 4 * n)
                                + len(srcs) * int(np.sum((k[srcs] + 7) // 8)))
        # the execute's timed phases: distance kernel, row slicing (sliced
        # next-hop plans), next-hop kernel
        self.phases = self.plan.phase_kernels()
        self.kernels = tuple(k for k in self.phases if k)
        self.narrow = self.plan.row_mode()
        self._phase_bytes()
        self._algorithmic_bytes()
        self.parallelism = (
            f"sources split over {world} rank(s) ({self.layout.partition} partition, one LSDB), plan closure "
            f"{self.plan.closure_rows} rows for {len(srcs)} sources; per-source results "
            f"({self.wire}) gathered to rank 0 over RCCL in the step "
            f"({self.gather_bytes / 1e6:.0f} MB/step, send buffers double-buffered)"
            if gather else
            f"sources split over {world} rank(s) ({self.layout.partition} partition: "
            f"closure rows per rank {self.layout.closure}; one LSDB, graph replicated), "
            f"plan closure {self.plan.closure_rows} rows for {len(srcs)} sources; results "
            f"resident in each rank's HBM (no collective in the step); per-source digests "
            f"gathered to rank 0 after the timed steps"
            if split else
            f"weak: one LSDB snapshot per rank ({world} ranks), results stay on each GPU")

    def _algorithmic_bytes(self) -> None:
        """Algorithmic HBM bytes per execute and per phase: the outputs the
        path must produce (u32 distance rows, next-hop bitmaps) plus one read
        of the graph (row_ptr, col, metric, drain bits) per kernel."""
        m, n = len(self.srcs), self.n
        rows = 4 * m * n
        bitmaps = 4 * int(self.plan.nh_words)
        g = self.graph_bytes
        alg = {}
        bfs, sl, ecmp = self.phases
        if ecmp is None:  # exact / big kernels: rows and next hops in one kernel
            alg[bfs] = rows + bitmaps + g
        else:
            alg[bfs] = rows + g
            if sl:
                alg[sl] = 0  # an internal transform: no algorithmic output
            alg[ecmp] = bitmaps + g
        self.alg_bytes = alg
        self.alg_execute_bytes = rows + bitmaps + g

    def step(self) -> None:
        b = self.i % self.nbuf
        self.i += 1
        if self.works[b] is not None:  # the gather that last read this buffer
            self.works[b].wait()
        buf = self.send[b]
        if self.d32 is None:
            self.plan.execute(buf.ptr, buf.ptr + 4 * self.dist_words, self.dev.stream())
        else:
            self.plan.execute(self.d32.ptr, buf.ptr + 4 * self.dist_words, self.dev.stream())
            self.plan.copy_narrow_rows(buf.ptr, self.dev.stream())
        if self.gather:
            import torch.distributed as dist

            out = list(self.recv[b].unbind(0)) if self.rank == 0 else None
            self.works[b] = dist.gather(buf.t, out, dst=0, async_op=True)

    def verify(self):
        """Untimed, after the timed steps: every rank digests the rows and
        bitmaps its last execute left in its HBM (spf_plan_digest, on the
        GPU), rank 0 gathers the digests (RCCL) and compares every source with
        the oracle's committed digests (tests/golden/fullsize_<workload>.npz,
        oracle/spf_oracle.cpp).  None when there is nothing to compare (weak
        snapshots, u8 wire rows, no golden file)."""
        if self.results == "per-rank snapshot" or self.dist_bytes != 4:
            return None
        buf = self.send[(self.i - 1) % self.nbuf]
        m = len(self.srcs)
        dg = self.dev.buf(max(1, m), np.int64, zero=True)
        self.plan.digest(buf.ptr, buf.ptr + 4 * self.dist_words, dg.ptr, self.dev.stream())
        self.dev.sync()
        self.eng.check()
        if self.world > 1:
            from openr_amd.sharding import gather_padded

            got = gather_padded(dg.t, m)
            parts = [g.cpu().numpy().view(np.uint64) for g in got] if self.rank == 0 else None
        else:
            parts = [dg.numpy()[:m].view(np.uint64)]
        if self.rank != 0:
            return None
        digest = self.layout.assemble_digests(parts)
        gold = ROOT / "tests" / "golden" / f"fullsize_{self.name}.npz"
        if not gold.exists():
            return {"checked_sources": 0, "note": f"no {gold.name}"}
        z = np.load(gold)  # allow_pickle=False (default): arrays only
        want = np.zeros(self.n, np.uint64)
        want[z["srcs"].astype(np.int64)] = z["digest"].astype(np.uint64)
        bad = np.nonzero(digest != want)[0]
        return {"checked_sources": int(len(z["srcs"])), "mismatches": int(len(bad)),
                "first_mismatch": int(bad[0]) if len(bad) else None,
                "against": f"tests/golden/{gold.name} (oracle/spf_oracle.cpp digests of every "
                           "source), engine digests from spf_plan_digest on each rank's "
                           "resident rows, gathered to rank 0"}

    def _narrow_lossless(self, dev, m: int, pitch: int) -> bool:
        """One untimed execute: are this rank's u8 rows exact (no distance
        >= 254)?  Agreed over all ranks (every rank must ship the same form)."""
        import torch
        import torch.distributed as dist

        d32 = dev.buf(max(1, m * pitch))
        nh = dev.buf(max(1, int(self.plan.nh_words)))
        d8 = dev.buf(max(1, m * pitch // 4))
        self.plan.execute(d32.ptr, nh.ptr, dev.stream())
        self.plan.copy_narrow_rows(d8.ptr, dev.stream())
        a = d32.t[: m * pitch].to(torch.int64) & 0xFFFFFFFF
        b = d8.t.view(torch.uint8)[: m * pitch].to(torch.int64)
        inf = 0xFFFFFFFF
        ok = bool(((a == inf) | (a < 254)).all()) and bool(torch.equal(torch.where(a == inf, 255, a), b))
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        for x in (d32, nh, d8):
            x.free()
        return bool(flag.item())

    def finish(self) -> None:
        for w in self.works:
            if w is not None:
                w.wait()

    def enable_timing(self, k: int) -> None:
        self.plan.enable_timing(k)

    def _phase_bytes(self) -> None:
        tb = self.plan.traffic_phases()  # sliced plans: planes of the last execute
        self.kernel_bytes = {k: b for k, b in zip(self.phases, tb) if k}

    def kernel_ms(self):
        ms, cnt = self.plan.timing_phases()
        self._phase_bytes()
        return {k: t / max(cnt, 1) for k, t in zip(self.phases, ms) if k}

    def edges_per_unit(self) -> int:
        return self.e

    def cpu_baseline(self, budget_s: float):
        """The CPU oracle (faithful restatement of LinkState::runSpf, kind
        'port') timed on this host, 1 core, on a seeded sample of sources of
        the same workload, until `budget_s` seconds of work have accumulated."""
        orc = oracle()()
        orc.update_packed(self.topo.lsdb)
        order = np.random.default_rng(0).permutation(self.topo.n_nodes)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s and done < len(order):
            batch = [self.topo.nodes[int(i)] for i in order[done: done + 4]]
            orc.time_sources(batch)
            done += len(batch)
        dt = time.perf_counter() - t0
        one = {"value": done / dt, "cores": 1,
               "sample": f"{done} seeded-random sources of the same topology, full runSpf "
                         f"each ({dt:.1f} s on 1 core of {cpu_model()}; oracle/spf_oracle.cpp)"}
        multi = self.cpu_baseline_threads(budget_s / 2)
        return {"value": multi["value"], "unit": "solves/s", "cores": multi["cores"],
                "kind": "port", "sample": multi["sample"], "single_core": one}

    def cpu_baseline_threads(self, budget_s: float):
        """The same oracle on every host core this job may use (the box's
        share: $OMP_NUM_THREADS, 16 on the GPU pool): one LinkState replica
        per thread, seeded sources dealt round-robin (the
        reference itself is single-threaded).  ctypes drops the GIL for the
        C++ calls, so the threads run in parallel."""
        import threading

        cores = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1, 16))
        order = np.random.default_rng(1).permutation(self.topo.n_nodes)
        ready = threading.Barrier(cores + 1)
        counts = [0] * cores
        stop = [False]

        def work(t: int) -> None:
            orc = oracle()()
            orc.update_packed(self.topo.lsdb)
            mine = order[t::cores]
            ready.wait()
            i = 0
            while not stop[0] and i < len(mine):
                orc.time_sources([self.topo.nodes[int(x)] for x in mine[i: i + 2]])
                i += 2
                counts[t] = i
        threads = [threading.Thread(target=work, args=(t,)) for t in range(cores)]
        for th in threads:
            th.start()
        ready.wait()
        t0 = time.perf_counter()
        time.sleep(budget_s)
        stop[0] = True
        for th in threads:
            th.join()
        dt = time.perf_counter() - t0
        done = sum(counts)
        return {"value": done / dt, "cores": cores,
                "sample": f"{done} seeded-random sources of the same topology, full runSpf each, "
                          f"{cores} threads x one LinkState replica ({dt:.1f} s wall on "
                          f"{cpu_model()}; oracle/spf_oracle.cpp)"}


class AllSourcesMulti(AllSources):
    """configs[1]/[2] through the single-process multi-device context
    (spf_mctx / spf_mplan, include/openr_spf.h): ONE process -- as Open/R's
    Decision is (Decision.cpp:1484) -- drives every listed GPU; the sources
    are split over the members (locality partition), every member's rows and
    bitmaps stay in its HBM, digests are checked after the timed steps.
    Device ids may repeat (--devices 0,0,0,0 on a one-GPU box): members of one
    device then run one after another on it, so the per-member times are what
    each GPU of an N-GPU node would take (the slowest sets an N-GPU step)."""

    def __init__(self, name: str, devices, graphs: bool = False):
        from openr_amd.engine import SpfMultiEngine, graph_from_lsdb

        topo, self.desc = make_topology(name)
        self.name, self.topo, self.scaling = name, topo, "strong"
        names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
        self.n, self.e = len(names), len(col)
        self.devices = list(devices)
        self.m = SpfMultiEngine(self.devices)
        self.m.load(rp, col, met, lid, ovl)
        self.eng = self.m.member0
        self.plan = self.m.plan(np.arange(self.n, dtype=np.uint32))
        self.plan.set_graphs(graphs)
        self.graphs = graphs
        self.units = self.n
        self.results = "resident"
        self.narrow = self.plan.member_kernels(0)[0]
        k = np.array([len(self.m.neighbors(s)) for s in range(self.n)], np.int64)
        wpm = self.m.pitch // 32
        self.graph_bytes = 4 * (self.n + 1) + 8 * self.e + self.n
        # per member: its u32 rows + bitmaps + one graph read
        self.member_bytes = []
        for i in range(len(self.devices)):
            mine = [s for s in range(self.n) if self.plan.owner(s)[0] == i]
            self.member_bytes.append(4 * len(mine) * self.n + 4 * int(k[mine].sum()) * wpm
                                     + self.graph_bytes)
        self.survey_bytes = int(self.n * (self.graph_bytes + 4 * self.n) + self.n * int(np.sum((k + 7) // 8)))
        self.kernels = ("execute",)
        self.parallelism = (
            f"one process, {len(self.devices)} member(s) on device(s) {self.devices} "
            f"(spf_mctx); {self.plan.partition} partition, closure rows per member "
            f"{self.plan.closure_rows}, sources per member {self.plan.shard_sizes()}; results "
            f"resident on each member (no copy in the step); hipGraph replays "
            f"{'on' if graphs else 'off'}")

    def step(self) -> None:
        self.plan.execute()

    def finish(self) -> None:
        self.plan.synchronize()

    def verify(self):
        digest = self.plan.digest()
        gold = ROOT / "tests" / "golden" / f"fullsize_{self.name}.npz"
        if not gold.exists():
            return {"checked_sources": 0, "note": f"no {gold.name}"}
        z = np.load(gold)
        want = np.zeros(self.n, np.uint64)
        want[z["srcs"].astype(np.int64)] = z["digest"].astype(np.uint64)
        bad = np.nonzero(digest != want)[0]
        return {"checked_sources": int(len(z["srcs"])), "mismatches": int(len(bad)),
                "first_mismatch": int(bad[0]) if len(bad) else None,
                "against": f"tests/golden/{gold.name}, engine digests (spf_mplan_digest) of "
                           "every member's resident rows"}

    def enable_timing(self, k: int) -> None:
        self.plan.enable_timing(k)

    def kernel_ms(self):
        ms, cnt = self.plan.timing()
        self.member_ms = [t / max(cnt, 1) for t in ms]
        slow = int(np.argmax(self.member_ms))
        self.alg_bytes = {"execute": self.member_bytes[slow]}
        self.alg_execute_bytes = self.member_bytes[slow]
        self.kernel_bytes = {"execute": self.member_bytes[slow]}
        return {"execute": self.member_ms[slow]}


def enqueue_stagger(wl, reps: int) -> dict:
    """Host enqueue of an execute (after the timed steps, untimed): per member,
    us from spf_mplan_execute's start until that member's launches were
    enqueued -- the start stagger separate GPUs would see -- issued one member
    after another from this thread, then from per-member threads
    (spf_mplan_set_enqueue_threads)."""
    out = {}
    wl.plan.enable_timing(0)  # production executes: no timing events
    for mode, graphs, key in ((0, False, "serial"), (1, False, "threads"), (0, True, "serial_graphs")):
        wl.plan.set_enqueue_threads(mode)
        wl.plan.set_graphs(graphs)
        wl.plan.execute()  # (a graph capture happens on the first execute)
        wl.plan.synchronize()
        rows = []
        for _ in range(reps):
            wl.plan.execute()
            ns, _thr = wl.plan.enqueue_ns()
            rows.append(ns.astype(np.float64) / 1e3)
            wl.plan.synchronize()
        a = np.median(np.array(rows), axis=0)
        out[key] = {"member_done_us": [round(float(x), 1) for x in a],
                    "stagger_us": round(float(a.max() - a[a > 0].min()) if (a > 0).any() else 0.0, 1),
                    "last_member_us": round(float(a.max()), 1)}
    wl.plan.set_enqueue_threads(-1)
    wl.plan.set_graphs(wl.graphs)
    out["note"] = ("median over %d executes without timing events; members of one device share "
                   "its stream, so the threads row here times only the host side; serial_graphs: "
                   "each member's execute replayed from a captured hipGraph" % reps)
    return out


class Ksp2AllPairs:
    """configs[3]: KSP2 (k = 1 and k = 2 paths) for every pair of the WAN
    graph; sources dealt round-robin over ranks (strong scaling), the ranks'
    pair headers and path pools gathered to rank 0 with RCCL in the step."""

    scaling = "strong"
    unit = "pairs/s"
    kernels = ("sssp_kernel", "ksp2_kernel")

    def __init__(self, name: str, rank: int, world: int, dev, eng_cls, graph_from_lsdb):
        from openr_amd import topology as T
        from openr_amd.engine import PAIR_DTYPE

        self.topo = T.wan(2000, 1000, seed=1)
        self.desc = "wan N=2000, ring + 1000 seeded chords, metrics U[1,1000] (SURVEY.md §8(d) config 4)"
        names, rp, col, met, lid, ovl = graph_from_lsdb(self.topo.lsdb)
        self.n, self.e = len(names), len(col)
        eng = eng_cls(dev.index)
        eng.load(rp, col, met, lid, ovl)
        self.eng, self.dev, self.rank, self.world = eng, dev, rank, world
        self.srcs = list(range(rank, self.n, world))
        self.plan = eng.ksp2_plan(self.srcs)
        n_pairs = len(self.srcs) * self.n
        self.units = n_pairs
        self.pair_words = PAIR_DTYPE.itemsize // 4
        self.d_pairs = dev.buf(n_pairs * self.pair_words)
        self.d_cnt = dev.buf(4, np.int64, zero=True)
        # size the path pool with one untimed sizing run (the counter keeps
        # counting past an overflow)
        self.pool_words = 1 << 20
        pool0 = dev.buf(self.pool_words)
        self.plan.execute(self.d_pairs.ptr, pool0.ptr, self.pool_words, self.d_cnt.ptr, 0)
        dev.sync()
        self.pool_words = int(int(self.d_cnt.numpy()[0]) * 1.05) + (1 << 22)
        self.d_pool = dev.buf(self.pool_words)
        self.gathered = 0
        # one k = 2 solve per pair (B_solve without next hops)
        # + 4 B per output link; the k = 1 SPF rows are charged per source.
        n, e = self.n, self.e
        self.b_solve = 4 * (n + 1) + 8 * e + n + 4 * n
        self.survey_bytes = None  # known after the first execute (output links)
        self.parallelism = (f"sources dealt round-robin over {world} rank(s), graph replicated; "
                            "pair headers + path pools gathered to rank 0 (RCCL gather) in the step")

    def step(self) -> None:
        self.plan.execute(self.d_pairs.ptr, self.d_pool.ptr, self.pool_words, self.d_cnt.ptr,
                          self.dev.stream())
        if self.world > 1:
            # one exchange: every rank's pair headers and path pool to rank 0
            from openr_amd.sharding import gather_padded

            used = min(int(self.d_cnt.t[0].item()), self.d_pool.t.numel())
            gather_padded(self.d_pairs.t, self.d_pairs.t.numel())
            gather_padded(self.d_pool.t, used)

    def enable_timing(self, k: int) -> None:
        self.plan.enable_timing(k)

    def verify(self):
        """Untimed, after the timed steps: every rank digests the pairs and
        path pool its last execute left (spf_ksp2_digest, on the GPU), rank 0
        gathers the per-source digests and compares EVERY source with the
        oracle's (tests/golden/fullsize_wan2k_ksp2_all.npz: getKthPaths k = 1,
        2 for all 4M pairs, oracle/spf_oracle.cpp)."""
        from openr_amd.link_state import LinkState

        gold = ROOT / "tests" / "golden" / "fullsize_wan2k_ksp2_all.npz"
        ls = LinkState(device=-1)
        ls.updateAdjacencyDatabases(self.topo.lsdb)
        lid = ls.flatten()[4]
        lh = np.zeros(int(lid.max()) + 1, np.uint64)
        for l in np.unique(lid):
            (a, b), (c, d) = ls._link(int(l)).orderedNames
            lh[int(l)] = link_value_hash(a, b, c, d)
        ls.close()
        d_lh = self.dev.buf(len(lh), np.int64)
        if d_lh.t is not None:
            import torch

            d_lh.t.copy_(torch.from_numpy(lh.view(np.int64)))
        else:
            d_lh.h.upload(lh.view(np.int64))
        m = len(self.srcs)
        dg = self.dev.buf(max(1, m), np.int64, zero=True)
        self.plan.digest(self.d_pairs.ptr, self.d_pool.ptr, d_lh.ptr, dg.ptr, self.dev.stream())
        self.dev.sync()
        self.eng.check()
        if self.world > 1:
            from openr_amd.sharding import gather_padded

            got = gather_padded(dg.t, m)
            parts = [g.cpu().numpy().view(np.uint64) for g in got] if self.rank == 0 else None
        else:
            parts = [dg.numpy()[:m].view(np.uint64)]
        if self.rank != 0:
            return None
        digest = np.zeros(self.n, np.uint64)
        for r, part in enumerate(parts):
            digest[np.arange(r, self.n, self.world)] = part[: len(range(r, self.n, self.world))]
        if not gold.exists():
            return {"checked_sources": 0, "note": f"no {gold.name}"}
        z = np.load(gold)
        want = np.zeros(self.n, np.uint64)
        want[z["srcs"].astype(np.int64)] = z["digest"].astype(np.uint64)
        bad = np.nonzero(digest[z["srcs"]] != want[z["srcs"]])[0]
        return {"checked_sources": int(len(z["srcs"])),
                "checked_pairs": int(len(z["srcs"])) * self.n, "mismatches": int(len(bad)),
                "first_mismatch": int(z["srcs"][bad[0]]) if len(bad) else None,
                "against": f"tests/golden/{gold.name} (oracle getKthPaths k=1,2 of every pair), "
                           "engine digests from spf_ksp2_digest on each rank's last execute"}

    def kernel_ms(self):
        a, b, cnt = self.plan.timing()
        cnt_h = self.d_cnt.numpy()
        if cnt_h[2] & 1:
            raise SystemExit("KSP2 path pool overflowed: raise pool_words")
        # path pool words = records [len, next, links]; output links ~ words
        self.survey_bytes = int(self.units * self.b_solve + len(self.srcs) * self.b_solve
                                + 4 * int(cnt_h[0]))
        self.k2_runs = int(cnt_h[1])
        # compulsory bytes: the k = 1 SPF reads the CSR once per source and
        # writes a distance row; the KSP2 kernel stages the graph once per
        # block (destination x the plan's source chunk) and writes the pair
        # records and path pool once
        n, e = self.n, self.e
        csr = 4 * (n + 1) + 12 * e
        chunk = self.plan.chunk()
        blocks = n * ((len(self.srcs) + chunk - 1) // chunk)
        self.kernel_bytes = {
            "sssp_kernel": len(self.srcs) * (4 * (n + 1) + 8 * e + n + 4 * self.eng.pitch),
            "ksp2_kernel": blocks * csr + 16 * self.units + 4 * int(cnt_h[0])}
        # algorithmic: the k = 1 distance rows (u32) + one graph read; the
        # pair records (16 B) + path pool + one graph read (incl. link ids)
        g = 4 * (n + 1) + 8 * e + n
        self.alg_bytes = {"sssp_kernel": 4 * len(self.srcs) * n + g,
                          "ksp2_kernel": 16 * self.units + 4 * int(cnt_h[0]) + g + 4 * e}
        self.alg_execute_bytes = sum(self.alg_bytes.values())
        return {"sssp_kernel": a / max(cnt, 1), "ksp2_kernel": b / max(cnt, 1)}

    def edges_per_unit(self) -> int:
        return self.e

    def cpu_baseline(self, budget_s: float):
        orc = oracle()()
        orc.update_packed(self.topo.lsdb)
        rng = np.random.default_rng(0)
        src = self.topo.nodes[int(rng.integers(self.n))]
        dsts = [self.topo.nodes[int(i)] for i in rng.permutation(self.n)]
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s and done < len(dsts):
            orc.time_ksp2(src, dsts[done: done + 16])
            done += 16
        dt = time.perf_counter() - t0
        return {"value": done / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
                "sample": f"{done} seeded-random destinations of one source, getKthPaths k=1 "
                          f"and k=2 each ({dt:.1f} s on 1 core of {cpu_model()}; "
                          "oracle/spf_oracle.cpp)"}


class WhatIfAllLinks:
    """configs[4]: SPF of node "0" re-run for every single-link failure of the
    Barabasi-Albert graph (250k nodes, ~1M links), one digest per failure
    (include/openr_spf.h spf_whatif_*).  Failures dealt round-robin over ranks
    (strong scaling); every rank recomputes the unfailed SPF and its digests
    are gathered to rank 0 with RCCL inside the step."""

    scaling = "strong"
    unit = "failures/s"
    kernels = ("base", "failures")

    def __init__(self, name: str, rank: int, world: int, dev, eng_cls, graph_from_lsdb):
        from openr_amd import topology as T
        from openr_amd.engine import DIGEST_DTYPE
        from openr_amd.link_state import LinkState

        self.topo = T.barabasi_albert(250_000, 4, seed=1)
        self.desc = ("Barabasi-Albert N=250000 m=4 seed=1, metrics U[1,16]; source \"0\"; "
                     "every single-link failure (SURVEY.md §8(d) config 5)")
        ls = LinkState(device=-1)
        ls.updateAdjacencyDatabases(self.topo.lsdb)
        names, rp, col, met, lid, ovl = ls.flatten()
        self.ls, self.names = ls, names
        self.n, self.e = len(names), len(col)
        eng = eng_cls(dev.index)
        eng.load(rp, col, met, lid, ovl)
        self.eng, self.dev, self.rank, self.world = eng, dev, rank, world
        self.src = names.index("0")
        all_links = np.unique(lid).astype(np.uint32)  # every up link
        self.links = all_links[rank::world]
        self.plan = eng.whatif_plan(self.src, self.links)
        self.units = len(self.links)
        self.d_out = dev.buf(max(1, self.units) * DIGEST_DTYPE.itemsize // 8, np.int64)
        self.d_base = dev.buf(2, np.int64)
        # a what-if solve is B_solve with a 24 B digest in
        # place of the dense result: 4(N+1) + 8E + N + 24
        n, e = self.n, self.e
        self.survey_bytes = int((self.units + 1) * (4 * (n + 1) + 8 * e + n + 24))
        # compulsory bytes: the unfailed pass reads the CSR (row_ptr, col,
        # metric, link id) once and writes distances + next-hop rows; the
        # failure pass reads the failure list and the CSR once and writes a
        # 16-byte digest per failure (affected regions re-read the CSR, which
        # is repair work, not charged)
        csr = 4 * (n + 1) + 12 * e + n
        words = (len(eng.neighbors(self.src)) + 31) // 32
        self.kernel_bytes = {"base": csr + 4 * n + 4 * words * n,
                             "failures": csr + 4 * self.units + 16 * self.units}
        # algorithmic: the unfailed distances + next-hop words + one graph
        # read; the failure list, one graph read and a digest per failure
        g = 4 * (n + 1) + 8 * e + n
        self.alg_bytes = {"base": g + 4 * n + 4 * words * n,
                          "failures": g + 4 * self.units + 16 * self.units}
        self.alg_execute_bytes = sum(self.alg_bytes.values())
        self.pmc_kernels = {"base": ["whatif_base_kernel"],
                            "failures": ["classify_kernel", "sort_big_kernel", "repair_wave_kernel",
                                         "repair_group_kernel", "repair_block_kernel",
                                         "base_digest_kernel"]}
        self.parallelism = (f"failures dealt round-robin over {world} rank(s), graph replicated, "
                            "unfailed SPF recomputed per rank; digests gathered to rank 0 "
                            "(RCCL gather) in the step")

    def step(self) -> None:
        self.plan.execute(self.d_out.ptr, self.d_base.ptr, self.dev.stream())
        if self.world > 1:  # one exchange: every rank's digests to rank 0
            from openr_amd.sharding import gather_padded

            gather_padded(self.d_out.t, self.d_out.t.numel())

    def enable_timing(self, k: int) -> None:
        self.plan.enable_timing(k)

    def verify(self):
        """Untimed, after the timed steps: the digests of the failures the
        committed fixture holds (tests/golden/fullsize_ba250k_whatif.npz:
        16.5k of the step's ~1M failures -- uniform and tight links and the
        3000 shortest-path-tree links with the largest subtrees, oracle
        runSpf(src, true, {l})), read from the last execute's output on the
        rank that computed them, compared at rank 0; plus the unfailed
        digest."""
        from openr_amd.engine import DIGEST_DTYPE

        gold = ROOT / "tests" / "golden" / "fullsize_ba250k_whatif.npz"
        if not gold.exists():
            return {"checked_failures": 0, "note": f"no {gold.name}"}
        z = np.load(gold)
        self.dev.sync()
        self.eng.check()
        mine = self.d_out.numpy().view(DIGEST_DTYPE)[: self.units]
        base = self.d_base.numpy().view(DIGEST_DTYPE)[0]
        pos = np.searchsorted(self.links, z["links"])
        ok = (pos < len(self.links)) & (self.links[np.minimum(pos, len(self.links) - 1)] == z["links"])
        sel = np.nonzero(ok)[0]
        bad_local = sum(int(np.count_nonzero(mine[f][pos[sel]] != z[f][sel]))
                        for f in ("n_dist_changed", "n_nh_changed", "hash"))
        base_ok = (int(base["n_dist_changed"]), int(base["n_nh_changed"]), int(base["hash"])) == \
            tuple(int(x) for x in z["base"])
        checked = len(sel)
        if self.world > 1:
            import torch
            import torch.distributed as dist

            t = torch.tensor([checked, bad_local, 0 if base_ok else 1], dtype=torch.int64,
                             device=self.dev.device)
            dist.all_reduce(t)
            checked, bad_local, base_bad = (int(x) for x in t.tolist())
            base_ok = base_bad == 0
        if self.rank != 0:
            return None
        return {"checked_failures": int(checked), "mismatches": int(bad_local) + (0 if base_ok else 1),
                "unfailed_digest_ok": bool(base_ok),
                "against": f"tests/golden/{gold.name} (oracle runSpf(\"0\", true, {{l}}) digests "
                           "of 16.5k failures incl. the largest repairs), the step's own output"}

    def kernel_ms(self):
        a, b, cnt = self.plan.timing()
        self.n_hot, self.n_big = self.plan.stats()
        return {"base": a / max(cnt, 1), "failures": b / max(cnt, 1)}

    def edges_per_unit(self) -> int:
        return self.e - 2

    def cpu_baseline(self, budget_s: float):
        orc = oracle()()
        from oracle import time_whatif  # tests/ is on sys.path now

        orc.update_packed(self.topo.lsdb)
        rng = np.random.default_rng(0)
        order = rng.permutation(len(self.links))
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s and done < len(order):
            lk = self.ls._link(int(self.links[order[done]]))
            time_whatif(orc, "0", [(lk._n1, lk._if1)], fast=True)
            done += 1
        dt = time.perf_counter() - t0
        return {"value": done / dt, "unit": "failures/s", "cores": 1, "kind": "port",
                "sample": f"{done} seeded-random single-link failures, one full runSpf each "
                          f"({dt:.1f} s on 1 core of {cpu_model()}; oracle/spf_oracle.cpp "
                          "runSpfFast: same result as the reference's runSpf with a lazy heap "
                          "instead of make_heap per decrease, which needs ~18 min per run on "
                          "this graph)"}


class FacadeLfa:
    """CS-1 latency through the LinkState facade (the C-ABI drop-in): after an
    adjacency-database publication that drains (or undrains) one rack switch
    -- BM_DecisionFabric's per-iteration perturbation,
    RoutingBenchmarkUtils.cpp:406-447 -- the SPFs a route build with LFA
    needs: getSpfResult(me) and getSpfResult(n) for every neighbour n
    (Decision.cpp:1107-1196), each a full SpfResult (metrics, next hops,
    pathLinks) in host memory.  A step = one publication + those 1 + deg(me)
    results; value = steps per second, ms_per_step = the latency."""

    scaling = "replicas"
    unit = "lfa_spf_sets/s"
    kernels = ("facade",)

    def __init__(self, name: str, rank: int, world: int, dev, eng_cls, graph_from_lsdb):
        from openr_amd import topology as T
        from openr_amd.link_state import LinkState
        from openr_amd.wire import unpack

        self.topo = T.fabric(10000, full=True)
        self.desc = ("fabric_full numOfSws=10000; me = rack switch 3-0-0; per step one publication "
                     "toggling rack switch 3-1-0's overload bit, then getSpfResult(me) + "
                     "getSpfResult(neighbour) for each of me's neighbours (LFA)")
        self.ls = LinkState(device=dev.index)
        self.ls.updateAdjacencyDatabases(self.topo.lsdb)
        self.me = "3-0-0"
        self.nbrs = sorted({l.getOtherNodeName(self.me) for l in self.ls.linksFromNode(self.me)})
        names = self.ls.flatten()[0]
        self.n, self.e = len(names), len(self.ls.flatten()[2])
        dbs = {d.thisNodeName: d for d in unpack(self.topo.lsdb)}
        self.victim = dbs["3-1-0"]
        self.units = 1
        self.world = world
        self.i = 0
        self.kernel_bytes = {"facade": 1}
        self.survey_bytes = 0
        self.parallelism = "one LinkState per process (replicas)"
        self.lat, self.pub = [], []
        self.prefetch = os.environ.get("BENCH_LFA_PREFETCH", "1") != "0"

    def step(self) -> None:
        # the C-ABI the C++ binding calls: the results are
        # the LinkState's memo arrays (ls_spf_view); no Python objects built.
        # me + every neighbour in one batched plan (ls_prefetch_spf_results,
        # what SpfSolver's LFA does), then the per-node getSpfResult reads
        t0 = time.perf_counter()
        self.victim.isOverloaded = not self.victim.isOverloaded
        self.ls.updateAdjacencyDatabase(self.victim)
        t1 = time.perf_counter()
        if self.prefetch:
            self.ls.prefetchSpfResults([self.me] + self.nbrs)
        for node in [self.me] + self.nbrs:
            v = self.ls._spf_view(node)
            assert v.n > 0
        t2 = time.perf_counter()
        self.lat.append(t2 - t0)
        self.pub.append(t1 - t0)

    def enable_timing(self, k: int) -> None:
        self.lat, self.pub = [], []
        self.ph0 = self.ls.debugPhaseNs()

    def kernel_ms(self):
        ph = [(b - a) / 1e6 / max(1, len(self.lat)) for a, b in zip(self.ph0, self.ls.debugPhaseNs())]
        self.phase_ms = {"publication (updateAdjacencyDatabase; the CSR patch runs in the first query)":
                         1e3 * float(np.mean(self.pub)) if self.pub else 0.0,
                         "plan build": ph[0], "GPU execute + copy back": ph[1],
                         "pathLinks (batched preds kernel + copy back)": ph[2],
                         "host result assembly": ph[3]}
        return {"facade": 1e3 * float(np.mean(self.lat)) if self.lat else 0.0}

    def edges_per_unit(self) -> int:
        return self.e * (1 + len(self.nbrs))

    def cpu_baseline(self, budget_s: float):
        orc = oracle()()
        orc.update_packed(self.topo.lsdb)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s:
            orc.time_sources([self.me] + self.nbrs)
            done += 1
        dt = time.perf_counter() - t0
        return {"value": done / dt, "unit": "lfa_spf_sets/s", "cores": 1, "kind": "port",
                "sample": f"{done} x (runSpf(me) + runSpf(each of {len(self.nbrs)} neighbours)) "
                          f"({dt:.1f} s on 1 core of {cpu_model()}; oracle/spf_oracle.cpp)"}


class RoutesAllNodes:
    """CS-2: Decision::getDecisionRouteDb(node) for EVERY node
    (Decision.cpp:1480-1500, `breeze decision routes --nodes all`) on the
    10k fabric, every node advertising a loopback: per step one all-sources
    pass on the GPU (LinkState.prefetchAllSources, rows and bitmaps resident)
    and every node's route selection towards every loopback with LFA
    (getNextHopsWithMetric + getNextHopsThrift, Decision.cpp:1082-1305) from
    the resident rows (spf_mplan_route_digests), reduced to a digest per
    node on the GPU -- no per-node SPF, no host round trip per node.  Thrift
    formatting of the 100M routes is not in the step.  value = route
    databases (nodes) per second."""

    scaling = "replicas"
    unit = "route_dbs/s"
    kernels = ("allsources", "routes")

    def __init__(self, name: str, rank: int, world: int, dev, eng_cls, graph_from_lsdb):
        from openr_amd import topology as T
        from openr_amd.link_state import LinkState

        self.topo = T.fabric(10000, full=True)
        self.lfa = os.environ.get("BENCH_ROUTES_LFA", "1") != "0"
        self.desc = ("fabric_full numOfSws=10000, a loopback per node; per step: all-sources SPF "
                     "(resident) + every node's route selection towards every loopback"
                     + (" with LFA" if self.lfa else "") + " (Decision.cpp:1082-1305)")
        self.ls = LinkState(devices=[dev.index])
        self.ls.updateAdjacencyDatabases(self.topo.lsdb)
        names = self.ls.flatten()[0]
        self.names = list(names)
        self.n, self.e = len(names), len(self.ls.flatten()[2])
        self.set_ptr = np.arange(self.n + 1, dtype=np.uint32)
        self.set_nodes = np.arange(self.n, dtype=np.uint32)
        self.ls.prefetchAllSources()
        self.ls.linkValueHashes()  # cached: the digests' link identities
        self.units = self.n
        self.world = world
        self.kernel_bytes = {"allsources": 1, "routes": 1}
        self.survey_bytes = 0
        self.parallelism = "one LinkState per process (replicas); all sources resident on its GPU"
        self.t_pass, self.t_routes = [], []
        self.digests = None
        self.n_records = 0
        # algorithmic bytes of the route kernel: every resident u32 row and
        # next-hop bitmap read once, the CSR, and the outputs (digests here;
        # headers + records when materialised)
        rp = self.ls.flatten()[1].astype(np.int64)
        col = self.ls.flatten()[2].astype(np.int64)
        k = np.array([len(np.unique(col[rp[v]:rp[v + 1]])) for v in range(self.n)], np.int64)
        wpm = (self.n + 31) // 32
        self.read_bytes = 4 * self.n * self.n + 4 * int(k.sum()) * wpm + 4 * (self.n + 1) + 12 * self.e
        self.pmc_kernels = {"routes": ["route_quads_kernel"]}

    def route_step(self):
        self.digests, kms = self.ls.allSourcesRouteDigests(self.set_ptr, self.set_nodes, self.lfa)
        return kms

    def out_bytes(self) -> int:
        return 8 * self.n

    def step(self) -> None:
        t0 = time.perf_counter()
        self.ls.prefetchAllSources()  # execute + synchronize
        t1 = time.perf_counter()
        kms = self.route_step()
        self.t_pass.append(t1 - t0)
        self.t_routes.append(kms)

    def enable_timing(self, k: int) -> None:
        self.t_pass, self.t_routes = [], []

    def kernel_ms(self):
        self.phase_ms = {"all-sources pass (execute + sync, host clock)": 1e3 * float(np.mean(self.t_pass)),
                         "route selection kernel (HIP events)": float(np.mean(self.t_routes))}
        self.alg_bytes = {"allsources": 0, "routes": self.read_bytes + self.out_bytes()}
        self.kernel_bytes = dict(self.alg_bytes)
        return {"allsources": 1e3 * float(np.mean(self.t_pass)), "routes": float(np.mean(self.t_routes))}

    def edges_per_unit(self) -> int:
        return self.e

    def _oracle_digests(self, mes, orc=None, kept_min=False):
        sys.path.insert(0, str(ROOT / "tests"))
        from oracle import NameTable, route_digests  # checker / CPU baseline only

        if orc is None:
            orc = oracle()()
            orc.update_packed(self.topo.lsdb)
        return route_digests(orc, NameTable(self.names), mes, self.set_ptr, self.set_nodes, self.lfa,
                             kept_min=kept_min)

    def verify(self):
        """The last step's digests of 48 nodes (the 16 highest-degree ones
        and 32 random) against the oracle's restatement."""
        deg = np.diff(self.ls.flatten()[1].astype(np.int64))
        rng = np.random.default_rng(11)
        mes = np.unique(np.concatenate([np.argsort(-deg)[:16], rng.choice(self.n, 32, replace=False)]))
        want = self._oracle_digests(mes)
        bad = np.nonzero(self.digests[mes] != want)[0]
        return {"checked_nodes": int(len(mes)), "sets_per_node": int(len(self.set_ptr) - 1),
                "mismatches": int(len(bad)),
                "first_mismatch": self.names[int(mes[bad[0]])] if len(bad) else None,
                "against": "oracle/spf_oracle.cpp orc_ls_route_digests (getMinCostNodes + "
                           "getNextHopsWithMetric + getNextHopsThrift restated), same digest"}

    def cpu_baseline(self, budget_s: float):
        orc = oracle()()
        orc.update_packed(self.topo.lsdb)
        rng = np.random.default_rng(5)
        done, t0, mes_all = 0, time.perf_counter(), rng.permutation(self.n)
        while time.perf_counter() - t0 < budget_s and done < self.n:
            self._oracle_digests(mes_all[done:done + 4], orc)
            done += 4
        dt = time.perf_counter() - t0
        return {"value": done / dt, "unit": "route_dbs/s", "cores": host_cores(), "kind": "port",
                "sample": f"{done} nodes' route selections towards all {self.n} loopbacks"
                          f"{' with LFA' if self.lfa else ''}, their SPFs (+ neighbours') included, "
                          f"{dt:.1f} s on {host_cores()} cores of {cpu_model()} (oracle/spf_oracle.cpp)"}


class RouteDbsAllNodes(RoutesAllNodes):
    """CS-2 with every node's route database MATERIALISED:
    per step one all-sources pass and every node's next-hop records towards
    every loopback with LFA written into its GPU's HBM
    (spf_mplan_route_records: per node and route a header, per next hop a
    u64 record = CSR edge -- link, interface, neighbour -- | metric), what
    Decision::getDecisionRouteDb(node) returns for every node
    (Decision.cpp:1480-1500 -> buildRouteDb :556-722) minus the thrift
    encoding.  value = route databases (nodes) materialised per second;
    verify reads 48 nodes' databases back and checks them against the
    oracle's restatement."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.desc = self.desc.replace("route selection", "route database (next-hop records, in HBM)")

    def route_step(self):
        self.n_records, kms = self.ls.allSourcesRouteRecords(self.set_ptr, self.set_nodes, self.lfa)
        return kms

    def out_bytes(self) -> int:
        return 8 * self.n * (len(self.set_ptr) - 1) + 8 * self.n_records

    def verify(self):
        """48 nodes' databases (the 16 highest-degree and 32 random) read back,
        reduced with the digest formula, against the oracle's restatement."""
        sys.path.insert(0, str(ROOT / "tests"))
        from helpers import route_db_digest  # checker only

        deg = np.diff(self.ls.flatten()[1].astype(np.int64))
        rng = np.random.default_rng(11)
        mes = np.unique(np.concatenate([np.argsort(-deg)[:16], rng.choice(self.n, 32, replace=False)]))
        lid = self.ls.flatten()[4]
        lh = self.ls.linkValueHashes()
        got = np.array([route_db_digest(*self.ls.allSourcesRouteDb(int(t)), lid, lh) for t in mes], np.uint64)
        want = self._oracle_digests(mes, kept_min=True)
        bad = np.nonzero(got != want)[0]
        return {"checked_nodes": int(len(mes)), "sets_per_node": int(len(self.set_ptr) - 1),
                "records": int(self.n_records), "mismatches": int(len(bad)),
                "first_mismatch": self.names[int(mes[bad[0]])] if len(bad) else None,
                "against": "oracle/spf_oracle.cpp orc_ls_route_digests (getMinCostNodes + "
                           "getNextHopsWithMetric + getNextHopsThrift restated); each read-back "
                           "database reduced with the same digest (tests/helpers.py route_db_digest)"}


class FacadeRouteBuild:
    """CS-1 / CS-4 (RoutingBenchmarkUtils.cpp:406-511): after a
    publication toggling one rack switch's overload bit, SpfSolver.buildRouteDb
    (me) with LFA over the facade -- every node's loopback prefix and node
    label, adjacency labels -- as BM_DecisionFabric times it (all of
    buildRouteDb, processTimes[2]).  value = route builds per second."""

    scaling = "replicas"
    unit = "route_builds/s"
    kernels = ("route_build",)

    def __init__(self, name: str, rank: int, world: int, dev, eng_cls, graph_from_lsdb):
        from openr_amd import topology as T
        from openr_amd.link_state import LinkState
        from openr_amd.lsdb import PackedLsdb
        from openr_amd.spf_solver import PrefixEntry, PrefixState
        from openr_amd.wire import unpack

        topo = T.fabric(10000, full=True)
        dbs = topo.lsdb.dbs.copy()
        dbs["node_label"] = 1 + np.arange(len(dbs), dtype=np.int32)
        self.lsdb = PackedLsdb(topo.lsdb.blob, dbs, topo.lsdb.adjs)
        self.desc = ("fabric_full numOfSws=10000; me = rack switch 3-0-0, LFA on; a v6 loopback "
                     "and a node label per node; per step one publication toggling rack switch "
                     "3-1-0's overload bit, then SpfSolver.buildRouteDb(me)")
        self.ls = LinkState(device=dev.index)
        self.ls.updateAdjacencyDatabases(self.lsdb)
        self.me = "3-0-0"
        names = self.ls.flatten()[0]
        self.n, self.e = len(names), len(self.ls.flatten()[2])
        self.ps = PrefixState()
        for i, nm in enumerate(names):
            self.ps.updatePrefix(nm, self.ls.getArea(), PrefixEntry(f"fd00:{i // 65536:x}:{i % 65536:x}::/64"))
        dbs = {d.thisNodeName: d for d in unpack(self.lsdb)}
        self.victim = dbs["3-1-0"]
        self.units = 1
        self.world = world
        self.kernel_bytes = {"route_build": 1}
        self.survey_bytes = 0
        self.parallelism = "one LinkState per process (replicas)"
        self.pub, self.build, self.routes = [], [], 0
        # Decision's one SpfSolver (C++, include/openr_decision.h): its route
        # DB is built and left native, as a C++ Decision consumes it
        from openr_amd.spf_solver import SpfSolver

        self.solver = SpfSolver(self.me, True, True)

    def step(self) -> None:
        t0 = time.perf_counter()
        self.victim.isOverloaded = not self.victim.isOverloaded
        self.ls.updateAdjacencyDatabase(self.victim)
        self._patch()
        t1 = time.perf_counter()
        ndb = self.solver.buildRouteDbNative(self.me, {self.ls.getArea(): self.ls}, self.ps)
        t2 = time.perf_counter()
        self.routes = ndb.unicastCount() + ndb.mplsCount()
        self.nexthops = ndb.nexthopCount()
        ndb.close()
        self.pub.append(t1 - t0)
        self.build.append(t2 - t1)

    def _patch(self) -> None:
        """The CSR update of the publication (ls_flatten: rows patched in
        place, or the graph reloaded), which the first query would otherwise
        run inside the route build -- timed with the publication."""
        import ctypes as C

        from openr_amd import _native as N

        n, e = C.c_uint32(), C.c_uint32()
        N.raise_for(N.lib.ls_flatten(self.ls._h, C.byref(n), C.byref(e)), "ls_flatten")

    def verify(self):
        """The native route DB of the current state against the Python
        restatement of Decision.cpp's route computation (SpfSolver.native =
        False), route by route: prefixes, next-hop sets, best entries."""
        from openr_amd.spf_solver import SpfSolver

        areas = {self.ls.getArea(): self.ls}
        t0 = time.perf_counter()
        ndb = self.solver.buildRouteDbNative(self.me, areas, self.ps)
        nat = ndb.routeDb()
        ndb.close()
        t1 = time.perf_counter()
        old = SpfSolver.native
        SpfSolver.native = False
        try:
            py = SpfSolver(self.me, True, True).buildRouteDb(self.me, areas, self.ps)
        finally:
            SpfSolver.native = old
        t2 = time.perf_counter()
        bad = sum(1 for p, r in py.unicastRoutes.items()
                  if p not in nat.unicastRoutes or set(nat.unicastRoutes[p].nexthops) != set(r.nexthops)
                  or nat.unicastRoutes[p].bestPrefixEntry is not r.bestPrefixEntry)
        bad += len(set(nat.unicastRoutes) ^ set(py.unicastRoutes))
        bad += sum(1 for l, r in py.mplsRoutes.items()
                   if l not in nat.mplsRoutes or set(nat.mplsRoutes[l].nexthops) != set(r.nexthops))
        bad += len(set(nat.mplsRoutes) ^ set(py.mplsRoutes))
        self.verify_ms = {"native build + materialise into Python objects": 1e3 * (t1 - t0),
                          "python restatement build": 1e3 * (t2 - t1)}
        return {"checked": "every route of the native DB vs the Python restatement "
                           "(openr_amd/spf_solver.py, native=False)",
                "routes": len(py.unicastRoutes) + len(py.mplsRoutes), "mismatches": bad}

    def _solver_ns(self):
        import ctypes as C

        from openr_amd import _native as N

        out = (C.c_uint64 * 6)()
        nat = self.solver._native_solver(self.me)
        N.lib.dc_debug_phase_ns(nat._h, out)
        return list(out)

    def enable_timing(self, k: int) -> None:
        self.pub, self.build = [], []
        self.ph0 = self.ls.debugPhaseNs()
        self.sv0 = self._solver_ns()

    def kernel_ms(self):
        ph = [(b - a) / 1e6 / max(1, len(self.build)) for a, b in zip(self.ph0, self.ls.debugPhaseNs())]
        self.phase_ms = {"publication (updateAdjacencyDatabase + CSR patch, ls_flatten)": 1e3 * float(np.mean(self.pub)),
                         "buildRouteDb (C++ SpfSolver: selection kernel + route assembly)":
                             1e3 * float(np.mean(self.build)),
                         "of which getSpfResult(me) facade phases (plan, execute+copy, pathLinks, "
                         "host)": ph,
                         "of which C++ SpfSolver phases (setup + getSpfResult(me), prefix walk, "
                         "label sets, batched selection, route assembly, adjacency/static)":
                             [(b - a) / 1e6 / max(1, len(self.build))
                              for a, b in zip(self.sv0, self._solver_ns())],
                         "routes_per_build": self.routes,
                         "nexthop_records_per_build": self.nexthops}
        return {"route_build": 1e3 * (float(np.mean(self.pub)) + float(np.mean(self.build)))}

    def edges_per_unit(self) -> int:
        return self.e

    def cpu_baseline(self, budget_s: float):
        """The oracle's route selection for me towards every loopback with LFA
        (its SPFs from me and each neighbour included), after the same
        publication; the host route assembly (labels, MPLS routes) is not in
        it, so this favours the CPU."""
        sys.path.insert(0, str(ROOT / "tests"))
        from oracle import NameTable, route_digests  # CPU baseline only

        names = self.ls.flatten()[0]
        set_ptr = np.arange(self.n + 1, dtype=np.uint32)
        set_nodes = np.arange(self.n, dtype=np.uint32)
        me = np.array([list(names).index(self.me)], dtype=np.int64)
        orc = oracle()()
        orc.update_packed(self.lsdb)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s or done == 0:
            route_digests(orc, NameTable(names), me, set_ptr, set_nodes, True)
            done += 1
        dt = time.perf_counter() - t0
        return {"value": done / dt, "unit": "route_builds/s", "cores": host_cores(), "kind": "port",
                "sample": f"{done} route selections of {self.me} towards all {self.n} loopbacks with "
                          f"LFA (SPF from {self.me} and its neighbours included; no host route "
                          f"assembly), {dt:.1f} s on {host_cores()} cores of {cpu_model()} "
                          f"(oracle/spf_oracle.cpp)"}


class FacadeFlapRouteBuild(FacadeRouteBuild):
    """CS-1 with a link flap (Overview.md:26, "local failures in under
    100ms"): per step rack switch 3-1-0 publishes its adjacency database
    with one uplink withdrawn, and on the next step with it advertised again
    -- the link leaves linksFromNode and comes back (LinkState.cpp:564-719) --
    then SpfSolver.buildRouteDb(me) with LFA.  The publication patches the
    engine's CSR rows in place (dead slots, spf_graph_patch_rows): the line
    reports the graph reloads (0) and row patches of the timed steps."""

    def __init__(self, name: str, rank: int, world: int, dev, eng_cls, graph_from_lsdb):
        super().__init__(name, rank, world, dev, eng_cls, graph_from_lsdb)
        self.desc = ("fabric_full numOfSws=10000; me = rack switch 3-0-0, LFA on; a v6 loopback "
                     "and a node label per node; per step one publication of rack switch 3-1-0 "
                     "withdrawing (odd steps: re-advertising) its first uplink, then "
                     "SpfSolver.buildRouteDb(me)")
        self.held = None

    def step(self) -> None:
        import copy

        t0 = time.perf_counter()
        if self.held is None:
            self.held = self.victim.adjacencies.pop(0)
        else:
            self.victim.adjacencies.insert(0, self.held)
            self.held = None
        self.ls.updateAdjacencyDatabase(copy.copy(self.victim))
        self._patch()
        t1 = time.perf_counter()
        ndb = self.solver.buildRouteDbNative(self.me, {self.ls.getArea(): self.ls}, self.ps)
        t2 = time.perf_counter()
        self.routes = ndb.unicastCount() + ndb.mplsCount()
        self.nexthops = ndb.nexthopCount()
        ndb.close()
        self.pub.append(t1 - t0)
        self.build.append(t2 - t1)

    def enable_timing(self, k: int) -> None:
        from openr_amd import _native as N
        from openr_amd.engine import SpfEngine

        super().enable_timing(k)
        self.loads0 = SpfEngine(handle=self.ls.engine_handle()).loads
        self.patches0 = int(N.lib.ls_debug_row_patches(self.ls._h))

    def kernel_ms(self):
        from openr_amd import _native as N
        from openr_amd.engine import SpfEngine

        out = super().kernel_ms()
        self.phase_ms["graph_reloads_in_timed_steps"] = int(
            SpfEngine(handle=self.ls.engine_handle()).loads - self.loads0)
        self.phase_ms["row_patches_in_timed_steps"] = int(N.lib.ls_debug_row_patches(self.ls._h)) - self.patches0
        return out


def host_cores() -> int:
    sys.path.insert(0, str(ROOT / "tests"))
    from oracle import host_threads

    return host_threads()


WORKLOADS = {"fabric_full": AllSources, "fabric_ref": AllSources, "grid100": AllSources,
             "fabric_rtt": AllSources,
             "wan_ksp2": Ksp2AllPairs, "ba_whatif": WhatIfAllLinks, "fabric_lfa": FacadeLfa,
             "fabric_routes": RoutesAllNodes, "fabric_route_dbs": RouteDbsAllNodes,
             "fabric_lfa_routes": FacadeRouteBuild,
             "fabric_flap_routes": FacadeFlapRouteBuild}


def _pmc_kernels(workload: str, kernels):
    """Per-kernel PMC records of the kernels whose names start with one of
    `kernels` in the committed profiles/pmc_<workload>.json
    (tools/pmc_summary.py): ([(name, record)], provenance) or ([], reason)."""
    pmc = ROOT / "profiles" / f"pmc_{workload}.json"
    if not pmc.exists():
        return [], f"{pmc.relative_to(ROOT)} not found"
    try:
        pj = json.loads(pmc.read_text())
    except Exception as e:  # noqa: BLE001
        return [], f"{pmc.relative_to(ROOT)}: {e!r}"
    hits = []
    for kname, kv in pj.get("per_kernel", {}).items():
        # (the staged-graph KSP2 kernel is ksp2_lds_kernel)
        if any(kname.startswith(k) or kname.replace("_lds", "").startswith(k) for k in kernels):
            hits.append((kname, kv))
    if not hits:
        return [], f"{pmc.relative_to(ROOT)} has no {'/'.join(kernels)}"
    return hits, (f"{pmc.relative_to(ROOT)} ({pj.get('source', 'rocprofv3 --pmc')}; kernels "
                  f"{', '.join(h[0] for h in hits)}; FETCH_SIZE x2 + WRITE_SIZE per dispatch)")


def roofline_block(wl, kms, launch_ms: float, workload: str, rank: int):
    """Roofline of the dominant kernel (largest HIP-event time of one execute).

    frac (= frac_algorithmic): the algorithmic bytes of that kernel -- the
    outputs the path must write plus one read of the graph
    (wl.alg_bytes) -- over its time, over 8 TB/s.  frac_measured: the same
    kernel's HBM bytes from the committed PMC run (FETCH_SIZE x 2 +
    WRITE_SIZE, MI355X_MICROARCH.md's gfx950 corrections) over the same
    time.  l2_frac: the bytes the kernel's structure moves through L2 (per
    workgroup graph sweeps, internal u8 / bit-plane rows: wl.kernel_bytes,
    spf_plan_traffic) over the time -- what round 2 reported as frac.
    limiter: what the PMC says bounds the kernel."""
    alg = getattr(wl, "alg_bytes", None)
    if not alg:
        return None
    dominant = max(kms, key=kms.get)
    t = kms[dominant] * 1e-3
    achieved = alg[dominant] / t / 1e9
    hits, src = _pmc_kernels(workload, getattr(wl, "pmc_kernels", {}).get(dominant, [dominant]))
    traffic = sum(kv["fetch_bytes_x2"] + kv["write_bytes"] for _, kv in hits) if hits else None
    limiter = None
    if hits:  # the phase's busiest kernel (most wave cycles) names the limiter
        kv = max(hits, key=lambda h: h[1].get("counters_per_dispatch", {}).get("SQ_WAVE_CYCLES", 0))[1]
        cs = kv.get("counters_per_dispatch", {})
        wc = cs.get("SQ_WAVE_CYCLES") or 0
        wait = kv.get("sq_wait_any_per_wave_cycle")
        valu = kv.get("sq_active_inst_valu_per_wave_cycle")
        anyi = kv.get("sq_active_inst_any_per_wave_cycle")
        lds = cs.get("SQ_INSTS_LDS", 0) / wc if wc else None
        hbm_frac = traffic / t / 1e9 / HBM_PEAK_GBS
        kind = ("hbm" if hbm_frac >= 0.6 else
                "latency (waves waiting on memory / LDS)" if (wait or 0) >= 0.45 else
                "issue (instruction-bound)" if (anyi or 0) >= 0.45 else "mixed")
        limiter = {"kind": kind, "sq_wait_any_per_wave_cycle": wait,
                   "sq_active_inst_valu_per_wave_cycle": valu,
                   "sq_active_inst_any_per_wave_cycle": anyi,
                   "sq_insts_lds_per_wave_cycle": lds,
                   "l2_hit_rate": kv.get("l2_hit_rate"), "source": src}
    elif rank == 0:
        print(f"bench: {src}: roofline.traffic is null", file=sys.stderr)
    kb = wl.kernel_bytes
    practical = None
    eng = getattr(wl, "eng", None)
    if eng is not None and os.environ.get("BENCH_NO_COPY_BW") is None:
        try:  # the measured copy ceiling beside the spec peak
            practical = eng.copy_bandwidth(1 << 30, 10)
        except Exception as e:  # noqa: BLE001
            print(f"bench: copy bandwidth: {e!r}", file=sys.stderr)
    out = {
        "bound": "hbm",
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "practical_peak": practical,
        "practical_peak_source": "spf_debug_copy_bandwidth: 1 GiB 16-byte copy kernel on this GPU, "
                                 "read + written bytes / time (HIP events)" if practical else None,
        "frac_of_practical": achieved / practical if practical else None,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "frac_algorithmic": achieved / HBM_PEAK_GBS,
        "frac_measured": None if traffic is None else traffic / t / 1e9 / HBM_PEAK_GBS,
        "traffic": traffic,
        "traffic_source": src if traffic is not None else None,
        "kernel": dominant,
        "kernel_ms": kms,
        "algorithmic_bytes": alg,
        "algorithmic_bytes_note": getattr(wl, "alg_note", "outputs + one graph read per kernel"),
        "l2_frac": kb[dominant] / t / 1e9 / HBM_PEAK_GBS,
        "l2_bytes": kb,
        "limiter": limiter,
        # the whole execute: algorithmic bytes over the summed kernel time
        "execute_frac_algorithmic": getattr(wl, "alg_execute_bytes", sum(alg.values()))
        / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
        # SURVEY.md §8(d)'s per-solve figure (a full CSR sweep charged to every
        # solve) over the algorithmic bytes: how much sweep work batching shares
        "survey_bytes_per_launch": wl.survey_bytes,
        "reuse_factor": wl.survey_bytes / max(1, sum(alg.values())),
    }
    return out


def _dump_maps_at_exit(path: str) -> None:
    """Diagnostics: copy /proc/self/maps when the interpreter finalises, so
    addresses in a native crash during exit-time teardown can be attributed
    to a library (BENCH_DUMP_MAPS=<file>)."""
    import atexit
    import shutil

    atexit.register(lambda: shutil.copy("/proc/self/maps", path))


def main() -> None:
    if os.environ.get("BENCH_DUMP_MAPS"):
        _dump_maps_at_exit(os.environ["BENCH_DUMP_MAPS"])
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="fabric_full", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-budget", type=float, default=12.0,
                    help="seconds of CPU-baseline sampling (0 disables)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="all-sources workloads: split one LSDB's sources over ranks "
                         "(strong), or one LSDB snapshot per rank (weak)")
    ap.add_argument("--results", default="resident", choices=["resident", "gather"],
                    help="strong all-sources: results stay in each rank's HBM, digests "
                         "checked after the run (resident), or every rank's rows and "
                         "bitmaps gathered to rank 0 inside the step (gather)")
    ap.add_argument("--devices", default=None,
                    help="single-process multi-device run (spf_mctx): comma-separated device "
                         "ids, repeats allowed (0,0,0,0 emulates 4 GPUs on one); default with "
                         "--gpus N > 1 and no torchrun: 0..N-1")
    ap.add_argument("--graphs", action="store_true",
                    help="multi-device run: replay each member's execute as a hipGraph")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and (args.devices or args.gpus > 1):
        return main_multi(args)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        dist.init_process_group("nccl")
    dev = Dev(local, world)

    from openr_amd.engine import SpfEngine, graph_from_lsdb

    cls = WORKLOADS[args.workload]
    if rank == 0:  # progress on stderr: building a 250k-node graph takes a while
        print(f"bench: building {args.workload} (world {world})", file=sys.stderr, flush=True)
    if cls is AllSources:
        wl = cls(args.workload, rank, world, dev, SpfEngine, graph_from_lsdb, scaling=args.scaling,
                 results=args.results)
    else:
        wl = cls(args.workload, rank, world, dev, SpfEngine, graph_from_lsdb)
    if rank == 0:
        print(f"bench: {args.workload} built; {args.warmup} warmup + {args.steps} timed steps",
              file=sys.stderr, flush=True)
    for _ in range(args.warmup):
        wl.step()
    getattr(wl, "finish", lambda: None)()
    dev.sync()
    # kernel timing: HIP events on the execute stream inside the timed steps
    # (the roofline's per-kernel times).  A multi-GPU all-sources rank takes
    # ~0.07 ms per step, where 4 events per execute would add ~10 us: there
    # the events time separate executes after the timed region instead.
    events_in_timed = world == 1 or cls is not AllSources
    if events_in_timed:
        wl.enable_timing(max(1, args.steps))

    if world > 1:
        dist.barrier()
    dev.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl.step()
    getattr(wl, "finish", lambda: None)()
    dev.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if not events_in_timed:
        k = max(1, min(args.steps, 10))
        wl.enable_timing(k)
        for _ in range(k):
            wl.step()
        getattr(wl, "finish", lambda: None)()
        dev.sync()
    kms = wl.kernel_ms()
    launch_ms = sum(kms.values())
    parity = wl.verify() if hasattr(wl, "verify") else None
    if hasattr(wl, "eng"):
        wl.eng.check()  # a grid-resident kernel's barrier gave up: the run is invalid

    # whole-job units: weak = every rank did `units`; strong = ranks split them
    units = wl.units
    if world > 1:
        u = torch.tensor([units], dtype=torch.float64, device=dev.device)
        dist.all_reduce(u)
        units = float(u.item())
    value = units * args.steps / elapsed
    gteps = units * wl.edges_per_unit() * args.steps / elapsed / 1e9

    roofline = roofline_block(wl, kms, launch_ms, args.workload, rank)
    if parity and parity.get("mismatches"):
        print(f"bench: PARITY FAILURE: {parity['mismatches']} checked results differ from "
              f"the oracle ({parity})", file=sys.stderr)
    out = {
        "metric": METRIC if isinstance(wl, AllSources) else (
            "all-pairs KSP2 (k=1,2 edge-disjoint paths) pairs/sec, 2k-node WAN"
            if isinstance(wl, Ksp2AllPairs) else
            "LinkState facade: publication + getSpfResult(me and every LFA neighbour) per sec"
            if isinstance(wl, FacadeLfa) else
            "getDecisionRouteDb for every node, route databases materialised in HBM (all-sources SPF "
            "+ next-hop records) per sec, 10k fabric"
            if isinstance(wl, RouteDbsAllNodes) else
            "getDecisionRouteDb for every node (all-sources SPF + route selection) per sec, 10k fabric"
            if isinstance(wl, RoutesAllNodes) else
            "link-flap publication + SpfSolver.buildRouteDb(me) with LFA per sec, 10k fabric"
            if isinstance(wl, FacadeFlapRouteBuild) else
            "publication + SpfSolver.buildRouteDb(me) with LFA per sec, 10k fabric"
            if isinstance(wl, FacadeRouteBuild) else
            "what-if single-link-failure SPF reruns/sec, 1M-link scale-free graph"),
        "value": value,
        "unit": wl.unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": wl.scaling,
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "gteps": gteps,
        "config": {
            "workload": wl.desc,
            "nodes": wl.n,
            "directed_up_edges": wl.e,
            "units_per_step_per_rank": wl.units,
            "parallelism": wl.parallelism,
        },
        "roofline": roofline,
        "cpu_baseline": None,
    }
    if parity is not None:
        out["parity"] = parity
    if getattr(wl, "gather", False):
        out["config"]["gather_bytes_per_step"] = wl.gather_bytes
    if isinstance(wl, AllSources):
        out["config"]["results"] = wl.results
    if isinstance(wl, AllSources):
        out["config"]["next_hop_rows"] = wl.narrow  # u32 | u8 | sliced (bit planes)
    if isinstance(wl, (RoutesAllNodes, FacadeRouteBuild)):
        out["config"]["phase_ms_per_step"] = wl.phase_ms
    if getattr(wl, "verify_ms", None):
        out["config"]["verify_ms"] = wl.verify_ms
    if isinstance(wl, FacadeLfa):
        out["config"]["phase_ms_per_step"] = wl.phase_ms
        out["config"]["batched_prefetch"] = wl.prefetch
    if isinstance(wl, WhatIfAllLinks):
        out["config"]["hot_failures_per_rank"] = wl.n_hot
        out["config"]["workgroup_team_failures_per_rank"] = wl.n_big
    if rank == 0 and world == 1 and args.cpu_budget > 0:
        out["cpu_baseline"] = wl.cpu_baseline(args.cpu_budget)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    from openr_amd.engine import close_all

    close_all()  # plans before contexts, while the HIP runtime is up
    dev.close()
    if world == 1 and os.environ.get("BENCH_DEVICE_RESET"):
        dev.hip.device_reset()
    if parity and parity.get("mismatches"):
        sys.exit(3)  # a result that differs from the oracle is not a measurement


def main_multi(args) -> None:
    """--devices / --gpus N without torchrun: the single-process
    multi-device context (AllSourcesMulti)."""
    if WORKLOADS.get(args.workload) is not AllSources:
        raise SystemExit("the single-process multi-device run covers the all-sources workloads")
    devices = ([int(x) for x in args.devices.split(",")] if args.devices
               else list(range(args.gpus)))
    from openr_amd import hiprt

    hiprt.set_device(devices[0])
    wl = AllSourcesMulti(args.workload, devices, graphs=args.graphs)
    for _ in range(args.warmup):
        wl.step()
    wl.finish()
    wl.enable_timing(max(1, args.steps))
    wl.finish()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl.step()
    wl.finish()
    elapsed = time.perf_counter() - t0
    kms = wl.kernel_ms()
    enq = enqueue_stagger(wl, max(5, args.steps))
    parity = wl.verify()
    distinct = sorted(set(devices))
    value = wl.units * args.steps / elapsed
    slow = max(wl.member_ms)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": wl.unit,
        "n_gpus": len(distinct),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "gteps": wl.units * wl.e * args.steps / elapsed / 1e9,
        "config": {
            "workload": wl.desc, "nodes": wl.n, "directed_up_edges": wl.e,
            "members": len(devices), "devices": devices, "parallelism": wl.parallelism,
            "member_execute_ms": wl.member_ms,
            # members sharing a GPU run one after another: the slowest member
            # is what a step of len(devices) separate GPUs would take
            "projected_step_ms_one_member_per_gpu": slow,
            "projected_value_one_member_per_gpu": wl.units / (slow * 1e-3),
            "hip_graphs": wl.graphs,
            "host_enqueue": enq,
        },
        "roofline": roofline_block(wl, kms, sum(kms.values()), args.workload, 0),
        "cpu_baseline": None,
        "parity": parity,
    }
    print(json.dumps(out), flush=True)
    from openr_amd.engine import close_all

    close_all()
    if parity and parity.get("mismatches"):
        sys.exit(3)


if __name__ == "__main__":
    main()
