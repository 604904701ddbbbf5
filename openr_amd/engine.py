"""Batched all-sources SPF on device buffers (include/openr_spf.h).

This is the path ``SpfSolver`` takes when it needs many sources at once
(all-sources route builds, ``breeze decision routes --nodes all`` =
``Decision::getDecisionRouteDb`` per node, Decision.cpp:1480-1500; LFA's
SPF-from-every-neighbour, Decision.cpp:1158-1192).  One ``SpfPlan`` fixes the
source batch; ``execute`` enqueues the kernels on a HIP stream without host
synchronisation, so it can be timed with HIP events or captured in a graph.
"""

from __future__ import annotations

import ctypes as C
import weakref
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from ._native import NativeHandle, close_all  # noqa: F401



HOP_COUNT = N.SPF_FLAG_HOP_COUNT
DIST64 = N.SPF_FLAG_DIST64
UNREACHABLE = N.SPF_UNREACHABLE
UNREACHABLE64 = N.SPF_UNREACHABLE64


@dataclass
class SolveResult:
    dist: np.ndarray  # [n_src, n_nodes] uint32 (UNREACHABLE), uint64 for dist64 plans
    nh: np.ndarray  # destination bitmaps, one per (source, neighbour)
    nh_off: np.ndarray  # [n_src] uint64 word offset of each source's bitmaps
    words: np.ndarray  # [n_src] number of bitmaps (= distinct up neighbours)
    pitch: int

    def nh_matrix(self, i: int) -> np.ndarray:
        """bool [k_i, n_nodes]: row j = destinations whose next-hop set holds
        the source's j-th neighbour (ascending id)."""
        return nh_matrix(self.nh, int(self.nh_off[i]), int(self.words[i]), self.pitch,
                         self.dist.shape[1])


def nh_matrix(nh: np.ndarray, off: int, k: int, pitch: int, n: int) -> np.ndarray:
    wpm = pitch // 32
    words = nh[off: off + k * wpm].reshape(k, wpm).astype(np.uint32)
    bits = np.unpackbits(words.view(np.uint8).reshape(k, wpm * 4), axis=1, bitorder="little")
    return bits[:, :n].astype(bool)


class SpfPlan(NativeHandle):
    _destroy = "spf_plan_destroy"

    def __init__(self, eng: "SpfEngine", srcs: Sequence[int], flags: int) -> None:
        self._eng = eng
        self.srcs = np.ascontiguousarray(srcs, np.uint32)
        self.flags = flags
        h = C.c_void_p()
        eng._err(N.lib.spf_plan_create(eng._h, N.ptr(self.srcs), len(self.srcs), flags,
                                       C.byref(h)))
        self._adopt(h)
        self.nh_words = int(N.lib.spf_plan_nh_words(h))
        self.closure_rows = int(N.lib.spf_plan_closure_rows(h))
        self.nh_off = np.zeros(len(self.srcs), np.uint64)
        self.words = np.zeros(len(self.srcs), np.uint32)
        N.lib.spf_plan_nh_layout(h, N.ptr(self.nh_off, C.c_uint64), N.ptr(self.words))

    @property
    def n_src(self) -> int:
        return len(self.srcs)

    def execute(self, d_dist: int, d_nh: int, stream: int = 0) -> None:
        """Enqueue on `stream` (raw hipStream_t as int; 0 = engine stream)."""
        self._eng._err(N.lib.spf_plan_execute(self._h, C.c_void_p(d_dist), C.c_void_p(d_nh),
                                              C.c_void_p(stream) if stream else None))

    def copy_narrow_rows(self, d_out: int, stream: int = 0) -> None:
        """Enqueue a copy of the last execute's u8 rows (n_src x pitch bytes,
        254 = saturated, 255 = unreachable) to d_out (spf_plan_copy_narrow_rows)."""
        self._eng._err(N.lib.spf_plan_copy_narrow_rows(self._h, C.c_void_p(d_out),
                                                       C.c_void_p(stream) if stream else None))

    def digest(self, d_dist: int, d_nh: int, d_out: int, stream: int = 0) -> None:
        """Enqueue per-source u64 digests of an execute's output into d_out
        (n_src words, spf_plan_digest)."""
        self._eng._err(N.lib.spf_plan_digest(self._h, C.c_void_p(d_dist), C.c_void_p(d_nh),
                                             C.c_void_p(d_out),
                                             C.c_void_p(stream) if stream else None))

    def execute_host(self) -> "SolveResult":
        """Execute into host arrays (spf_plan_execute_host)."""
        n = self._eng.n_nodes
        dist = np.zeros((self.n_src, n), np.uint64 if self.flags & DIST64 else np.uint32)
        nh = np.zeros(max(1, self.nh_words), np.uint32)
        self._eng._err(N.lib.spf_plan_execute_host(self._h, N.ptr(dist), N.ptr(nh)))
        return SolveResult(dist, nh, self.nh_off, self.words, self._eng.pitch)

    BFS_KERNELS = ("sssp_kernel", "msbfs_kernel", "msbfs_planes_kernel", "exact_spf_kernel",
                   "spf_big_kernel", "mssp_kernel", "msbfs_team_kernel")
    ROW_MODES = ("u32", "u8", "sliced", "sliced_bfs")

    def kernels(self) -> Tuple[str, bool]:
        """(distance kernel name, next-hop pass reads u8 narrow rows or their
        bit-sliced form) of the next execute (spf_plan_kernels)."""
        bfs, narrow = self._kernel_codes()
        return self.BFS_KERNELS[bfs], bool(narrow)

    def _kernel_codes(self) -> Tuple[int, int]:
        bfs, narrow = C.c_uint32(), C.c_uint32()
        self._eng._err(N.lib.spf_plan_kernels(self._h, C.byref(bfs), C.byref(narrow)))
        return bfs.value, narrow.value

    def row_mode(self) -> str:
        """Rows the next-hop pass reads: "u32", "u8", "sliced" (bit planes from
        the u8 rows) or "sliced_bfs" (bit planes written by the team BFS)."""
        return self.ROW_MODES[self._kernel_codes()[1]]

    def phase_kernels(self) -> Tuple[str, Optional[str], Optional[str]]:
        """Kernel names of the execute's three timed phases (distance kernel,
        row slicing, next-hop pass); None where a phase launches nothing."""
        bfs, narrow = self._kernel_codes()
        name = self.BFS_KERNELS[bfs]
        if bfs in (3, 4) or not self.nh_words:  # exact / big kernels: next hops inside
            return name, None, None
        if narrow == 2:
            return name, "slice_rows_kernel", "ecmp_sliced_kernel"
        if narrow == 3:
            return name, None, "ecmp_sliced_kernel"
        return name, None, "ecmp_kernel"

    def traffic(self) -> Tuple[int, int]:
        """Compulsory HBM bytes of (distance kernel, next-hop pass incl. row
        slicing) per execute (spf_plan_traffic)."""
        a, b = C.c_uint64(), C.c_uint64()
        self._eng._err(N.lib.spf_plan_traffic(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def traffic_phases(self) -> Tuple[int, int, int]:
        """Compulsory bytes per phase (distance kernel, slicing, next hops)."""
        b = (C.c_uint64 * 3)()
        self._eng._err(N.lib.spf_plan_traffic_phases(self._h, b))
        return b[0], b[1], b[2]

    def enable_timing(self, max_executes: int) -> None:
        self._eng._err(N.lib.spf_plan_enable_timing(self._h, max_executes))

    def timing(self) -> Tuple[float, float, int]:
        """(summed SSSP ms, summed ECMP ms, executes) since enable/last call."""
        a, b, n = C.c_double(), C.c_double(), C.c_uint32()
        self._eng._err(N.lib.spf_plan_timing(self._h, C.byref(a), C.byref(b), C.byref(n)))
        return a.value, b.value, n.value

    def timing_phases(self) -> Tuple[Tuple[float, float, float], int]:
        """((distance, slicing, next-hop) summed ms, executes) since
        enable/last call (spf_plan_timing_phases)."""
        ms, n = (C.c_double * 3)(), C.c_uint32()
        self._eng._err(N.lib.spf_plan_timing_phases(self._h, ms, C.byref(n)))
        return (ms[0], ms[1], ms[2]), n.value

    def execute_torch(self, dist, nh, stream=None) -> None:
        """dist: int32/uint32 tensor [n_src, pitch] on the engine's device;
        nh: tensor with >= nh_words 32-bit words; stream: torch.cuda.Stream."""
        import torch

        assert dist.is_cuda and dist.numel() >= self.n_src * self._eng.pitch
        assert nh.is_cuda and nh.numel() >= max(1, self.nh_words)
        s = (stream or torch.cuda.current_stream(dist.device)).cuda_stream
        self.execute(dist.data_ptr(), nh.data_ptr(), s)


KSP2_NONE = N.SPF_KSP2_NONE
PAIR_DTYPE = np.dtype([("first", "<u4", (2,)), ("n_paths", "<u4", (2,))])  # spf_ksp2_pair


@dataclass
class Ksp2Result:
    """All-destinations KSP2 of a source batch (include/openr_spf.h)."""

    srcs: np.ndarray  # [n_src]
    n_nodes: int
    pairs: np.ndarray  # [n_src * n_nodes] PAIR_DTYPE
    pool: np.ndarray  # u32 path records [n_links, next, links...]

    def paths(self, i: int, d: int, k: int) -> List[List[int]]:
        """getKthPaths(srcs[i], d, k) for k in (1, 2): lists of link ids."""
        rec = self.pairs[i * self.n_nodes + d]
        out: List[List[int]] = []
        at = int(rec["first"][k - 1])
        for _ in range(int(rec["n_paths"][k - 1])):
            n = int(self.pool[at])
            out.append([int(x) for x in self.pool[at + 2: at + 2 + n]])
            at = int(self.pool[at + 1])
        return out


class Ksp2Plan(NativeHandle):
    """A fixed source batch for batched KSP2 (``spf_ksp2_plan``)."""

    _destroy = "spf_ksp2_plan_destroy"

    def __init__(self, eng: "SpfEngine", srcs: Sequence[int]) -> None:
        self._eng = eng
        self.srcs = np.ascontiguousarray(srcs, np.uint32)
        h = C.c_void_p()
        eng._err(N.lib.spf_ksp2_plan_create(eng._h, N.ptr(self.srcs), len(self.srcs), C.byref(h)))
        self._adopt(h)

    def execute(self, d_pairs: int, d_pool: int, pool_words: int, d_counters: int,
                stream: int = 0) -> None:
        self._eng._err(N.lib.spf_ksp2_execute(self._h, C.c_void_p(d_pairs), C.c_void_p(d_pool),
                                              pool_words, C.c_void_p(d_counters),
                                              C.c_void_p(stream) if stream else None))

    def digest(self, d_pairs: int, d_pool: int, d_link_hash: int, d_out: int,
               stream: int = 0) -> None:
        """Enqueue per-source u64 digests of an execute's pairs and pool into
        d_out (spf_ksp2_digest; d_link_hash: u64 value hash per link id)."""
        self._eng._err(N.lib.spf_ksp2_digest(self._h, C.c_void_p(d_pairs), C.c_void_p(d_pool),
                                             C.c_void_p(d_link_hash), C.c_void_p(d_out),
                                             C.c_void_p(stream) if stream else None))

    def chunk(self) -> int:
        """Sources per KSP2 workgroup (spf_ksp2_plan_chunk)."""
        return int(N.lib.spf_ksp2_plan_chunk(self._h))

    def enable_timing(self, max_executes: int) -> None:
        self._eng._err(N.lib.spf_ksp2_enable_timing(self._h, max_executes))

    def timing(self) -> Tuple[float, float, int]:
        a, b, n = C.c_double(), C.c_double(), C.c_uint32()
        self._eng._err(N.lib.spf_ksp2_timing(self._h, C.byref(a), C.byref(b), C.byref(n)))
        return a.value, b.value, n.value


DIGEST_DTYPE = np.dtype([("n_dist_changed", "<u4"), ("n_nh_changed", "<u4"),
                         ("hash", "<u8")])  # spf_whatif_digest


class WhatIfPlan(NativeHandle):
    """One source, a list of single-link failures (``spf_whatif_plan``)."""

    _destroy = "spf_whatif_plan_destroy"

    def __init__(self, eng: "SpfEngine", src: int, links: Optional[Sequence[int]]) -> None:
        self._eng = eng
        h = C.c_void_p()
        arr = None if links is None else np.ascontiguousarray(links, np.uint32)
        eng._err(N.lib.spf_whatif_plan_create(eng._h, src, None if arr is None else N.ptr(arr),
                                              0 if arr is None else len(arr), C.byref(h)))
        self._adopt(h)
        self.n_fail = int(N.lib.spf_whatif_plan_failures(h))
        self.links = np.zeros(max(1, self.n_fail), np.uint32)
        eng._err(N.lib.spf_whatif_plan_links(h, N.ptr(self.links)))
        self.links = self.links[: self.n_fail]

    def execute(self, d_out: int, d_base: int = 0, stream: int = 0) -> None:
        self._eng._err(N.lib.spf_whatif_execute(self._h, C.c_void_p(d_out),
                                                C.c_void_p(d_base) if d_base else None,
                                                C.c_void_p(stream) if stream else None))

    def stats(self) -> Tuple[int, int]:
        a, b = C.c_uint32(), C.c_uint32()
        self._eng._err(N.lib.spf_whatif_stats(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def enable_timing(self, max_executes: int) -> None:
        self._eng._err(N.lib.spf_whatif_enable_timing(self._h, max_executes))

    def timing(self) -> Tuple[float, float, int]:
        a, b, n = C.c_double(), C.c_double(), C.c_uint32()
        self._eng._err(N.lib.spf_whatif_timing(self._h, C.byref(a), C.byref(b), C.byref(n)))
        return a.value, b.value, n.value


class SpfEngine(NativeHandle):
    """An engine context with one graph loaded (``spf_ctx``).  ``close()``
    (or ``with SpfEngine(0) as eng:``) first closes the plans created on it,
    then destroys the context (its streams, events and device buffers)."""

    _LEVEL = 1
    _destroy = "spf_ctx_destroy"

    def __init__(self, device: int = 0, handle: Optional[C.c_void_p] = None) -> None:
        self._owned = handle is None
        self._plans: "weakref.WeakSet[NativeHandle]" = weakref.WeakSet()
        if handle is None:
            h = C.c_void_p()
            st = N.lib.spf_ctx_create(device, C.byref(h))
            N.raise_for(st, N.global_error())
            self._adopt(h)
        else:
            self._h = handle
        self._graph = None

    def close(self) -> None:
        for p in list(getattr(self, "_plans", ())):
            p.close()
        super().close()

    def _track(self, plan):
        self._plans.add(plan)
        return plan

    def _err(self, st: int) -> None:
        N.raise_for(st, (N.lib.spf_last_error(self._h) or b"").decode())

    # ---- graph -----------------------------------------------------------------
    def load(self, row_ptr, col, metric, link_id, overloaded) -> None:
        arrs = (np.ascontiguousarray(row_ptr, np.uint32), np.ascontiguousarray(col, np.uint32),
                np.ascontiguousarray(metric, np.int32), np.ascontiguousarray(link_id, np.uint32),
                np.ascontiguousarray(overloaded, np.uint8))
        g = N.SpfGraph()
        g.n_nodes = len(arrs[0]) - 1
        g.n_edges = len(arrs[1])
        g.row_ptr = N.ptr(arrs[0])
        g.col = N.ptr(arrs[1])
        g.metric = N.ptr(arrs[2], C.c_int32)
        g.link_id = N.ptr(arrs[3])
        g.overloaded = N.ptr(arrs[4], C.c_uint8)
        self._err(N.lib.spf_graph_load(self._h, C.byref(g)))
        self._graph = arrs

    def set_overload(self, nodes, overloaded) -> None:
        """Drain / undrain nodes in place (spf_graph_set_overload): SPF plans
        re-derive on their next execute, KSP2 / what-if plans must be recreated."""
        nodes = np.ascontiguousarray(nodes, np.uint32)
        vals = np.ascontiguousarray(overloaded, np.uint8)
        if len(nodes) != len(vals):
            raise ValueError("nodes / overloaded length mismatch")
        self._err(N.lib.spf_graph_set_overload(self._h, N.ptr(nodes), N.ptr(vals, C.c_uint8),
                                               len(nodes)))
        if self._graph is not None:
            self._graph[4][nodes] = vals

    def set_metric(self, edges, metric) -> None:
        """New metrics of directed CSR edges in place (spf_graph_set_metric)."""
        edges = np.ascontiguousarray(edges, np.uint32)
        mets = np.ascontiguousarray(metric, np.int32)
        if len(edges) != len(mets):
            raise ValueError("edges / metric length mismatch")
        self._err(N.lib.spf_graph_set_metric(self._h, N.ptr(edges), N.ptr(mets, C.c_int32),
                                             len(edges)))
        if self._graph is not None:
            self._graph[2][edges] = mets

    @property
    def epoch(self) -> int:
        """Graph version: bumped by every load and in-place patch."""
        return int(N.lib.spf_graph_epoch(self._h))

    @property
    def loads(self) -> int:
        """spf_graph_load calls so far (in-place patches do not count)."""
        return int(N.lib.spf_graph_loads(self._h))

    @property
    def pitch(self) -> int:
        return int(N.lib.spf_row_pitch(self._h))

    @property
    def n_nodes(self) -> int:
        return len(self._graph[0]) - 1 if self._graph is not None else 0

    def neighbors(self, src: int) -> np.ndarray:
        cnt = C.c_uint32()
        self._err(N.lib.spf_src_neighbors(self._h, src, None, 0, C.byref(cnt)))
        out = np.zeros(max(1, cnt.value), np.uint32)
        self._err(N.lib.spf_src_neighbors(self._h, src, N.ptr(out), cnt.value, C.byref(cnt)))
        return out[: cnt.value]

    def debug_stamps(self) -> np.ndarray:
        """BFS phase clocks of workgroup 0 (needs SPF_STAMPS=1 at first execute):
        [16 waves, 64] -- column 0 is the count, columns 1.. the clocks."""
        return self._stamp_words()[: 64 * 16].reshape(16, 64)

    def _stamp_words(self) -> np.ndarray:
        out = np.zeros(64 * 16 + 1 + 2 * 1024, np.uint64)
        n = C.c_uint32()
        self._err(N.lib.spf_debug_stamps(self._h, N.ptr(out, C.c_uint64), out.size, C.byref(n)))
        return out

    def debug_timeline(self) -> np.ndarray:
        """Team BFS block timeline (SPF_STAMPS set): [block, (start, end)]
        s_memrealtime ticks (100 MHz), zeros for blocks that did not run."""
        return self._stamp_words()[64 * 16 + 1:].reshape(1024, 2)

    def solves(self) -> int:
        return int(N.lib.spf_solves(self._h))

    def copy_bandwidth(self, nbytes: int = 1 << 30, reps: int = 10) -> float:
        """Measured practical HBM ceiling in GB/s (spf_debug_copy_bandwidth)."""
        g = C.c_double()
        self._err(N.lib.spf_debug_copy_bandwidth(self._h, nbytes, reps, C.byref(g)))
        return g.value

    def check(self) -> None:
        """Wait for the device and raise if a grid-resident kernel's barrier
        gave up waiting since the last check (spf_device_check): the outputs
        of those launches are invalid."""
        self._err(N.lib.spf_device_check(self._h))

    # ---- solves -----------------------------------------------------------------
    @property
    def needs_dist64(self) -> bool:
        """Weighted solves of this graph need u64 distances (spf_graph_needs_dist64)."""
        return bool(N.lib.spf_graph_needs_dist64(self._h))

    def plan(self, srcs: Sequence[int], hop: bool = False, dist64: bool = False) -> SpfPlan:
        return self._track(SpfPlan(self, srcs, (HOP_COUNT if hop else 0) |
                                   (DIST64 if dist64 else 0)))

    def solve(self, srcs: Sequence[int], hop: bool = False, dist64: bool = False) -> SolveResult:
        """All of `srcs` in one plan, results on the host.  dist64: u64
        distance rows (the exact kernel; needed when needs_dist64)."""
        with self.plan(srcs, hop, dist64) as p:
            return p.execute_host()

    def solve_exact(self, src: int, hop: bool = False,
                    ignore_links: Optional[Sequence[int]] = None):
        """runSpf on the exact kernel (spf_solve_exact): (dist u64 [N],
        next-hop bitmaps [k, N] bool, pop rank [N] u32)."""
        ign = np.ascontiguousarray(ignore_links if ignore_links is not None else [], np.uint32)
        n = self.n_nodes
        k = len(self.neighbors(src))
        dist = np.zeros(n, np.uint64)
        nh = np.zeros(max(1, k * self.pitch // 32), np.uint32)
        pop = np.zeros(n, np.uint32)
        self._err(N.lib.spf_solve_exact(self._h, src, HOP_COUNT if hop else 0,
                                        N.ptr(ign) if len(ign) else None, len(ign),
                                        N.ptr(dist, C.c_uint64), None, N.ptr(nh), N.ptr(pop)))
        return dist, nh_matrix(nh, 0, k, self.pitch, n), pop

    def ksp2_plan(self, srcs: Sequence[int]) -> Ksp2Plan:
        return self._track(Ksp2Plan(self, srcs))

    def ksp2(self, srcs: Sequence[int]) -> Ksp2Result:
        """getKthPaths(s, d, 1) and (s, d, 2) for every s in srcs, every d."""
        srcs = np.ascontiguousarray(srcs, np.uint32)
        n = self.n_nodes
        pairs = np.zeros(len(srcs) * n, PAIR_DTYPE)
        used = C.c_uint64()
        pool = np.empty(len(pairs) * 12 + (1 << 20), np.uint32)  # lazily backed
        for _ in range(2):
            st = N.lib.spf_ksp2_solve(self._h, N.ptr(srcs), len(srcs),
                                      N.ptr(pairs.view(np.uint32)), N.ptr(pool), pool.size,
                                      C.byref(used))
            if st != N.SPF_E_NOMEM or used.value <= pool.size:
                break
            pool = np.empty(used.value, np.uint32)  # too small: size it exactly, rerun
        self._err(st)
        pool = pool[: used.value]
        return Ksp2Result(srcs, n, pairs, pool)

    def whatif_plan(self, src: int, links: Optional[Sequence[int]] = None) -> WhatIfPlan:
        return self._track(WhatIfPlan(self, src, links))

    def whatif(self, src: int, links: Optional[Sequence[int]] = None):
        """Digests of runSpf(src, true, {l}) for each failed link l (every up
        link when `links` is None): (links, digests[n], base digest)."""
        if links is None:
            links = self.whatif_plan(src).links
        arr = np.ascontiguousarray(links, np.uint32)
        out = np.zeros(max(1, len(arr)), DIGEST_DTYPE)
        base = np.zeros(1, DIGEST_DTYPE)
        self._err(N.lib.spf_whatif_solve(self._h, src, N.ptr(arr), len(arr),
                                         out.ctypes.data, base.ctypes.data))
        return arr, out[: len(arr)], base[0]

    def sssp(self, src: int, hop: bool = False,
             ignore_links: Optional[Sequence[int]] = None) -> np.ndarray:
        ign = np.ascontiguousarray(ignore_links if ignore_links is not None else [], np.uint32)
        out = np.zeros(self.n_nodes, np.uint32)
        self._err(N.lib.spf_sssp(self._h, src, HOP_COUNT if hop else 0,
                                 N.ptr(ign) if len(ign) else None, len(ign), N.ptr(out)))
        return out

    def preds(self, src: int, dist: np.ndarray, hop: bool = False,
              ignore_links: Optional[Sequence[int]] = None) -> Tuple[np.ndarray, np.ndarray]:
        ign = np.ascontiguousarray(ignore_links if ignore_links is not None else [], np.uint32)
        dist = np.ascontiguousarray(dist, np.uint32)
        ptr_ = np.zeros(self.n_nodes + 1, np.uint32)
        cnt = C.c_uint32()
        args = (self._h, src, HOP_COUNT if hop else 0, N.ptr(ign) if len(ign) else None, len(ign),
                N.ptr(dist), N.ptr(ptr_))
        self._err(N.lib.spf_preds(*args, None, 0, C.byref(cnt)))
        edges = np.zeros(max(1, cnt.value), np.uint32)
        self._err(N.lib.spf_preds(*args, N.ptr(edges), cnt.value, C.byref(cnt)))
        return ptr_, edges[: cnt.value]


def partition_sources(nb_ptr, nb_id, srcs, n_parts: int, mode: str = "auto"):
    """Sources to parts (spf_partition_sources, host only): (part of each
    source [n_src] u32, the rule taken: "contiguous" | "locality").
    nb_ptr / nb_id: distinct up neighbours of every node in CSR form."""
    nb_ptr = np.ascontiguousarray(nb_ptr, np.uint32)
    nb_id = np.ascontiguousarray(nb_id if len(nb_id) else [0], np.uint32)
    srcs = np.ascontiguousarray(srcs, np.uint32)
    code = {"auto": N.SPF_PARTITION_AUTO, "contiguous": N.SPF_PARTITION_CONTIGUOUS,
            "locality": N.SPF_PARTITION_LOCALITY}[mode]
    part = np.zeros(max(1, len(srcs)), np.uint32)
    used = C.c_uint32()
    st = N.lib.spf_partition_sources(N.ptr(nb_ptr), N.ptr(nb_id), len(nb_ptr) - 1, N.ptr(srcs),
                                     len(srcs), n_parts, code, N.ptr(part), C.byref(used))
    N.raise_for(st, N.global_error())
    return part[: len(srcs)], N.PARTITION_NAMES[used.value]


class SpfMultiPlan(NativeHandle):
    """A source batch split over the members of an ``SpfMultiEngine``
    (``spf_mplan``): every member's rows and bitmaps stay on its device."""

    _destroy = "spf_mplan_destroy"

    def __init__(self, eng: "SpfMultiEngine", srcs: Sequence[int], flags: int,
                 mode: str = "auto") -> None:
        self._eng = eng
        self.srcs = np.ascontiguousarray(srcs, np.uint32)
        self.flags = flags
        code = {"auto": N.SPF_PARTITION_AUTO, "contiguous": N.SPF_PARTITION_CONTIGUOUS,
                "locality": N.SPF_PARTITION_LOCALITY}[mode]
        h = C.c_void_p()
        eng._err(N.lib.spf_mplan_create(eng._h, N.ptr(self.srcs), len(self.srcs), flags, code,
                                        C.byref(h)))
        self._adopt(h)
        self.partition = N.PARTITION_NAMES[int(N.lib.spf_mplan_partition(h))]
        self.members = eng.size
        self.closure_rows = [int(N.lib.spf_mplan_closure_rows(h, i)) for i in range(self.members)]

    def owner(self, i: int) -> Tuple[int, int]:
        """(member, row) holding request index i."""
        m, r = C.c_uint32(), C.c_uint32()
        self._eng._err(N.lib.spf_mplan_owner(self._h, i, C.byref(m), C.byref(r)))
        return m.value, r.value

    def shard_sizes(self) -> List[int]:
        out = []
        for i in range(self.members):
            n = C.c_uint32()
            self._eng._err(N.lib.spf_mplan_shard(self._h, i, C.byref(n), None, None, None))
            out.append(n.value)
        return out

    def member_kernels(self, i: int) -> Optional[Tuple[str, bool]]:
        """The member's plan kernels (SpfPlan.kernels), None for an idle member."""
        n, plan = C.c_uint32(), C.c_void_p()
        self._eng._err(N.lib.spf_mplan_shard(self._h, i, C.byref(n), C.byref(plan), None, None))
        if not plan.value:
            return None
        bfs, narrow = C.c_uint32(), C.c_uint32()
        N.raise_for(N.lib.spf_plan_kernels(plan, C.byref(bfs), C.byref(narrow)), "spf_plan_kernels")
        return SpfPlan.BFS_KERNELS[bfs.value], bool(narrow.value)

    def set_graphs(self, enable: bool) -> None:
        self._eng._err(N.lib.spf_mplan_set_graphs(self._h, int(bool(enable))))

    def set_enqueue_threads(self, mode: int) -> None:
        """1: each member's execute enqueued from its own host thread, 0: one
        after another from the caller's, -1: threads for distinct devices."""
        self._eng._err(N.lib.spf_mplan_set_enqueue_threads(self._h, int(mode)))

    def enqueue_ns(self) -> Tuple[np.ndarray, bool]:
        """The last execute's host enqueue: per member, ns from the execute's
        start until its launches were enqueued; and whether threads issued them."""
        n = len(self.shard_sizes())
        out = np.zeros(max(1, n), np.uint64)
        thr = C.c_int()
        self._eng._err(N.lib.spf_mplan_enqueue_ns(self._h, N.ptr(out, C.c_uint64), n, C.byref(thr)))
        return out[:n], bool(thr.value)

    def execute(self) -> None:
        self._eng._err(N.lib.spf_mplan_execute(self._h))

    def synchronize(self) -> None:
        self._eng._err(N.lib.spf_mplan_synchronize(self._h))

    def digest(self) -> np.ndarray:
        out = np.zeros(max(1, len(self.srcs)), np.uint64)
        self._eng._err(N.lib.spf_mplan_digest(self._h, N.ptr(out, C.c_uint64)))
        return out[: len(self.srcs)]

    def read(self, i: int) -> Tuple[np.ndarray, np.ndarray]:
        """Request i's (dist [n_nodes], next-hop bitmaps bool [k, n_nodes]) from its owner."""
        n = self._eng.n_nodes
        k = len(self._eng.neighbors(int(self.srcs[i])))
        dist = np.zeros(n, np.uint64 if self.flags & DIST64 else np.uint32)
        nh = np.zeros(max(1, k * self._eng.pitch // 32), np.uint32)
        self._eng._err(N.lib.spf_mplan_read(self._h, i, dist.ctypes.data, N.ptr(nh)))
        return dist, nh_matrix(nh, 0, k, self._eng.pitch, n)

    def preds(self, i: int) -> Tuple[np.ndarray, np.ndarray]:
        n = self._eng.n_nodes
        ptr_ = np.zeros(n + 1, np.uint32)
        cnt = C.c_uint32()
        self._eng._err(N.lib.spf_mplan_preds(self._h, i, N.ptr(ptr_), None, 0, C.byref(cnt)))
        edges = np.zeros(max(1, cnt.value), np.uint32)
        self._eng._err(N.lib.spf_mplan_preds(self._h, i, N.ptr(ptr_), N.ptr(edges), cnt.value,
                                             C.byref(cnt)))
        return ptr_, edges[: cnt.value]

    def enable_timing(self, max_executes: int) -> None:
        self._eng._err(N.lib.spf_mplan_enable_timing(self._h, max_executes))

    def timing(self) -> Tuple[List[float], int]:
        """(per-member summed execute ms, executes) since enable / the last call."""
        ms = (C.c_double * self.members)()
        n = C.c_uint32()
        self._eng._err(N.lib.spf_mplan_timing(self._h, ms, C.byref(n)))
        return [ms[i] for i in range(self.members)], n.value


class SpfMultiEngine(NativeHandle):
    """Several GPUs behind one context (``spf_mctx``): one member engine per
    device id (ids may repeat), the graph replicated to each."""

    _LEVEL = 1
    _destroy = "spf_mctx_destroy"

    def __init__(self, devices: Sequence[int]) -> None:
        ids = (C.c_int * len(devices))(*[int(d) for d in devices])
        h = C.c_void_p()
        st = N.lib.spf_mctx_create(ids, len(devices), C.byref(h))
        N.raise_for(st, N.global_error())
        self._adopt(h)
        self._plans: "weakref.WeakSet[NativeHandle]" = weakref.WeakSet()
        self.devices = list(devices)
        # member 0 answers the graph queries (neighbours, pitch)
        self.member0 = SpfEngine(handle=C.c_void_p(N.lib.spf_mctx_member(h, 0)))

    @property
    def size(self) -> int:
        return int(N.lib.spf_mctx_size(self._h))

    def close(self) -> None:
        for p in list(getattr(self, "_plans", ())):
            p.close()
        super().close()

    def _err(self, st: int) -> None:
        N.raise_for(st, (N.lib.spf_mctx_last_error(self._h) or b"").decode())

    def load(self, row_ptr, col, metric, link_id, overloaded) -> None:
        arrs = (np.ascontiguousarray(row_ptr, np.uint32), np.ascontiguousarray(col, np.uint32),
                np.ascontiguousarray(metric, np.int32), np.ascontiguousarray(link_id, np.uint32),
                np.ascontiguousarray(overloaded, np.uint8))
        g = N.SpfGraph()
        g.n_nodes = len(arrs[0]) - 1
        g.n_edges = len(arrs[1])
        g.row_ptr = N.ptr(arrs[0])
        g.col = N.ptr(arrs[1])
        g.metric = N.ptr(arrs[2], C.c_int32)
        g.link_id = N.ptr(arrs[3])
        g.overloaded = N.ptr(arrs[4], C.c_uint8)
        self._err(N.lib.spf_mctx_graph_load(self._h, C.byref(g)))
        self.member0._graph = arrs

    def set_overload(self, nodes, overloaded) -> None:
        nodes = np.ascontiguousarray(nodes, np.uint32)
        vals = np.ascontiguousarray(overloaded, np.uint8)
        self._err(N.lib.spf_mctx_graph_set_overload(self._h, N.ptr(nodes), N.ptr(vals, C.c_uint8),
                                                    len(nodes)))
        self.member0._graph[4][nodes] = vals

    @property
    def pitch(self) -> int:
        return self.member0.pitch

    @property
    def n_nodes(self) -> int:
        return self.member0.n_nodes

    def neighbors(self, src: int) -> np.ndarray:
        return self.member0.neighbors(src)

    def plan(self, srcs: Sequence[int], hop: bool = False, dist64: bool = False,
             mode: str = "auto") -> SpfMultiPlan:
        p = SpfMultiPlan(self, srcs, (HOP_COUNT if hop else 0) | (DIST64 if dist64 else 0), mode)
        self._plans.add(p)
        return p


def graph_from_lsdb(lsdb, area: str = "0"):
    """Flatten a packed LSDB with the LinkState facade (host side only).
    Returns (node_names, row_ptr, col, metric, link_id, overloaded)."""
    from .link_state import LinkState

    ls = LinkState(area, device=-1)
    ls.updateAdjacencyDatabases(lsdb)
    return ls.flatten()
