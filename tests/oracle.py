"""ctypes binding of the CPU oracle (oracle/liborc_spf.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product (openr_amd/) never does.
"""

from __future__ import annotations

import ctypes as C
import json
import subprocess
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE_DIR = ROOT / "oracle"
LIB = ORACLE_DIR / "liborc_spf.so"


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def _load() -> C.CDLL:
    if not LIB.exists():
        build()
    lib = C.CDLL(str(LIB))
    vp, u8p, u32p, u64p = C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)
    sig = {
        "orc_ls_new": (vp, [C.c_char_p]),
        "orc_ls_free": (None, [vp]),
        "orc_spf_runs": (C.c_uint64, []),
        "orc_ls_update_packed": (C.c_int, [vp, C.c_char_p, vp, C.c_uint32, vp, C.c_uint64,
                                           C.c_uint64, u8p]),
        "orc_ls_delete": (C.c_int, [vp, C.c_char_p, u8p]),
        "orc_ls_decrement_holds": (C.c_int, [vp, u8p]),
        "orc_ls_has_holds": (C.c_int, [vp]),
        "orc_ls_num_links": (C.c_uint64, [vp]),
        "orc_ls_num_nodes": (C.c_uint64, [vp]),
        "orc_ls_is_overloaded": (C.c_int, [vp, C.c_char_p]),
        "orc_ls_metric_a_to_b": (C.c_int, [vp, C.c_char_p, C.c_char_p, C.c_int, u64p]),
        "orc_ls_max_hops": (C.c_uint64, [vp, C.c_char_p]),
        "orc_ls_spf_json": (C.c_char_p, [vp, C.c_char_p, C.c_int]),
        "orc_ls_kth_paths_json": (C.c_char_p, [vp, C.c_char_p, C.c_char_p, C.c_uint64]),
        "orc_ls_links_json": (C.c_char_p, [vp, C.c_char_p]),
        "orc_ls_dense": (C.c_int, [vp, C.c_char_p, u32p, u32p, C.c_uint32, u32p, C.c_uint32,
                                   C.c_int, u64p, u32p, u64p, u32p]),
        "orc_ls_time_sources": (C.c_uint64, [vp, C.POINTER(C.c_char_p), C.c_uint32, C.c_int]),
        "orc_ls_time_ksp2": (C.c_uint64, [vp, C.c_char_p, C.POINTER(C.c_char_p), C.c_uint32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def _p(a, t=C.c_uint32):
    return a.ctypes.data_as(C.POINTER(t))


class OracleLinkState:
    """The restated reference LinkState (oracle/spf_oracle.cpp)."""

    def __init__(self, area: str = "0") -> None:
        self._h = C.c_void_p(lib.orc_ls_new(area.encode()))

    def __del__(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            lib.orc_ls_free(self._h)
            self._h = C.c_void_p()

    def update_packed(self, packed, hold_up: int = 0, hold_down: int = 0) -> List[tuple]:
        n = len(packed.dbs)
        out = np.zeros(3 * max(n, 1), np.uint8)
        lib.orc_ls_update_packed(self._h, packed.blob, packed.dbs.ctypes.data, n,
                                 packed.adjs.ctypes.data if len(packed.adjs) else None,
                                 hold_up, hold_down, _p(out, C.c_uint8))
        return [tuple(bool(x) for x in out[3 * i:3 * i + 3]) for i in range(n)]

    def update(self, dbs, hold_up: int = 0, hold_down: int = 0) -> List[tuple]:
        from openr_amd.lsdb import pack

        return self.update_packed(pack(dbs), hold_up, hold_down)

    def delete(self, node: str) -> tuple:
        out = np.zeros(3, np.uint8)
        lib.orc_ls_delete(self._h, node.encode(), _p(out, C.c_uint8))
        return tuple(bool(x) for x in out)

    def decrement_holds(self) -> tuple:
        out = np.zeros(3, np.uint8)
        lib.orc_ls_decrement_holds(self._h, _p(out, C.c_uint8))
        return tuple(bool(x) for x in out)

    def has_holds(self) -> bool:
        return bool(lib.orc_ls_has_holds(self._h))

    def num_links(self) -> int:
        return int(lib.orc_ls_num_links(self._h))

    def num_nodes(self) -> int:
        return int(lib.orc_ls_num_nodes(self._h))

    def is_overloaded(self, n: str) -> bool:
        return bool(lib.orc_ls_is_overloaded(self._h, n.encode()))

    def spf(self, src: str, use_link_metric: bool = True) -> Dict:
        return json.loads(lib.orc_ls_spf_json(self._h, src.encode(), int(use_link_metric)))

    def kth_paths(self, src: str, dst: str, k: int) -> List[List[List[str]]]:
        return json.loads(lib.orc_ls_kth_paths_json(self._h, src.encode(), dst.encode(), k))

    def links(self, node: str) -> List:
        return json.loads(lib.orc_ls_links_json(self._h, node.encode()))

    def metric_a_to_b(self, a: str, b: str, ulm: bool = True) -> Optional[int]:
        out = C.c_uint64()
        return int(out.value) if lib.orc_ls_metric_a_to_b(
            self._h, a.encode(), b.encode(), int(ulm), C.byref(out)) else None

    def max_hops(self, n: str) -> int:
        return int(lib.orc_ls_max_hops(self._h, n.encode()))

    def dense(self, names: Sequence[str], src_ids: Sequence[int], ulm: bool = True):
        """All-sources rendering in node-id order (names ascending):
        dist [n_src, N] u64 (UINT64_MAX = unreachable) and, per source, a bool
        matrix [k, N] whose row j marks the destinations whose nextHops()
        contain the source's j-th distinct up neighbour (ascending name)."""
        blob = "".join(names).encode()
        lens = np.array([len(s.encode()) for s in names], np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint32)
        srcs = np.asarray(src_ids, np.uint32)
        n, ns = len(names), len(srcs)
        words = np.zeros(ns, np.uint32)
        lib.orc_ls_dense(self._h, blob, _p(offs), _p(lens), n, _p(srcs), ns, int(ulm), None,
                         None, None, _p(words))
        off = np.concatenate([[0], np.cumsum(words.astype(np.uint64) * n)[:-1]]).astype(np.uint64)
        dist = np.zeros((ns, n), np.uint64)
        raw = np.zeros(max(1, int((words.astype(np.uint64) * n).sum())), np.uint32)
        lib.orc_ls_dense(self._h, blob, _p(offs), _p(lens), n, _p(srcs), ns, int(ulm),
                         _p(dist, C.c_uint64), _p(raw), _p(off, C.c_uint64), _p(words))
        mats = []
        for i in range(ns):
            w = int(words[i])
            blk = raw[int(off[i]): int(off[i]) + w * n].reshape(n, w)
            bits = np.unpackbits(blk.astype("<u4").view(np.uint8).reshape(n, 4 * w), axis=1,
                                 bitorder="little").astype(bool)  # [N, 32w]
            mats.append(bits.T.copy())  # [32w, N]; rows >= k are all False
        return dist, mats

    def time_sources(self, srcs: Sequence[str], ulm: bool = True) -> int:
        arr = (C.c_char_p * len(srcs))(*[s.encode() for s in srcs])
        return int(lib.orc_ls_time_sources(self._h, arr, len(srcs), int(ulm)))


    def time_ksp2(self, src: str, dsts: Sequence[str]) -> int:
        arr = (C.c_char_p * len(dsts))(*[s.encode() for s in dsts])
        return int(lib.orc_ls_time_ksp2(self._h, src.encode(), arr, len(dsts)))


def spf_runs() -> int:
    return int(lib.orc_spf_runs())


# ---- what-if digests ----------------------------------------------------------
class OrcDigest(C.Structure):
    _fields_ = [("n_dist_changed", C.c_uint32), ("n_nh_changed", C.c_uint32),
                ("hash", C.c_uint64)]


lib.orc_ls_whatif_digests.restype = C.c_int
lib.orc_ls_whatif_digests.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_uint32),
                                      C.POINTER(C.c_uint32), C.c_uint32, C.c_char_p,
                                      C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.c_uint32,
                                      C.c_int, C.POINTER(OrcDigest), C.POINTER(OrcDigest)]
lib.orc_ls_time_whatif.restype = C.c_uint64
lib.orc_ls_time_whatif.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_char_p),
                                   C.POINTER(C.c_char_p), C.c_uint32, C.c_int]


class NameTable:
    """Node names in id order (ascending), packed for the oracle's C API."""

    def __init__(self, names: Sequence[str]) -> None:
        self.blob = "".join(names).encode()
        self.lens = np.array([len(s.encode()) for s in names], np.uint32)
        self.offs = np.concatenate([[0], np.cumsum(self.lens)[:-1]]).astype(np.uint32)
        self.n = len(names)


def whatif_digests(orc: "OracleLinkState", table: NameTable, src: str,
                   fails: Sequence[tuple], fast: bool = True):
    """Digests (n_dist_changed, n_nh_changed, hash) of the unfailed SPF of
    src and of runSpf(src, true, {link}) for each failure (node, ifName): the
    link of `node` whose interface on `node` is `ifName`.  Returns
    (base, [per failure])."""
    n = len(fails)
    fn = (C.c_char_p * max(1, n))(*[f[0].encode() for f in fails])
    fi = (C.c_char_p * max(1, n))(*[f[1].encode() for f in fails])
    base = OrcDigest()
    out = (OrcDigest * max(1, n))()
    rc = lib.orc_ls_whatif_digests(orc._h, table.blob, _p(table.offs), _p(table.lens), table.n,
                                   src.encode(), fn, fi, n, int(fast), C.byref(base), out)
    assert rc == 0, f"failed link {-rc - 1} not found"
    t = lambda d: (int(d.n_dist_changed), int(d.n_nh_changed), int(d.hash))  # noqa: E731
    return t(base), [t(out[i]) for i in range(n)]


def time_whatif(orc: "OracleLinkState", src: str, fails: Sequence[tuple], fast: bool = True) -> int:
    fn = (C.c_char_p * len(fails))(*[f[0].encode() for f in fails])
    fi = (C.c_char_p * len(fails))(*[f[1].encode() for f in fails])
    return int(lib.orc_ls_time_whatif(orc._h, src.encode(), fn, fi, len(fails), int(fast)))


# ---- SpfSolver next hops --------------------------------------------------------
lib.orc_ls_nexthops_json.restype = C.c_char_p
lib.orc_ls_nexthops_json.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_char_p), C.c_uint32,
                                     C.c_int, C.c_int, C.c_int64]


def nexthops(orc: "OracleLinkState", me: str, dsts: Sequence[str], lfa: bool = False,
             v4: bool = False, swap_label: Optional[int] = None) -> Dict:
    """getNextHopsWithMetric + getNextHopsThrift (Decision.cpp:1107-1305) of
    `me` towards `dsts`: {"min": metric|None, "nh": sorted rows [ifName, metric,
    neighbour, addrHex, action|None, swapLabel|None]}."""
    arr = (C.c_char_p * max(1, len(dsts)))(*[d.encode() for d in dsts])
    raw = lib.orc_ls_nexthops_json(orc._h, me.encode(), arr, len(dsts), int(lfa), int(v4),
                                   -1 if swap_label is None else swap_label)
    return json.loads(raw)


lib.orc_ls_sr_nexthops_json.restype = C.c_char_p
lib.orc_ls_sr_nexthops_json.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_char_p),
                                        C.POINTER(C.c_int64), C.c_uint32, C.c_int, C.c_int,
                                        C.c_int]


def sr_nexthops(orc: "OracleLinkState", me: str, dsts: Dict[str, Optional[int]], lfa: bool,
                v4: bool, ksp2: bool) -> List[list]:
    """SR_MPLS next hops of one prefix (Decision.cpp:829-1018): `dsts` maps
    each best advertiser to its entry's prependLabel.  Sorted rows [ifName,
    metric, neighbour, addrHex, "PUSH"|None, [labels]|None]."""
    names = sorted(dsts)
    arr = (C.c_char_p * max(1, len(names)))(*[d.encode() for d in names])
    pre = (C.c_int64 * max(1, len(names)))(*[-1 if dsts[d] is None else dsts[d] for d in names])
    raw = lib.orc_ls_sr_nexthops_json(orc._h, me.encode(), arr, pre, len(names), int(lfa),
                                      int(v4), int(ksp2))
    return json.loads(raw)["nh"]


# ---- full-size parity digests (oracle/spf_oracle.cpp, "Full-size parity digests") ----
_u32p, _u64p = C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)
lib.orc_ls_route_digests.restype = C.c_int
lib.orc_ls_route_digests.argtypes = [C.c_void_p, C.c_char_p, _u32p, _u32p, C.c_uint32, _u32p,
                                     C.c_uint32, _u32p, _u32p, C.c_uint32, C.c_int, C.c_int, _u64p]
lib.orc_link_keyhash.restype = C.c_uint64
lib.orc_link_keyhash.argtypes = [C.c_char_p] * 4
lib.orc_ls_source_digests.restype = C.c_int
lib.orc_ls_source_digests.argtypes = [C.c_void_p, C.c_char_p, _u32p, _u32p, C.c_uint32, _u32p,
                                      C.c_uint32, C.c_int, C.c_int, C.c_int, _u64p]
lib.orc_digest_planar.restype = C.c_int
lib.orc_digest_planar.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, _u32p, _u32p, _u64p, _u32p,
                                  C.c_int, _u64p]
lib.orc_ls_ksp2_digests.restype = C.c_int
lib.orc_ls_ksp2_digests.argtypes = [C.c_void_p, C.c_char_p, _u32p, _u32p, C.c_uint32, _u32p,
                                    C.c_uint32, C.c_int, _u64p, _u64p]
lib.orc_digest_ksp2.restype = C.c_int
lib.orc_digest_ksp2.argtypes = [C.c_uint32, C.c_uint32, _u32p, _u32p, _u64p, C.c_int, _u64p, _u64p]
lib.orc_ls_whatif_int.restype = C.c_int
lib.orc_ls_whatif_int.argtypes = [C.c_void_p, C.c_char_p, _u32p, _u32p, C.c_uint32, C.c_char_p,
                                  C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.c_uint32,
                                  C.c_int, C.POINTER(OrcDigest), C.POINTER(OrcDigest)]


def host_threads() -> int:
    import os

    return max(1, min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1),
                      os.cpu_count() or 1, 16))


def link_keyhash(key: Sequence[str]) -> int:
    """Hash of a link's ordered key [n1, if1, n2, if2] (helpers.link_key)."""
    return int(lib.orc_link_keyhash(*[s.encode() for s in key]))


def source_digests(orc: "OracleLinkState", table: NameTable, srcs: Sequence[int],
                   ulm: bool = True, int_path: bool = False, threads: int = 0) -> np.ndarray:
    """u64 digest of runSpf(src) per source (ids into `table`)."""
    srcs = np.ascontiguousarray(srcs, np.uint32)
    out = np.zeros(max(1, len(srcs)), np.uint64)
    lib.orc_ls_source_digests(orc._h, table.blob, _p(table.offs), _p(table.lens), table.n,
                              _p(srcs), len(srcs), int(ulm), int(int_path),
                              threads or host_threads(), _p(out, C.c_uint64))
    return out[: len(srcs)]


def digest_planar(dist: np.ndarray, nh: np.ndarray, nh_off: np.ndarray, k: np.ndarray,
                  pitch: int, threads: int = 0) -> np.ndarray:
    """The same digest over the engine's output layout (dist [n_src, n] u32)."""
    dist = np.ascontiguousarray(dist, np.uint32)
    nh = np.ascontiguousarray(nh, np.uint32)
    nh_off = np.ascontiguousarray(nh_off, np.uint64)
    k = np.ascontiguousarray(k, np.uint32)
    n_src, n = dist.shape
    out = np.zeros(max(1, n_src), np.uint64)
    lib.orc_digest_planar(n_src, n, pitch, _p(dist), _p(nh), _p(nh_off, C.c_uint64), _p(k),
                          threads or host_threads(), _p(out, C.c_uint64))
    return out[:n_src]


def ksp2_digests(orc: "OracleLinkState", table: NameTable, srcs: Sequence[int],
                 pairs: bool = False, threads: int = 0):
    """Per-source digest of getKthPaths(src, d, 1|2) over every d; with
    pairs=True also the per-pair digests [n_src, n]."""
    srcs = np.ascontiguousarray(srcs, np.uint32)
    out = np.zeros(max(1, len(srcs)), np.uint64)
    pout = np.zeros((len(srcs), table.n), np.uint64) if pairs else None
    lib.orc_ls_ksp2_digests(orc._h, table.blob, _p(table.offs), _p(table.lens), table.n,
                            _p(srcs), len(srcs), threads or host_threads(), _p(out, C.c_uint64),
                            _p(pout, C.c_uint64) if pairs else None)
    return (out[: len(srcs)], pout) if pairs else out[: len(srcs)]


def digest_ksp2(pairs: np.ndarray, pool: np.ndarray, n_src: int, n: int,
                link_hash: np.ndarray, with_pairs: bool = False, threads: int = 0):
    """The same reduction over engine KSP2 output (spf_ksp2_pair records)."""
    pr = np.ascontiguousarray(pairs).view(np.uint32)
    pool = np.ascontiguousarray(pool, np.uint32)
    if pool.size == 0:
        pool = np.zeros(1, np.uint32)
    lh = np.ascontiguousarray(link_hash, np.uint64)
    out = np.zeros(max(1, n_src), np.uint64)
    pout = np.zeros((n_src, n), np.uint64) if with_pairs else None
    lib.orc_digest_ksp2(n_src, n, _p(pr), _p(pool), _p(lh, C.c_uint64), threads or host_threads(),
                        _p(out, C.c_uint64), _p(pout, C.c_uint64) if with_pairs else None)
    return (out[:n_src], pout) if with_pairs else out[:n_src]


def whatif_digests_int(orc: "OracleLinkState", table: NameTable, src: str,
                       fails: Sequence[tuple], threads: int = 0):
    """whatif_digests on the integer-CSR restatement, multi-threaded; returns
    (base tuple, structured DIGEST array [n])."""
    n = len(fails)
    fn = (C.c_char_p * max(1, n))(*[f[0].encode() for f in fails])
    fi = (C.c_char_p * max(1, n))(*[f[1].encode() for f in fails])
    base = OrcDigest()
    out = (OrcDigest * max(1, n))()
    rc = lib.orc_ls_whatif_int(orc._h, table.blob, _p(table.offs), _p(table.lens), table.n,
                               src.encode(), fn, fi, n, threads or host_threads(), C.byref(base),
                               out)
    assert rc == 0, f"failed link {-rc - 1} not found"
    arr = np.frombuffer(out, dtype=np.dtype([("n_dist_changed", "<u4"), ("n_nh_changed", "<u4"),
                                             ("hash", "<u8")]), count=n).copy()
    return (int(base.n_dist_changed), int(base.n_nh_changed), int(base.hash)), arr


lib.orc_keyvals_order.restype = C.c_uint32
lib.orc_keyvals_order.argtypes = [C.POINTER(C.c_char_p), C.c_uint32, _u32p]


def keyvals_order(keys: Sequence[str]) -> List[int]:
    """Wire indices of a publication's keyVals in the order the reference's
    std::unordered_map visits them (Decision.cpp:1726)."""
    arr = (C.c_char_p * max(1, len(keys)))(*[k.encode() for k in keys])
    out = np.zeros(max(1, len(keys)), np.uint32)
    k = lib.orc_keyvals_order(arr, len(keys), _p(out))
    return [int(x) for x in out[:k]]


lib.orc_node_area_map_order.restype = C.c_uint32
lib.orc_node_area_map_order.argtypes = [C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                        C.POINTER(C.c_uint8), C.c_uint32, _u32p]


def node_area_map_order(ops: Sequence[Tuple[int, Tuple[str, str]]]) -> List[Tuple[str, str]]:
    """Surviving (node, area) keys of a PrefixEntries map in the reference's
    iteration order after the emplace (1) / erase (0) history ``ops``."""
    n = max(1, len(ops))
    nodes = (C.c_char_p * n)(*[k[0].encode() for _, k in ops])
    areas = (C.c_char_p * n)(*[k[1].encode() for _, k in ops])
    code = (C.c_uint8 * n)(*[o for o, _ in ops])
    out = np.zeros(n, np.uint32)
    k = lib.orc_node_area_map_order(nodes, areas, code, len(ops), _p(out))
    return [ops[int(i)][1] for i in out[:k]]


def route_digests(orc: "OracleLinkState", table: NameTable, mes: Sequence[int],
                  set_ptr: np.ndarray, set_nodes: np.ndarray, lfa: bool,
                  threads: int = 0, kept_min: bool = False) -> np.ndarray:
    """spf_mplan_route_digests' reduction of the reference's route selection
    (orc_ls_route_digests): one u64 per me (ids into `table`).  kept_min:
    each route keyed by its smallest next-hop metric instead of the shortest
    distance (the form a materialised database is checked in)."""
    mes = np.ascontiguousarray(mes, np.uint32)
    sp = np.ascontiguousarray(set_ptr, np.uint32)
    sn = np.ascontiguousarray(set_nodes if len(set_nodes) else [0], np.uint32)
    out = np.zeros(max(1, len(mes)), np.uint64)
    rc = lib.orc_ls_route_digests(orc._h, table.blob, _p(table.offs), _p(table.lens), table.n,
                                  _p(mes), len(mes), _p(sp), _p(sn), len(sp) - 1, int(lfa) | (2 if kept_min else 0),
                                  threads or host_threads(), _p(out, C.c_uint64))
    assert rc == 0
    return out[: len(mes)]
