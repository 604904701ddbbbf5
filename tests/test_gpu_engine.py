"""Engine parity on the MI355X: batched all-sources SPF + ECMP (libopenr_spf.so)
against the CPU oracle, bit-exact.

Small graphs: every source, full dist + next-hop bitsets.  Full BASELINE sizes
(fabric 10k, grid 100x100): sampled sources compared exactly, plus
size-independent properties over ALL sources of one batched plan.
"""

import numpy as np
import pytest

from oracle import OracleLinkState
from openr_amd import topology as T
from openr_amd.engine import SpfEngine, graph_from_lsdb

pytestmark = pytest.mark.gpu

U32_INF = np.uint32(0xFFFFFFFF)


def load(topo):
    names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
    eng = SpfEngine(0)
    eng.load(rp, col, met, lid, ovl)
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    return names, eng, orc


def compare(names, eng, orc, srcs, hop=False):
    res = eng.solve(srcs, hop=hop)
    dist, mats = orc.dense(names, srcs, ulm=not hop)
    exp = np.where(dist == np.iinfo(np.uint64).max, U32_INF, dist).astype(np.uint32)
    assert np.array_equal(res.dist, exp), "distance mismatch"
    for i, s in enumerate(srcs):
        k = len(eng.neighbors(s))
        assert int(res.words[i]) == k
        got = res.nh_matrix(i)
        want = mats[i][:k]
        assert not mats[i][k:].any()
        if not np.array_equal(got, want):
            j, v = (int(x[0]) for x in np.nonzero(got != want))
            raise AssertionError(f"next-hop mismatch src {names[s]} dst {names[v]} "
                                 f"neighbour {names[eng.neighbors(s)[j]]}: "
                                 f"gpu {bool(got[j, v])} oracle {bool(want[j, v])}")
    return res


SMALL = [
    ("grid10", lambda: T.grid(10)),
    ("dtgrid8", lambda: T.decision_test_grid(8)),
    ("fabric_ref1000", lambda: T.fabric(1000, full=False)),
    ("fabric_full1000", lambda: T.fabric(1000, full=True)),
    ("wan300", lambda: T.wan(300, 150, seed=3)),
] + [
    (f"rand{seed}", (lambda s: lambda: T.random_graph(
        60, 150, s, max_metric=8, parallel_frac=0.2, overload_frac=0.1,
        link_overload_frac=0.05))(seed))
    for seed in range(6)
]


@pytest.mark.parametrize("name,make", SMALL, ids=[s[0] for s in SMALL])
@pytest.mark.parametrize("hop", [False, True], ids=["metric", "hops"])
def test_all_sources_exact(name, make, hop):
    names, eng, orc = load(make())
    compare(names, eng, orc, list(range(len(names))), hop=hop)


def test_subset_and_duplicates_exact():
    """Non-closed source sets (engine adds neighbour rows internally),
    duplicates and a single source."""
    names, eng, orc = load(T.random_graph(50, 120, 11, overload_frac=0.15))
    rng = np.random.default_rng(0)
    for srcs in ([7], [3, 3, 9], list(rng.choice(len(names), 13, replace=False))):
        compare(names, eng, orc, [int(s) for s in srcs])


def test_all_overloaded_and_isolated():
    topo = T.random_graph(30, 40, 5, overload_frac=0.9)
    names, eng, orc = load(topo)
    compare(names, eng, orc, list(range(len(names))))


@pytest.mark.parametrize("which", ["fabric_full", "grid100"])
def test_baseline_size_sampled_exact_and_all_sources_properties(which):
    topo = T.fabric(10000, full=True) if which == "fabric_full" else T.grid(100)
    names, eng, orc = load(topo)
    n = len(names)
    rng = np.random.default_rng(1)
    sample = sorted(int(x) for x in rng.choice(n, 6, replace=False))
    compare(names, eng, orc, sample)
    # all sources in one batched plan: properties that hold for any source
    res = eng.solve(list(range(n)))
    d = res.dist
    assert (d.diagonal() == 0).all()
    assert (d != U32_INF).all()  # connected
    assert np.array_equal(d, d.T)  # unit symmetric metrics, nothing drained
    # rows of the batch equal the same sources solved alone
    for s in sample:
        one = eng.solve([s])
        assert np.array_equal(one.dist[0], d[s])
        assert np.array_equal(one.nh_matrix(0), res.nh_matrix(s))
    # next hops: empty only at the source, and x in nh_s(v) <=> d(x,v) = d(s,v) - 1
    for s in sample:
        mat = res.nh_matrix(s)
        nbrs = eng.neighbors(s)
        has = mat.any(axis=0)
        assert not has[s] and has[np.arange(n) != s].all()
        for j, x in enumerate(nbrs):
            assert np.array_equal(mat[j], d[x].astype(np.int64) + 1 == d[s])


def test_zero_metric_runs_the_exact_kernel():
    """A zero-metric link routes weighted plans to the exact kernel
    (test_gpu_exact.py covers it in depth); hop counts stay on the BFS."""
    topo = T.random_graph(20, 30, 2)
    topo.lsdb.adjs["metric"][0] = 0
    names, eng, orc = load(topo)
    assert eng.plan([0]).kernels()[0] == "exact_spf_kernel"
    assert eng.plan([0], hop=True).kernels()[0] != "exact_spf_kernel"
    compare(names, eng, orc, list(range(len(names))))
    compare(names, eng, orc, list(range(len(names))), hop=True)
    compare(names, eng, orc, [3, 1, 3, 0])  # unsorted, duplicated sources


ROW_MODES = {"0": "u32", "1": "u8", "2": "sliced"}


@pytest.mark.parametrize("narrow", ["0", "1", "2"])
@pytest.mark.parametrize("name,make", [
    ("fabric_full1000", lambda: T.fabric(1000, full=True)),
    ("grid12", lambda: T.grid(12)),
    ("rand_drained", lambda: T.random_graph(60, 150, 7, max_metric=1, overload_frac=0.15)),
    ("fabric_drained", lambda: T.random_graph(300, 3000, 11, max_metric=1, overload_frac=0.1)),
], ids=["fabric", "grid", "rand", "dense_drained"])
def test_next_hop_pass_every_row_form(name, make, narrow, monkeypatch):
    """The BFS plans' next-hop pass on the exact u32 rows, on u8 narrow rows
    and on their bit-sliced planes (the plan picks by degree and BFS kernel;
    SPF_NARROW=0/1/2 forces it), unit metrics and hop counts."""
    monkeypatch.setenv("SPF_NARROW", narrow)
    monkeypatch.setenv("SPF_MSBFS", "masks")  # the per-level BFS reports the depth slicing needs
    monkeypatch.setenv("SPF_MSBFS_TEAM", "0")  # msbfs_kernel's row forms (team: test_gpu_team.py)
    names, eng, orc = load(make())
    assert eng.plan([0], hop=True).row_mode() == ROW_MODES[narrow]
    compare(names, eng, orc, list(range(len(names))), hop=True)
    compare(names, eng, orc, list(range(len(names))))


@pytest.mark.parametrize("narrow", ["1", "2"])
def test_saturated_narrow_rows_fall_back_to_exact(narrow, monkeypatch):
    """Hop distances >= 254 saturate the u8 copy: the byte pass decides those
    waves on the u32 rows, the sliced pass the whole plan.  A 700-node ring
    has distances up to 350."""
    monkeypatch.setenv("SPF_NARROW", narrow)
    monkeypatch.setenv("SPF_MSBFS", "masks")
    topo = T.wan(700, 0, seed=1)  # ring only
    names, eng, orc = load(topo)
    rng = np.random.default_rng(5)
    compare(names, eng, orc, sorted(int(x) for x in rng.choice(len(names), 40, replace=False)),
            hop=True)


@pytest.mark.parametrize("depth", [1, 2, 3, 6, 7, 14, 15, 30, 31, 126, 127, 253])
def test_sliced_plane_counts(depth, monkeypatch):
    """Every plane count of the sliced pass: a dense core with a path tail
    whose length sets the deepest level (P = bits of maxd + 1 changes at
    maxd = 1, 3, 7, ... 127; 253 is the last depth before the u8 copy
    saturates)."""
    monkeypatch.setenv("SPF_NARROW", "2")
    monkeypatch.setenv("SPF_MSBFS", "masks")
    monkeypatch.setenv("SPF_MSBFS_TEAM", "0")  # slice_rows_kernel's plane counts
    names, eng, orc = load(T.clique_with_tail(12, depth))
    p = eng.plan([0], hop=True)
    assert p.row_mode() == "sliced"
    compare(names, eng, orc, list(range(len(names))), hop=True)


@pytest.mark.parametrize("variant", ["planes", "masks"])
@pytest.mark.parametrize("name,make", [
    ("fabric_full1000", lambda: T.fabric(1000, full=True)),
    ("grid30", lambda: T.grid(30)),
    ("rand_drained", lambda: T.random_graph(60, 150, 7, max_metric=1, overload_frac=0.15)),
    ("ring1200", lambda: T.wan(1200, 0, seed=1)),  # 600 levels: three plane windows
    ("ring_drained", lambda: T.random_graph(400, 400, 3, max_metric=1, overload_frac=0.05)),
], ids=["fabric", "grid", "rand", "ring1200", "sparse_drained"])
def test_bfs_variants_exact(name, make, variant, monkeypatch):
    """Both multi-source BFS kernels (register bit planes, 32 sources per
    workgroup; per-level mask stores, 64 sources), with both next-hop row
    widths; SPF_MSBFS / SPF_NARROW force the choice the plan makes by degree."""
    monkeypatch.setenv("SPF_MSBFS", variant)
    names, eng, orc = load(make())
    for narrow in ("0", "1", "2"):
        monkeypatch.setenv("SPF_NARROW", narrow)
        compare(names, eng, orc, list(range(len(names))), hop=True)


@pytest.mark.parametrize("name,make", SMALL, ids=[n for n, _ in SMALL])
def test_big_graph_kernel_exact(name, make, monkeypatch):
    """spf_big_kernel (the plans on graphs beyond the LDS-resident kernels:
    cooperative frontier SSSP, next hops in distance order, transpose to the
    bitmap layout) forced onto small graphs (SPF_BIG=1), every source,
    weighted and hop counts, against the oracle."""
    monkeypatch.setenv("SPF_BIG", "1")
    names, eng, orc = load(make())
    assert eng.plan([0]).kernels()[0] == "spf_big_kernel"
    compare(names, eng, orc, list(range(len(names))))
    compare(names, eng, orc, list(range(len(names))), hop=True)
    compare(names, eng, orc, [3, 1, 3, 0])  # unsorted, duplicated sources


@pytest.mark.parametrize("expand", ["0", "1"])
@pytest.mark.parametrize("name,make", [
    ("fabric_full1000", lambda: T.fabric(1000, full=True)),
    ("ring700", lambda: T.wan(700, 0, seed=1)),  # distances to 350: saturated u8 bytes
    ("rand_drained", lambda: T.random_graph(300, 3000, 11, max_metric=1, overload_frac=0.1)),
], ids=["fabric", "ring700", "dense_drained"])
def test_expanded_u32_rows(name, make, expand, monkeypatch):
    """Sliced plans whose BFS writes both row forms (default) and whose BFS
    stores only the u8 rows, the slicing pass expanding them into the u32
    rows (SPF_EXPAND=1): every source's rows and next hops against the
    oracle, including the saturated levels (>= 254) the BFS still writes as
    u32 in the second mode."""
    monkeypatch.setenv("SPF_EXPAND", expand)
    monkeypatch.setenv("SPF_NARROW", "2")
    monkeypatch.setenv("SPF_MSBFS", "masks")
    monkeypatch.setenv("SPF_MSBFS_TEAM", "0")
    names, eng, orc = load(make())
    assert eng.plan([0], hop=True).row_mode() == "sliced"
    compare(names, eng, orc, list(range(len(names))), hop=True)
    compare(names, eng, orc, list(range(0, len(names), 3)))


@pytest.mark.parametrize("name,make,srcs", [
    ("fabric_full1000", lambda: T.fabric(1000, full=True), slice(0, None)),
    ("grid30", lambda: T.grid(30), slice(0, None)),
    ("fabric_block", lambda: T.fabric(1000, full=True), slice(300, 500)),  # closure != sources
    ("ring700", lambda: T.wan(700, 0, seed=1), slice(0, 40)),  # distances past 254 saturate
], ids=["fabric", "grid", "fabric_block", "ring700"])
def test_copy_narrow_rows(name, make, srcs, monkeypatch):
    """spf_plan_copy_narrow_rows (the u8 rows the multi-GPU gather ships):
    byte = min(d, 254), 255 = unreachable and row padding, rows in plan
    source order, against the same execute's u32 rows."""
    from openr_amd.hiprt import DeviceArray, synchronize

    if name == "ring700":  # a sparse ring's plans read u32 rows unless told
        monkeypatch.setenv("SPF_NARROW", "2")
        monkeypatch.setenv("SPF_MSBFS", "masks")
    names, eng, orc = load(make())
    ids = list(range(len(names)))[srcs]
    plan = eng.plan(ids, hop=True)  # the ring's metrics are not unit: hop counts
    assert plan.row_mode() != "u32"
    pitch, m = eng.pitch, len(ids)
    d32 = DeviceArray(m * pitch, np.uint32)
    nh = DeviceArray(max(1, plan.nh_words), np.uint32)
    d8 = DeviceArray(m * pitch, np.uint8)
    try:
        plan.execute(d32.ptr, nh.ptr)
        plan.copy_narrow_rows(d8.ptr)
        synchronize()
        a = d32.numpy().reshape(m, pitch)
        b = d8.numpy().reshape(m, pitch)
        want = np.where(a == 0xFFFFFFFF, 255, np.minimum(a, 254)).astype(np.uint8)
        assert np.array_equal(b, want)
    finally:
        for x in (d32, nh, d8):
            x.free()


@pytest.mark.parametrize("narrow", ["0", "1"])
@pytest.mark.parametrize("name,make", [
    ("fabric_rtt600", lambda: T.fabric_rtt(num_sws=600)),
    ("wan_dense", lambda: T.random_graph(400, 3200, 5, max_metric=40, overload_frac=0.05)),
    ("wan_deep", lambda: T.random_graph(500, 2600, 9, max_metric=600)),  # rows saturate at 254
], ids=["fabric_rtt", "dense_drained", "deep"])
def test_weighted_narrow_rows(name, make, narrow, monkeypatch):
    """Weighted plans with a u8 copy of the rows (the next-hop pass matches
    bytes against d_s - w(s, x) per neighbour, exact u32 rows where a
    source slice saturates) and without (SPF_NARROW=0): every source's
    distances and next hops against the oracle."""
    monkeypatch.setenv("SPF_NARROW", narrow)
    names, eng, orc = load(make())
    plan = eng.plan([0])
    assert plan.row_mode() == ("u8" if narrow == "1" else "u32")
    compare(names, eng, orc, list(range(len(names))))


@pytest.mark.parametrize("name,make", [
    ("fabric_rtt600", lambda: T.fabric_rtt(num_sws=600)),
    ("wan_dense", lambda: T.random_graph(400, 3200, 5, max_metric=40, overload_frac=0.05)),
    ("wan_small_metrics", lambda: T.wan(300, 150, seed=4, max_metric=3)),
    ("wan_deep", lambda: T.random_graph(500, 2600, 9, max_metric=600)),  # saturates: u32 fallback
    ("rand_parallel", lambda: T.random_graph(120, 400, 7, max_metric=9, parallel_frac=0.2,
                                             overload_frac=0.1, link_overload_frac=0.05)),
], ids=["fabric_rtt", "dense_drained", "small_metrics", "deep", "parallel_drained"])
def test_weighted_sliced_next_hops(name, make, monkeypatch):
    """Weighted plans on mssp_kernel with bit-sliced rows (the default): next
    hops from d_x + w(s, x) == d_s formed bit-sliced per 32 destinations,
    drained neighbours, parallel links, metrics past the planes and rows
    deep enough to fall back to u32 rows -- every source against the oracle."""
    monkeypatch.setenv("SPF_NARROW", "2")  # u8 rows (then sliced) at any degree
    monkeypatch.delenv("SPF_WSLICED", raising=False)
    names, eng, orc = load(make())
    plan = eng.plan(list(range(len(names))))
    assert plan.kernels()[0] == "mssp_kernel" and plan.row_mode() == "sliced"
    compare(names, eng, orc, list(range(len(names))))
