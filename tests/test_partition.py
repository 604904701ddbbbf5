"""The engine's source partition (spf_partition_sources, host only: the rule
spf_mplan and bench.py's multi-rank layout use) against its numpy
restatement (sharding.locality_partition and AllSourcesLayout's contiguous
blocks), and the multi-device C-ABI refusing loudly without a GPU."""

import ctypes

import numpy as np
import pytest

from openr_amd import _native as N
from openr_amd import topology as T
from openr_amd.engine import graph_from_lsdb, partition_sources
from openr_amd.sharding import AllSourcesLayout, closure_sizes, locality_partition


def _neighbors(topo):
    """Distinct up neighbours per node, ascending (spf_src_neighbors' lists)."""
    names, rp, col, met, lid, ovl = graph_from_lsdb(topo.lsdb)
    n = len(names)
    nbrs = [np.unique(col[rp[u]:rp[u + 1]]).astype(np.uint32) for u in range(n)]
    nb_ptr = np.concatenate([[0], np.cumsum([len(x) for x in nbrs])]).astype(np.uint32)
    nb_id = np.concatenate(nbrs).astype(np.uint32) if n else np.zeros(0, np.uint32)
    return nbrs, nb_ptr, nb_id


TOPOS = {
    "fabric": lambda: T.fabric(1000, full=True),
    "fabric_ref": lambda: T.fabric(1200, full=False),
    "grid": lambda: T.grid(24),
    "wan": lambda: T.wan(400, 250, seed=5),
}


@pytest.mark.parametrize("topo", sorted(TOPOS))
@pytest.mark.parametrize("world", [2, 3, 8])
def test_native_locality_partition_equals_numpy_restatement(topo, world):
    nbrs, nb_ptr, nb_id = _neighbors(TOPOS[topo]())
    n = len(nbrs)
    k = np.array([len(x) for x in nbrs], np.int64)
    want = locality_partition(nbrs, k + AllSourcesLayout.ROW_COST, world)
    part, used = partition_sources(nb_ptr, nb_id, np.arange(n), world, "locality")
    assert used == "locality"
    for r in range(world):
        assert np.array_equal(np.flatnonzero(part == r), want[r]), f"part {r} differs"


@pytest.mark.parametrize("topo", sorted(TOPOS))
@pytest.mark.parametrize("world", [2, 4, 8])
def test_native_contiguous_and_auto_equal_layout(topo, world):
    nbrs, nb_ptr, nb_id = _neighbors(TOPOS[topo]())
    n = len(nbrs)
    k = np.array([len(x) for x in nbrs], np.int64)
    # contiguous blocks: the layout without neighbour lists
    plain = AllSourcesLayout(k, 1024, world)
    part, used = partition_sources(nb_ptr, nb_id, np.arange(n), world, "contiguous")
    assert used == "contiguous"
    for r in range(world):
        assert np.array_equal(np.flatnonzero(part == r), plain.srcs[r])
    # auto: the smaller largest closure, exactly as the numpy rule picks
    loc = locality_partition(nbrs, k + AllSourcesLayout.ROW_COST, world)
    pick_loc = max(closure_sizes(loc, nbrs, n)) < max(closure_sizes(plain.srcs, nbrs, n))
    part, used = partition_sources(nb_ptr, nb_id, np.arange(n), world, "auto")
    assert used == ("locality" if pick_loc else "contiguous")
    lay = AllSourcesLayout(k, 1024, world, nbrs=nbrs)
    assert lay.partition == used
    for r in range(world):
        assert np.array_equal(np.flatnonzero(part == r), lay.srcs[r])


def test_partition_of_a_source_subset_covers_it_once():
    nbrs, nb_ptr, nb_id = _neighbors(T.fabric(1000, full=True))
    srcs = np.arange(3, len(nbrs), 7, dtype=np.uint32)
    for mode in ("contiguous", "locality", "auto"):
        part, _ = partition_sources(nb_ptr, nb_id, srcs, 4, mode)
        assert len(part) == len(srcs) and part.max() < 4
        assert np.bincount(part, minlength=4).min() > 0


def test_partition_rejects_bad_arguments():
    nb_ptr = np.array([0, 1, 2], np.uint32)
    nb_id = np.array([1, 0], np.uint32)
    with pytest.raises(N.SpfError):
        partition_sources(nb_ptr, nb_id, [0, 5], 2)  # source out of range
    with pytest.raises(N.SpfError):
        partition_sources(nb_ptr, nb_id, [0, 1], 0)  # no parts


def test_multi_context_without_gpu_reports_no_device():
    import torch

    if torch.cuda.is_available():
        return
    ids = (ctypes.c_int * 2)(0, 0)
    h = ctypes.c_void_p()
    st = N.lib.spf_mctx_create(ids, 2, ctypes.byref(h))
    assert st == N.SPF_E_NO_DEVICE and not h.value
    st = N.lib.ls_create_multi(b"0", ids, 2, ctypes.byref(h))
    assert st == N.SPF_E_NO_DEVICE and not h.value
