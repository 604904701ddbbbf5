"""Batched KSP2 and what-if outside the positive-u32 envelope, on the exact
kernel (csrc/exact.hip): zero-metric plateaus (next hops and pathLinks
follow the reference's (metric, name) pop order, LinkState.h:488-498),
negative metrics (the i32 -> u64 conversion wraps, LinkState.h:22) and
graphs forced there (SPF_KSP2_EXACT), against the oracle's getKthPaths
(LinkState.cpp:762-791) and its runSpf(src, true, {l}) digests."""

import numpy as np
import pytest

from oracle import NameTable, whatif_digests
from openr_amd import topology as T
from test_gpu_ksp2 import check_pairs, setup as ksp_setup
from test_gpu_whatif import as_tuple, fail_of, setup as wi_setup

pytestmark = pytest.mark.gpu


def _zero(topo, frac, seed, negative=False):
    m = topo.lsdb.adjs["metric"]
    rng = np.random.default_rng(seed)
    pick = rng.choice(len(m), max(1, int(len(m) * frac)), replace=False)
    m[pick] = 0
    if negative:
        m[pick[: max(1, len(pick) // 4)]] = -3
    return topo


CASES = [
    ("rand_zero", lambda: _zero(T.random_graph(30, 70, 41, max_metric=4, parallel_frac=0.25,
                                               overload_frac=0.1, link_overload_frac=0.05), 0.3, 1)),
    ("grid_zero", lambda: _zero(T.grid(6), 0.4, 2)),
    ("wan_zero", lambda: _zero(T.wan(60, 30, seed=9, max_metric=5), 0.25, 3)),
    ("rand_negative", lambda: _zero(T.random_graph(25, 50, 43, max_metric=4), 0.3, 4, negative=True)),
]


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_exact_ksp2_all_pairs(name, make):
    names, eng, orc, key, _ = ksp_setup(make())
    check_pairs(names, eng, orc, key, list(range(len(names))))


@pytest.mark.parametrize("name,make", [
    ("grid6", lambda: T.grid(6)),
    ("rand", lambda: T.random_graph(30, 70, 205, max_metric=6, parallel_frac=0.25,
                                    overload_frac=0.1, link_overload_frac=0.05)),
], ids=["grid6", "rand"])
def test_exact_ksp2_forced_on_positive_graphs(name, make, monkeypatch):
    """The exact KSP2 path (what graphs past 65535 nodes or the LDS take)
    forced onto positive-metric graphs (SPF_KSP2_EXACT=1)."""
    monkeypatch.setenv("SPF_KSP2_EXACT", "1")
    names, eng, orc, key, _ = ksp_setup(make())
    check_pairs(names, eng, orc, key, list(range(len(names))))


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_exact_whatif_every_failure(name, make):
    ls, names, eng, orc, _ = wi_setup(make())
    for s in (0, len(names) // 2):
        links, got, base = eng.whatif(s)
        obase, want = whatif_digests(orc, NameTable(names), names[s],
                                     [fail_of(ls, l) for l in links], fast=False)
        assert as_tuple(base) == obase
        for l, g, w in zip(links, got, want):
            assert as_tuple(g) == w, (names[s], fail_of(ls, l))
