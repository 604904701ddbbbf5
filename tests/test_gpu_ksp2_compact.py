"""Compact KSP2 waves (u16 labels, 512-entry stack / queue per wave, the u32
redo pass behind them; openr_amd/csrc/ksp2.hip) against the u32 waves and the
CPU oracle's getKthPaths (LinkState.cpp:762-791).

Each case forces one of the compact waves' limits:
  * ring_deep      -- a 1100-node ring: k = 1 / k = 2 paths of up to 1099
                      links outgrow the 512-entry stack -> redo pass;
  * wan_big_metric -- metrics up to 60000: labels past 65534 -> redo pass;
  * rand_wide      -- the k = 2 SPF without its f = D + H order
                      (SPF_KSP2_DELTA = 2^32 - 1): BFS-like frontiers of more
                      than 512 nodes, worked in queue-sized chunks;
  * wan2000        -- BASELINE config 4's topology, where compact waves are
                      the default (no redo expected).
Every pair of a source batch must match the u32 waves path for path, the
k = 2 SPF count must match, and sampled pairs must match the oracle.
"""

import numpy as np
import pytest

from helpers import link_key
from oracle import OracleLinkState
from openr_amd import topology as T
from openr_amd.engine import PAIR_DTYPE, Ksp2Result, SpfEngine
from openr_amd.hiprt import DeviceArray
from openr_amd.link_state import LinkState

pytestmark = pytest.mark.gpu

CASES = [
    ("ring_deep", lambda: T.wan(1100, 0, seed=3, max_metric=3), {}, True),
    ("wan_big_metric", lambda: T.wan(300, 60, seed=4, max_metric=60000), {}, True),
    ("rand_wide", lambda: T.random_graph(4000, 6000, 11, max_metric=4),
     {"SPF_KSP2_DELTA": "4294967295"}, False),
    ("wan2000", lambda: T.wan(2000, 1000, seed=1), {}, False),
]


def run_plan(eng, srcs, n):
    p = eng.ksp2_plan(srcs)
    pairs = DeviceArray(len(srcs) * n * 4, np.uint32)
    cnt = DeviceArray(4, np.uint64, zero=True)
    words = len(srcs) * n * 24 + (1 << 22)
    pool = DeviceArray(words, np.uint32)
    try:
        p.execute(pairs.ptr, pool.ptr, words, cnt.ptr)
        eng.check()
        c = cnt.numpy().astype(np.int64)
        if c[0] > words:  # size the pool from the counter and run again
            pool.free()
            words = int(c[0]) + int(c[0]) // 4 + (1 << 20)  # grab slack varies run to run
            pool = DeviceArray(words, np.uint32)
            p.execute(pairs.ptr, pool.ptr, words, cnt.ptr)
            eng.check()
            c = cnt.numpy().astype(np.int64)
        assert c[0] <= words and not (c[2] & 3), c
        res = Ksp2Result(np.asarray(srcs, np.uint32), n,
                         pairs.numpy().view(PAIR_DTYPE).copy(), pool.numpy()[: c[0]].copy())
        return res, c
    finally:
        p.close()
        for b in (pairs, cnt, pool):
            b.free()


@pytest.mark.parametrize("name,make,env,expect_redo", CASES, ids=[c[0] for c in CASES])
def test_compact_waves_match_u32_waves_and_oracle(monkeypatch, name, make, env, expect_redo):
    topo = make()
    ls = LinkState(device=-1)
    ls.updateAdjacencyDatabases(topo.lsdb)
    names, rp, col, met, lid, ovl = ls.flatten()
    n = len(names)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(5)
    srcs = sorted(int(x) for x in rng.choice(n, 16, replace=False))
    with SpfEngine(0) as eng:
        eng.load(rp, col, met, lid, ovl)
        monkeypatch.setenv("SPF_KSP2_U16", "1")
        r16, c16 = run_plan(eng, srcs, n)
        monkeypatch.setenv("SPF_KSP2_U16", "0")
        r32, c32 = run_plan(eng, srcs, n)
    assert c16[1] == c32[1]  # k = 2 SPF runs, redone pairs counted once
    assert c32[3] == 0
    if expect_redo:
        assert c16[3] > 0
    elif name == "wan2000":
        assert c16[3] == 0
    for i in range(len(srcs)):
        for d in range(n):
            for k in (1, 2):
                assert r16.paths(i, d, k) == r32.paths(i, d, k), (name, srcs[i], d, k)
    orc = OracleLinkState()
    orc.update_packed(topo.lsdb)
    keys = {}

    def key(l):
        if l not in keys:
            keys[l] = link_key(ls._link(l))
        return keys[l]

    for i in (0, len(srcs) - 1):
        for d in sorted(int(x) for x in rng.choice(n, 12, replace=False)):
            for k in (1, 2):
                got = [[key(l) for l in p] for p in r16.paths(i, d, k)]
                assert got == orc.kth_paths(names[srcs[i]], names[d], k), (name, srcs[i], d, k)
