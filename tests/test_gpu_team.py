"""msbfs_team_kernel (csrc/msbfs_team.hip): the unit-metric multi-source BFS
whose batches are swept by a team of G workgroups on one XCD -- what a rank
of a multi-GPU all-sources pass runs (few sources per GPU) -- against the
oracle, every source, for every team size (SPF_MSBFS_TEAM = G), with drained
nodes, hop counts and every next-hop row form."""

import numpy as np
import pytest

from openr_amd import topology as T
from test_gpu_engine import compare, load

pytestmark = pytest.mark.gpu

GRAPHS = [
    ("fabric_full1000", lambda: T.fabric(1000, full=True)),
    ("fabric_ref1000", lambda: T.fabric(1000, full=False)),
    ("rand_drained", lambda: T.random_graph(300, 3000, 11, max_metric=1, overload_frac=0.1)),
    ("sparse_drained", lambda: T.random_graph(400, 600, 3, max_metric=1, overload_frac=0.05)),
]


@pytest.mark.parametrize("G", ["2", "4", "8", "16", "32"])
@pytest.mark.parametrize("name,make", GRAPHS, ids=[g[0] for g in GRAPHS])
def test_team_bfs_every_team_size(name, make, G, monkeypatch):
    monkeypatch.setenv("SPF_MSBFS_TEAM", G)
    monkeypatch.setenv("SPF_MSBFS", "masks")
    names, eng, orc = load(make())
    assert eng.plan([0], hop=True).kernels()[0] == "msbfs_team_kernel"
    compare(names, eng, orc, list(range(len(names))), hop=True)
    compare(names, eng, orc, list(range(len(names))))
    compare(names, eng, orc, [5, 1, 5, 0])  # unsorted, duplicated sources


@pytest.mark.parametrize("narrow,sdirect,mode", [("0", "1", "u32"), ("1", "1", "u8"),
                                                  ("2", "0", "sliced"), ("2", "1", "sliced_bfs")])
def test_team_bfs_every_row_form(narrow, sdirect, mode, monkeypatch):
    """Every row form behind the team BFS: u32 rows, u8 rows, bit planes
    sliced from the u8 rows, and bit planes the team kernel writes itself
    (sdirect: no u8 rows, no slicing pass)."""
    monkeypatch.setenv("SPF_MSBFS_TEAM", "8")
    monkeypatch.setenv("SPF_MSBFS", "masks")
    monkeypatch.setenv("SPF_NARROW", narrow)
    monkeypatch.setenv("SPF_SDIRECT", sdirect)
    names, eng, orc = load(T.fabric(1000, full=True))
    p = eng.plan([0], hop=True)
    assert p.kernels()[0] == "msbfs_team_kernel" and p.row_mode() == mode
    compare(names, eng, orc, list(range(len(names))))
    compare(names, eng, orc, list(range(0, len(names), 7)), hop=True)


@pytest.mark.parametrize("depth", [1, 2, 3, 5, 6, 13, 14, 15, 16, 40])
def test_team_planes_every_depth(depth, monkeypatch):
    """The team kernel's distances live in 4 register bit planes per node,
    written in windows of 15 levels: shallow graphs take the sdirect rows
    (the planes are the next-hop pass's input), deeper ones the u8 rows and
    window flushes (a dense core with a path tail sets the depth)."""
    monkeypatch.setenv("SPF_MSBFS_TEAM", "4")
    monkeypatch.setenv("SPF_MSBFS", "masks")
    monkeypatch.setenv("SPF_NARROW", "2")
    names, eng, orc = load(T.clique_with_tail(12, depth))
    p = eng.plan([0], hop=True)
    assert p.kernels()[0] == "msbfs_team_kernel"
    assert p.row_mode() in ("sliced", "sliced_bfs")
    compare(names, eng, orc, list(range(len(names))), hop=True)
    compare(names, eng, orc, list(range(len(names))))


def test_team_bfs_chosen_for_a_rank_share_of_the_fabric():
    """A world-8 rank's share of fabric_full (~1250 sources) takes the team
    kernel by default (the cost model in msbfs_team_size)."""
    names, eng, orc = load(T.fabric(10000, full=True))
    assert eng.plan(list(range(1250))).kernels()[0] == "msbfs_team_kernel"
    rng = np.random.default_rng(3)
    compare(names, eng, orc, sorted(int(x) for x in rng.choice(len(names), 40, replace=False)))


@pytest.mark.parametrize("group", ["0", "1"])
def test_sliced_next_hops_grouped_and_per_source(group, monkeypatch):
    """The sliced next-hop pass with grouped units (sources of one XCD list
    with identical neighbour rows share each row load) and without
    (SPF_SLICED_GROUP=0), on the BFS-written planes and on sliced u8 rows,
    with drained nodes (their sources are never grouped)."""
    monkeypatch.setenv("SPF_SLICED_GROUP", group)
    monkeypatch.setenv("SPF_NARROW", "2")
    for topo in (T.fabric(1000, full=True),
                 T.random_graph(300, 3000, 11, max_metric=1, overload_frac=0.1)):
        names, eng, orc = load(topo)
        assert eng.plan([0]).row_mode() in ("sliced", "sliced_bfs")
        compare(names, eng, orc, list(range(len(names))))


def test_team_timeout_turns_teams_off_and_the_plan_reruns_on_msbfs_kernel(monkeypatch):
    """A team barrier that times out (another process's grid holding CUs;
    here the kernel's test hook SPF_TEAM_FLUSH_DBG=32 reports one) fails the
    check loudly, and the same plan's next execute re-derives onto
    msbfs_kernel -- no second poll until timeout -- with oracle-exact rows."""
    from openr_amd._native import SpfError

    monkeypatch.setenv("SPF_MSBFS_TEAM", "8")
    monkeypatch.setenv("SPF_MSBFS", "masks")
    names, eng, orc = load(T.fabric(1000, full=True))
    srcs = list(range(0, len(names), 3))
    p = eng.plan(srcs)
    assert p.kernels()[0] == "msbfs_team_kernel"
    monkeypatch.setenv("SPF_TEAM_FLUSH_DBG", "32")
    with pytest.raises(SpfError, match="team BFS barrier timed out"):
        p.execute_host()
    monkeypatch.delenv("SPF_TEAM_FLUSH_DBG")
    res = p.execute_host()
    assert p.kernels()[0] == "msbfs_kernel"
    dist, mats = orc.dense(names, srcs, ulm=True)
    exp = np.where(dist == np.iinfo(np.uint64).max, 0xFFFFFFFF, dist).astype(np.uint32)
    assert np.array_equal(res.dist, exp)
    for i, s in enumerate(srcs):
        k = len(eng.neighbors(s))
        assert np.array_equal(res.nh_matrix(i), mats[i][:k])
    assert eng.plan(srcs).kernels()[0] == "msbfs_kernel"  # new plans too
