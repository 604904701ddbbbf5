"""bench.py's parity plumbing that runs on the host: the link value hash its
KSP2 line feeds spf_ksp2_digest equals the oracle's (the hash the committed
fixtures were made with), for every link of the config-4 WAN graph."""

import sys
from pathlib import Path

import numpy as np

from helpers import link_key
from oracle import link_keyhash
from openr_amd import topology as T
from openr_amd.link_state import LinkState

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bench import link_value_hash  # noqa: E402


def test_link_value_hash_equals_oracle_keyhash():
    topo = T.wan(2000, 1000, seed=1)
    ls = LinkState(device=-1)
    ls.updateAdjacencyDatabases(topo.lsdb)
    lid = ls.flatten()[4]
    links = np.unique(lid)
    assert len(links) == 3000
    for l in links:
        lk = ls._link(int(l))
        (a, b), (c, d) = lk.orderedNames
        assert link_value_hash(a, b, c, d) == link_keyhash(link_key(lk))
    ls.close()
