"""The CPU oracle against the reference's own test expectations (no GPU).

tests/golden/reference_expectations.json transcribes LinkStateTest.cpp and
DecisionTest.cpp (file:line in each case); passing here pins the oracle that
every GPU parity test compares against.
"""

import pytest

from adapters import OracleAdapter
from refcases import load_cases, run_case

CASES = load_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_tests(case):
    run_case(case, OracleAdapter)


def test_oracle_holdable_value_semantics():
    """HoldableValue through link metric holds (LinkStateTest.cpp:22-83 via
    LinkState): a metric increase is held for holdDownTtl decrements, a
    decrease for holdUpTtl; the SPF sees the held value until expiry."""
    from oracle import OracleLinkState
    from openr_amd.lsdb import create_adj_db, create_adjacency as A

    o = OracleLinkState()
    a12 = A("2", "1/2", "2/1", "fe80::2", "10.0.0.2", 10, 1)
    a21 = A("1", "2/1", "1/2", "fe80::1", "10.0.0.1", 10, 2)
    o.update([create_adj_db("1", [a12], 1), create_adj_db("2", [a21], 2)])
    assert o.spf("1")["2"]["metric"] == 10
    a12b = A("2", "1/2", "2/1", "fe80::2", "10.0.0.2", 30, 1)  # bringing down: holdDown
    chg = o.update([create_adj_db("1", [a12b], 1)], hold_up=10, hold_down=3)
    assert chg == [(False, False, False)] and o.has_holds()
    assert o.spf("1")["2"]["metric"] == 10
    assert o.decrement_holds() == (False, False, False)
    assert o.decrement_holds() == (False, False, False)
    assert o.decrement_holds() == (True, False, False)
    assert o.spf("1")["2"]["metric"] == 30 and not o.has_holds()
