"""Oracle JoinHash pinned to the reference's expected join tables (CPU only)."""
import pytest

import join_cases as jc
from helpers import assert_table_eq_unordered, tbl


@pytest.mark.parametrize("case", jc.CASES, ids=jc.CASE_IDS)
def test_oracle_join_matches_reference_fixture(hy, oracle, case):
    name, left, right, mode, cols, expected = case
    base = jc.BaseTables(hy)
    out = jc.eval_oracle(hy, oracle, base, ("join", left, right, mode, cols))
    if expected is None:
        return
    assert_table_eq_unordered(out, hy.load_table(tbl(expected), 1))


def test_oracle_radix_bits_golden(oracle):
    assert oracle.radix_bits(15_000_000, 4) == 13
    assert oracle.radix_bits(150_000_000, 4) == 16
