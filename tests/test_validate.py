"""Validate (MVCC visibility): oracle pinned to the reference's validate_test.cpp (CPU) and device parity (GPU)."""
import numpy as np
import pytest

from helpers import assert_identical, assert_table_eq_unordered, tbl, wrap


def validate_input(hy):
    """OperatorsValidateTest::SetUp (validate_test.cpp:18-26): every record visible (begin 0, end MAX_COMMIT_ID),
    then RowID{1, 0} deleted at commit id 2."""
    t = hy.load_table(tbl("validate_input.tbl"), 2)
    for c in range(t.chunk_count()):
        n = t.get_chunk(c).size()
        end = np.full(n, hy.MAX_COMMIT_ID, np.uint32)
        if c == 1:
            end[0] = 2
        t.get_chunk(c).set_mvcc_columns(np.zeros(n, np.uint32), np.zeros(n, np.uint32), end)
    return t


def mvcc_table(hy, rng, n, chunk):
    t = hy.Table.from_arrays([("a", hy.DataType.Int, False), ("b", hy.DataType.Int, False)],
                             [np.arange(n, dtype=np.int32), rng.integers(0, 100, n).astype(np.int32)], [None, None],
                             chunk)
    for c in range(t.chunk_count()):
        k = t.get_chunk(c).size()
        tids = np.where(rng.random(k) < 0.2, rng.integers(1, 4, k), 0).astype(np.uint32)
        begin = rng.integers(0, 12, k).astype(np.uint32)
        end = np.where(rng.random(k) < 0.3, rng.integers(0, 12, k), hy.MAX_COMMIT_ID).astype(np.uint32)
        t.get_chunk(c).set_mvcc_columns(tids, begin, end)
    return t


def test_oracle_validate_reference_cases(hy, oracle):
    t = validate_input(hy)
    out = oracle.validate(t, 1, 3)  # SimpleValidate: TransactionContext(1, 3)
    assert_table_eq_unordered(out, hy.load_table(tbl("validate_output_validated.tbl"), 2))
    scanned = oracle.table_scan(t, 0, hy.PredicateCondition.GreaterThanEquals, 2, [])  # ScanValidate
    assert_table_eq_unordered(oracle.validate(scanned, 1, 3),
                              hy.load_table(tbl("validate_output_validated_scanned.tbl"), 2))


def test_oracle_validate_visibility_rule(hy, oracle):
    """own uncommitted insert / past insert / deleted / future insert (docs tx.rst as cited in validate.cpp:17-22)."""
    t = hy.Table([("a", hy.DataType.Int, False)], hy.TableType.Data)
    for i in range(5):
        t.append([i])
    big = hy.MAX_COMMIT_ID
    t.get_chunk(0).set_mvcc_columns(np.array([7, 0, 0, 0, 7], np.uint32), np.array([big, 2, 2, 9, 2], np.uint32),
                                    np.array([big, big, 4, big, big], np.uint32))
    out = oracle.validate(t, 7, 5)
    rows = [r[1] for r in out.get_chunk(0).get_column(0).pos_list()]
    assert rows == [0, 1]  # own insert, past insert; deleted at 4, inserted at 9, own row already committed: invisible


def validate_op(hy, inp, tid, snap):
    """The reference's shape (validate.hpp:18-36): Validate(in) with the transaction's context set on the operator."""
    v = hy.Validate(inp)
    v.set_transaction_context(hy.TransactionContext(tid, snap))
    return v


def test_validate_needs_a_transaction_context(hy):
    """validate.cpp:45-47: without a TransactionContext the operator fails (before any device work)."""
    t = validate_input(hy)
    with pytest.raises(RuntimeError, match="transaction context"):
        hy.Validate(wrap(hy, t)).execute()


def test_aborted_transaction_skips_the_operator(hy):
    """abstract_operator.cpp:32-41: an aborted transaction's operators do not run (no device work); the output
    stays unset."""
    t = validate_input(hy)
    v = hy.Validate(wrap(hy, t))
    ctx = hy.TransactionContext(1, 3)
    ctx.set_aborted()
    v.set_transaction_context(ctx)
    v.execute()
    assert v.get_output() is None


@pytest.mark.gpu
def test_validate_reference_cases(hy, oracle):
    t = validate_input(hy)
    w = wrap(hy, t)
    v = validate_op(hy, w, 1, 3)
    v.execute()
    assert_identical(v.get_output(), oracle.validate(t, 1, 3))
    assert_table_eq_unordered(v.get_output(), hy.load_table(tbl("validate_output_validated.tbl"), 2))
    s = hy.TableScan(w, 0, hy.PredicateCondition.GreaterThanEquals, 2)
    s.execute()
    v2 = validate_op(hy, s, 1, 3)
    v2.execute()
    assert_identical(v2.get_output(), oracle.validate(s.get_output(), 1, 3))
    assert_table_eq_unordered(v2.get_output(), hy.load_table(tbl("validate_output_validated_scanned.tbl"), 2))


@pytest.mark.gpu
def test_validate_synthetic(hy, oracle):
    rng = np.random.default_rng(0x4D564343)
    t = mvcc_table(hy, rng, 200_000, 30_011)
    w = wrap(hy, t)
    for tid, snap in ((1, 0), (2, 5), (3, 11), (9, 20)):
        v = validate_op(hy, w, tid, snap)
        v.execute()
        assert_identical(v.get_output(), oracle.validate(t, tid, snap))
        s = hy.TableScan(w, 1, hy.PredicateCondition.LessThan, 40)
        s.execute()
        v2 = validate_op(hy, s, tid, snap)
        v2.execute()
        assert_identical(v2.get_output(), oracle.validate(s.get_output(), tid, snap))
    no_mvcc = wrap(hy, hy.load_table(tbl("int_float.tbl"), 2))
    with pytest.raises(RuntimeError):
        validate_op(hy, no_mvcc, 1, 1).execute()
