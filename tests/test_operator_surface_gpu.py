"""The drop-in operator surface on the device: prepared-statement parameters and plan copies executed against the
oracle, and operators executing concurrently on several threads (reference abstract_operator.cpp:77-173,
table_scan.cpp:63-78; operators run concurrently on NodeQueueScheduler workers, operator_task.cpp:61-85,
node_queue_scheduler.cpp:92-121). Every output is compared RowID for RowID / value for value with the oracle."""
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from helpers import assert_identical, tbl, wrap

pytestmark = pytest.mark.gpu


def int_int(hy):
    t = hy.load_table(tbl("int_int_shuffled.tbl"), 7)
    hy.encode_chunks(t, [0, 1], hy.EncodingType.Dictionary)
    return wrap(hy, t)


def test_set_parameters_then_execute(hy, oracle):
    """table_scan_test.cpp:632-655's scans, executed: a placeholder scans with the value set_parameters gave it."""
    w = int_int(hy)
    ge = hy.PredicateCondition.GreaterThanEquals
    for value, expected_param in ((4, None), (hy.ParameterID(2), 6)):
        scan = hy.TableScan(w, 0, ge, value)
        scan.set_parameters({3: 5, 2: 6})
        scan.execute()
        exp = oracle.table_scan(w.get_output(), 0, ge, expected_param if expected_param is not None else 4, [])
        assert_identical(scan.get_output(), exp)


def fact_dim(hy, seed, n_fact=40_000, n_dim=3_000, chunk=1_000):
    rng = np.random.default_rng(seed)
    dkey = rng.permutation(np.arange(n_dim, dtype=np.int32) * 3 + 1)
    grp = rng.integers(0, 7, n_dim).astype(np.int32)
    fkey = rng.integers(0, n_dim * 3 + 20, n_fact).astype(np.int32)
    qty = rng.integers(1, 51, n_fact).astype(np.int32)
    val = rng.integers(-1000, 1000, n_fact).astype(np.int32)
    dim = hy.Table.from_arrays([("d_key", hy.DataType.Int, False), ("d_grp", hy.DataType.Int, False)], [dkey, grp],
                               [], chunk)
    fact = hy.Table.from_arrays([("f_key", hy.DataType.Int, False), ("f_qty", hy.DataType.Int, False),
                                 ("f_val", hy.DataType.Int, False)], [fkey, qty, val], [], chunk)
    hy.encode_columns(fact, [1], hy.EncodingType.Dictionary)
    return fact, dim


def plan(hy, fact_op, dim_op, threshold=None):
    scan = hy.TableScan(fact_op, 1, hy.PredicateCondition.LessThan, hy.ParameterID(0))
    join = hy.JoinHash(dim_op, scan, hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
    agg = hy.Aggregate(join, [hy.AggregateColumnDefinition(4, hy.AggregateFunction.Sum),
                              hy.AggregateColumnDefinition(None, hy.AggregateFunction.Count)], [1])
    if threshold is not None:
        agg.set_parameters({0: threshold})
    return scan, join, agg


def check_plan(hy, oracle, fact, dim, threshold, scan, join, agg):
    exp_scan = oracle.table_scan(fact, 1, hy.PredicateCondition.LessThan, threshold, [])
    assert_identical(scan.get_output(), exp_scan)
    exp_join, _ = oracle.join_hash(dim, scan.get_output(), hy.JoinMode.Inner, (0, 0))
    assert_identical(join.get_output(), exp_join)
    exp_agg = oracle.aggregate(join.get_output(), [hy.AggregateColumnDefinition(4, hy.AggregateFunction.Sum),
                                                   hy.AggregateColumnDefinition(None, hy.AggregateFunction.Count)],
                               [1])
    assert_identical(agg.get_output(), exp_agg)


def test_deep_copy_then_execute(hy, oracle):
    """A prepared plan copied per execution (the plan cache's deep_copy, abstract_operator.cpp:77-81), each copy given
    its own parameter, executed and compared with the oracle; the prepared plan itself stays unexecuted."""
    fact, dim = fact_dim(hy, 1)
    f, d = wrap(hy, fact), wrap(hy, dim)
    prepared = plan(hy, f, d)[2]  # (the placeholder stays in the prepared plan)
    for threshold in (24, 7, 51):
        agg = prepared.deep_copy()
        agg.set_parameters({0: threshold})
        join = agg.input_left()
        scan = join.input_right()
        for op in (scan.input_left(), join.input_left(), scan, join, agg):  # (the copied TableWrappers run first)
            op.execute()
        check_plan(hy, oracle, fact, dim, threshold, scan, join, agg)
    assert prepared.get_output() is None
    assert prepared.input_left().input_right().right_parameter() == hy.ParameterID(0)


def test_projection_placeholder_executes(hy, oracle):
    w = int_int(hy)
    t = w.get_output()
    p = hy.ParameterExpression(1)
    exprs = [hy.ArithmeticExpression(hy.ArithmeticOperator.Multiplication, hy.PQPColumnExpression.from_table(t, 1), p)]
    proj = hy.Projection(w, exprs)
    proj.set_parameters({1: ("float", 0.5)})
    proj.execute()
    assert_identical(proj.get_output(), oracle.projection(t, exprs))


def test_concurrent_operators(hy, oracle):
    """4 threads, each running TableScan -> JoinHash -> Aggregate (execute releases the GIL) three times on its own
    tables and three times on one table every thread shares, whose HBM mirrors the threads create concurrently on
    first use. Every output equals the oracle's."""
    shared_fact, shared_dim = fact_dim(hy, 99)
    shared = (shared_fact, shared_dim, wrap(hy, shared_fact), wrap(hy, shared_dim))
    private = []
    for t in range(4):
        fact, dim = fact_dim(hy, 10 + t)
        private.append((fact, dim, wrap(hy, fact), wrap(hy, dim)))
    start = threading.Barrier(4)

    def worker(t):
        start.wait()
        done = []
        for it in range(6):
            fact, dim, f, d = private[t] if it % 2 == 0 else shared
            threshold = 5 + 7 * t + it
            ops = plan(hy, f, d, threshold)
            for op in ops:
                op.execute()
            done.append((fact, dim, threshold, ops))
        return done

    with ThreadPoolExecutor(4) as pool:
        results = [r for fut in [pool.submit(worker, t) for t in range(4)] for r in fut.result()]
    hy.synchronize()
    assert len(results) == 24
    for fact, dim, threshold, (scan, join, agg) in results:
        check_plan(hy, oracle, fact, dim, threshold, scan, join, agg)


@pytest.mark.parametrize("scheduler", ["pool", "inline"])
def test_operators_under_a_job_scheduler(hy, oracle, scheduler):
    """JoinHash's output chunk builders as jobs of a registered host scheduler (scheduler.hpp; join_hash.cpp:139-182
    waits for its JobTasks in CurrentScheduler::wait_for_tasks): a 3-worker pool shared by 4 threads that run
    TableScan -> JoinHash -> Aggregate concurrently (more jobs than workers: every thread's builders queue behind the
    others'), and the inline scheduler (jobs run as they are scheduled). HY_OP_PARTS_PER_JOB=64 (set for the whole
    session by conftest) splits even these small joins into several jobs. Every output equals the oracle's."""
    hy.set_job_scheduler(scheduler, 3)
    try:
        private = []
        for t in range(4):
            fact, dim = fact_dim(hy, 40 + t)
            private.append((fact, dim, wrap(hy, fact), wrap(hy, dim)))
        start = threading.Barrier(4)

        def worker(t):
            start.wait()
            done = []
            for it in range(3):
                fact, dim, f, d = private[t]
                threshold = 9 + 5 * t + it
                ops = plan(hy, f, d, threshold)
                for op in ops:
                    op.execute()
                done.append((fact, dim, threshold, ops))
            return done

        with ThreadPoolExecutor(4) as pool:
            results = [r for fut in [pool.submit(worker, t) for t in range(4)] for r in fut.result()]
        hy.synchronize()
        for fact, dim, threshold, (scan, join, agg) in results:
            check_plan(hy, oracle, fact, dim, threshold, scan, join, agg)
    finally:
        hy.set_job_scheduler(None)


def test_concurrent_pos_list_reads(hy, oracle):
    """Host reads of one lazy output PosList from several threads at once copy it down once and all see the same
    RowIDs (PosList::host per-list fetch, types.hpp)."""
    fact, dim = fact_dim(hy, 5, n_fact=200_000, chunk=50_000)
    scan = hy.TableScan(wrap(hy, fact), 1, hy.PredicateCondition.LessThan, 30)
    scan.execute()
    out = scan.get_output()
    columns = [out.get_chunk(c).get_column(0) for c in range(out.chunk_count())]
    with ThreadPoolExecutor(8) as pool:
        lists = list(pool.map(lambda k: columns[k % len(columns)].pos_list(), range(32)))
    exp = oracle.table_scan(fact, 1, hy.PredicateCondition.LessThan, 30, [])
    for k, pl in enumerate(lists):
        assert np.array_equal(pl, exp.get_chunk(k % len(columns)).get_column(0).pos_list())
