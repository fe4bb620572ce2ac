"""Aggregate cases of the reference's src/test/operators/aggregate_test.cpp (fixtures of its SetUp, :29-97), as
declarative plans run either through the oracle or through the device operators.

Each case: (name, input, aggregates, groupby, expected .tbl, also run on a reference table (test_output's
test_aggregate_on_reference_table flag, aggregate_test.cpp:99-121)). Aggregates are (column or None, function name).
`input` is a base-table key or a plan ("scan", key, column, condition, value) / ("join", l, r, mode, (lc, rc)).
"""
from helpers import tbl, wrap

BASE = {
    "1_1": ("aggregateoperator/groupby_int_1gb_1agg/input.tbl", 2, False),
    "1_1_null": ("aggregateoperator/groupby_int_1gb_1agg/input_null.tbl", 2, False),
    "1_2": ("aggregateoperator/groupby_int_1gb_2agg/input.tbl", 2, False),
    "2_1": ("aggregateoperator/groupby_int_2gb_1agg/input.tbl", 2, False),
    "2_2": ("aggregateoperator/groupby_int_2gb_2agg/input.tbl", 2, False),
    "2_0_null": ("aggregateoperator/groupby_int_2gb_0agg/input_null.tbl", 2, False),
    "3_1": ("aggregateoperator/groupby_int_3gb_1agg/input.tbl", 2, False),
    "3_0_null": ("aggregateoperator/groupby_int_3gb_0agg/input_null.tbl", 2, False),
    "1_1_string": ("aggregateoperator/groupby_string_1gb_1agg/input.tbl", 2, False),
    "1_1_string_null": ("aggregateoperator/groupby_string_1gb_1agg/input_null.tbl", 2, False),
    "2_0_a": ("aggregateoperator/join_2gb_0agg/input_a.tbl", 2, False),
    "2_0_b": ("aggregateoperator/join_2gb_0agg/input_b.tbl", 2, False),
    "1_1_dict": ("aggregateoperator/groupby_int_1gb_1agg/input.tbl", 2, True),
    "1_1_null_dict": ("aggregateoperator/groupby_int_1gb_1agg/input_null.tbl", 2, True),
}

A = "aggregateoperator/"
CASES = [
    ("CanCountStringColumns", "1_1_string", [(0, "Count")], [0], A + "groupby_string_1gb_1agg/count_str.tbl", True),
    ("SingleAggregateMax", "1_1", [(1, "Max")], [0], A + "groupby_int_1gb_1agg/max.tbl", True),
    ("SingleAggregateMin", "1_1", [(1, "Min")], [0], A + "groupby_int_1gb_1agg/min.tbl", True),
    ("SingleAggregateSum", "1_1", [(1, "Sum")], [0], A + "groupby_int_1gb_1agg/sum.tbl", True),
    ("SingleAggregateAvg", "1_1", [(1, "Avg")], [0], A + "groupby_int_1gb_1agg/avg.tbl", True),
    ("SingleAggregateCount", "1_1", [(1, "Count")], [0], A + "groupby_int_1gb_1agg/count.tbl", True),
    ("SingleAggregateCountDistinct", "1_1", [(1, "CountDistinct")], [0], A + "groupby_int_1gb_1agg/count_distinct.tbl",
     True),
    ("StringSingleAggregateMax", "1_1_string", [(1, "Max")], [0], A + "groupby_string_1gb_1agg/max.tbl", True),
    ("StringSingleAggregateMin", "1_1_string", [(1, "Min")], [0], A + "groupby_string_1gb_1agg/min.tbl", True),
    ("StringSingleAggregateStringMax", "1_1_string", [(0, "Max")], [], A + "groupby_string_1gb_1agg/max_str.tbl", True),
    ("StringSingleAggregateStringMin", "1_1_string", [(0, "Min")], [], A + "groupby_string_1gb_1agg/min_str.tbl", True),
    ("StringSingleAggregateSum", "1_1_string", [(1, "Sum")], [0], A + "groupby_string_1gb_1agg/sum.tbl", True),
    ("StringSingleAggregateAvg", "1_1_string", [(1, "Avg")], [0], A + "groupby_string_1gb_1agg/avg.tbl", True),
    ("StringSingleAggregateCount", "1_1_string", [(1, "Count")], [0], A + "groupby_string_1gb_1agg/count.tbl", True),
    ("DictionarySingleAggregateMax", "1_1_dict", [(1, "Max")], [0], A + "groupby_int_1gb_1agg/max.tbl", True),
    ("DictionarySingleAggregateMin", "1_1_dict", [(1, "Min")], [0], A + "groupby_int_1gb_1agg/min.tbl", True),
    ("DictionarySingleAggregateSum", "1_1_dict", [(1, "Sum")], [0], A + "groupby_int_1gb_1agg/sum.tbl", True),
    ("DictionarySingleAggregateAvg", "1_1_dict", [(1, "Avg")], [0], A + "groupby_int_1gb_1agg/avg.tbl", True),
    ("DictionarySingleAggregateCount", "1_1_dict", [(1, "Count")], [0], A + "groupby_int_1gb_1agg/count.tbl", True),
    ("TwoAggregateAvgMax", "1_2", [(1, "Max"), (2, "Avg")], [0], A + "groupby_int_1gb_2agg/max_avg.tbl", True),
    ("TwoAggregateMinAvg", "1_2", [(1, "Min"), (2, "Avg")], [0], A + "groupby_int_1gb_2agg/min_avg.tbl", True),
    ("TwoAggregateMinMax", "1_2", [(1, "Min"), (2, "Max")], [0], A + "groupby_int_1gb_2agg/min_max.tbl", True),
    ("TwoAggregateAvgAvg", "1_2", [(1, "Avg"), (2, "Avg")], [0], A + "groupby_int_1gb_2agg/avg_avg.tbl", True),
    ("TwoAggregateSumAvg", "1_2", [(1, "Sum"), (2, "Avg")], [0], A + "groupby_int_1gb_2agg/sum_avg.tbl", True),
    ("TwoAggregateSumSum", "1_2", [(1, "Sum"), (2, "Sum")], [0], A + "groupby_int_1gb_2agg/sum_sum.tbl", True),
    ("TwoAggregateSumCount", "1_2", [(1, "Sum"), (2, "Count")], [0], A + "groupby_int_1gb_2agg/sum_count.tbl", True),
    ("TwoGroupbyMax", "2_1", [(2, "Max")], [0, 1], A + "groupby_int_2gb_1agg/max.tbl", True),
    ("TwoGroupbyMin", "2_1", [(2, "Min")], [0, 1], A + "groupby_int_2gb_1agg/min.tbl", True),
    ("TwoGroupbySum", "2_1", [(2, "Sum")], [0, 1], A + "groupby_int_2gb_1agg/sum.tbl", True),
    ("TwoGroupbyAvg", "2_1", [(2, "Avg")], [0, 1], A + "groupby_int_2gb_1agg/avg.tbl", True),
    ("TwoGroupbyCount", "2_1", [(2, "Count")], [0, 1], A + "groupby_int_2gb_1agg/count.tbl", True),
    ("ThreeGroupbyMax", "3_1", [(2, "Max")], [0, 1, 3], A + "groupby_int_3gb_1agg/max.tbl", True),
    ("ThreeGroupbyMin", "3_1", [(2, "Min")], [0, 1, 3], A + "groupby_int_3gb_1agg/min.tbl", True),
    ("ThreeGroupbySum", "3_1", [(2, "Sum")], [0, 1, 3], A + "groupby_int_3gb_1agg/sum.tbl", True),
    ("ThreeGroupbyAvg", "3_1", [(2, "Avg")], [0, 1, 3], A + "groupby_int_3gb_1agg/avg.tbl", True),
    ("ThreeGroupbyCount", "3_1", [(2, "Count")], [0, 1, 3], A + "groupby_int_3gb_1agg/count.tbl", True),
    ("TwoGroupbyAndTwoAggregateMaxAvg", "2_2", [(2, "Max"), (3, "Avg")], [0, 1], A + "groupby_int_2gb_2agg/max_avg.tbl",
     True),
    ("TwoGroupbyAndTwoAggregateMinAvg", "2_2", [(2, "Min"), (3, "Avg")], [0, 1], A + "groupby_int_2gb_2agg/min_avg.tbl",
     True),
    ("TwoGroupbyAndTwoAggregateMinMax", "2_2", [(2, "Min"), (3, "Max")], [0, 1], A + "groupby_int_2gb_2agg/min_max.tbl",
     True),
    ("TwoGroupbyAndTwoAggregateSumAvg", "2_2", [(2, "Sum"), (3, "Avg")], [0, 1], A + "groupby_int_2gb_2agg/sum_avg.tbl",
     True),
    ("TwoGroupbyAndTwoAggregateSumSum", "2_2", [(2, "Sum"), (3, "Sum")], [0, 1], A + "groupby_int_2gb_2agg/sum_sum.tbl",
     True),
    ("TwoGroupbyAndTwoAggregateSumCount", "2_2", [(2, "Sum"), (3, "Count")], [0, 1],
     A + "groupby_int_2gb_2agg/sum_count.tbl", True),
    ("NoGroupbySingleAggregateMax", "1_1", [(1, "Max")], [], A + "0gb_1agg/max.tbl", True),
    ("NoGroupbySingleAggregateMin", "1_1", [(1, "Min")], [], A + "0gb_1agg/min.tbl", True),
    ("NoGroupbySingleAggregateSum", "1_1", [(1, "Sum")], [], A + "0gb_1agg/sum.tbl", True),
    ("NoGroupbySingleAggregateAvg", "1_1", [(1, "Avg")], [], A + "0gb_1agg/avg.tbl", True),
    ("NoGroupbySingleAggregateCount", "1_1", [(1, "Count")], [], A + "0gb_1agg/count.tbl", True),
    ("OneGroupbyAndNoAggregate", "1_1", [], [0], A + "groupby_int_1gb_0agg/result.tbl", True),
    ("TwoGroupbyAndNoAggregate", "1_1", [], [0, 1], A + "groupby_int_2gb_0agg/result.tbl", True),
    ("CanCountStringColumnsWithNull", "1_1_string_null", [(1, "Count")], [0],
     A + "groupby_string_1gb_1agg/count_str_null.tbl", False),
    ("SingleAggregateMaxWithNull", "1_1_null", [(1, "Max")], [0], A + "groupby_int_1gb_1agg/max_null.tbl", False),
    ("SingleAggregateMinWithNull", "1_1_null", [(1, "Min")], [0], A + "groupby_int_1gb_1agg/min_null.tbl", False),
    ("SingleAggregateSumWithNull", "1_1_null", [(1, "Sum")], [0], A + "groupby_int_1gb_1agg/sum_null.tbl", False),
    ("SingleAggregateAvgWithNull", "1_1_null", [(1, "Avg")], [0], A + "groupby_int_1gb_1agg/avg_null.tbl", False),
    ("SingleAggregateCountWithNull", "1_1_null", [(1, "Count")], [0], A + "groupby_int_1gb_1agg/count_null.tbl", False),
    ("OneGroupbyAndNoAggregateWithNull", "1_1_null", [], [0], A + "groupby_int_1gb_0agg/result_null.tbl", False),
    ("OneGroupbyCountStar", "1_1_null", [(None, "Count")], [0], A + "groupby_int_1gb_0agg/count_star.tbl", False),
    ("TwoGroupbyCountStar", "2_0_null", [(None, "Count")], [0, 2], A + "groupby_int_2gb_0agg/count_star.tbl", False),
    ("ThreeGroupbyCountStar", "3_0_null", [(None, "Count")], [0, 2, 3], A + "groupby_int_3gb_0agg/count_star.tbl",
     False),
    ("DictionarySingleAggregateMaxWithNull", "1_1_null_dict", [(1, "Max")], [0], A + "groupby_int_1gb_1agg/max_null.tbl",
     False),
    ("DictionarySingleAggregateMinWithNull", "1_1_null_dict", [(1, "Min")], [0], A + "groupby_int_1gb_1agg/min_null.tbl",
     False),
    ("DictionarySingleAggregateSumWithNull", "1_1_null_dict", [(1, "Sum")], [0], A + "groupby_int_1gb_1agg/sum_null.tbl",
     False),
    ("DictionarySingleAggregateAvgWithNull", "1_1_null_dict", [(1, "Avg")], [0], A + "groupby_int_1gb_1agg/avg_null.tbl",
     False),
    ("DictionarySingleAggregateCountWithNull", "1_1_null_dict", [(1, "Count")], [0],
     A + "groupby_int_1gb_1agg/count_null.tbl", False),
    ("TwoAggregateEmptyTable", ("scan", "1_2", 0, "LessThan", 0), [(1, "Max"), (2, "Count"), (None, "Count")], [],
     A + "0gb_3agg/max_count_count_empty.tbl", True),
    ("TwoAggregateEmptyTableGrouped", ("scan", "1_2", 0, "LessThan", 0), [(1, "Max"), (2, "Count"), (None, "Count")],
     [0], A + "groupby_int_1gb_3agg/max_count_count_empty.tbl", True),
    ("SingleAggregateMaxOnRef", ("scan", "1_1", 0, "LessThan", "100"), [(1, "Max")], [0],
     A + "groupby_int_1gb_1agg/max_filtered.tbl", True),
    ("TwoGroupbyAndTwoAggregateMinAvgOnRef", ("scan", "2_2", 0, "LessThan", "100"), [(2, "Min"), (3, "Avg")], [0, 1],
     A + "groupby_int_2gb_2agg/min_avg_filtered.tbl", True),
    ("TwoGroupbySumOnRef", ("scan", "2_1", 0, "LessThan", "100"), [(2, "Sum")], [0, 1],
     A + "groupby_int_2gb_1agg/sum_filtered.tbl", True),
    ("TwoAggregateSumAvgOnRef", ("scan", "1_2", 0, "LessThan", "100"), [(1, "Sum"), (2, "Avg")], [0],
     A + "groupby_int_1gb_2agg/sum_avg_filtered.tbl", True),
    ("DictionarySingleAggregateMinOnRef", ("scan", "1_1_dict", 0, "LessThan", "100"), [(1, "Min")], [0],
     A + "groupby_int_1gb_1agg/min_filtered.tbl", True),
    ("JoinThenAggregate", ("join", "2_0_a", "2_0_b", "Inner", (0, 0)), [], [0, 3],
     A + "join_2gb_0agg/result.tbl", True),
]
CASE_IDS = [c[0] for c in CASES]
# aggregate_test.cpp CannotSumStringColumns / CannotAvgStringColumns: execute() throws std::logic_error
FAILING = [("CannotSumStringColumns", "1_1_string", [(0, "Sum")], [0]),
           ("CannotAvgStringColumns", "1_1_string", [(0, "Avg")], [0])]


class BaseTables:
    def __init__(self, hy):
        self.hy = hy
        self.tables = {}

    def table(self, key):
        if key not in self.tables:
            name, chunk, encode = BASE[key]
            t = self.hy.load_table(tbl(name), chunk)
            if encode:
                self.hy.encode_all_chunks(t, self.hy.EncodingType.Dictionary)
            self.tables[key] = t
        return self.tables[key]


def agg_defs(hy, aggs):
    return [hy.AggregateColumnDefinition(c, getattr(hy.AggregateFunction, f)) for c, f in aggs]


def input_operator(hy, base, inp):
    """Device-path input operator for a case input (TableScan / JoinHash run on the device)."""
    if isinstance(inp, str):
        return wrap(hy, base.table(inp))
    if inp[0] == "scan":
        _, key, col, cond, value = inp
        op = hy.TableScan(wrap(hy, base.table(key)), col, getattr(hy.PredicateCondition, cond), value)
    else:
        _, l, r, mode, cols = inp
        op = hy.JoinHash(wrap(hy, base.table(l)), wrap(hy, base.table(r)), getattr(hy.JoinMode, mode), cols,
                         hy.PredicateCondition.Equals)
    op.execute()
    return op


def input_table_oracle(hy, oracle, base, inp):
    if isinstance(inp, str):
        return base.table(inp)
    if inp[0] == "scan":
        _, key, col, cond, value = inp
        return oracle.table_scan(base.table(key), col, getattr(hy.PredicateCondition, cond), value, [])
    _, l, r, mode, cols = inp
    out, _ = oracle.join_hash(base.table(l), base.table(r), getattr(hy.JoinMode, mode), cols)
    return out


def reference_input_plan(inp):
    """test_output's second run: the same aggregate on TableScan(in, ColumnID{0}, >=, 0) (aggregate_test.cpp:112-118)."""
    return ("scan_ge0", inp)
