"""JoinHash cases of the reference's join_equi_test.cpp, join_null_test.cpp and join_semi_anti_test.cpp (tables
of join_test.hpp:17-73), as declarative plans run either through the oracle or through the device operators."""
from helpers import tbl, wrap

BASE = {
    "a": ("int_float.tbl", 2, None),
    "b": ("int_float2.tbl", 2, None),
    "c": ("int_string.tbl", 4, None),
    "d": ("string_int.tbl", 3, None),
    "e": ("int_int.tbl", 4, None),
    "f": ("int_int2.tbl", 4, None),
    "g": ("int_int3.tbl", 4, None),
    "h": ("int_int4.tbl", 4, None),
    "i": ("int5.tbl", 1, None),
    "j": ("int3.tbl", 1, None),
    "k": ("int4.tbl", 1, None),
    "l": ("int.tbl", 1, None),
    "m": ("aggregateoperator/groupby_int_1gb_0agg/input_null.tbl", 20, None),
    "n": ("aggregateoperator/groupby_int_1gb_1agg/input_null.tbl", 20, None),
    "o": ("float_zero_precision.tbl", 1, None),
    "p": ("double_zero_precision.tbl", 1, None),
    "q": ("string_numbers.tbl", 1, None),
    "a_dict": ("int_float.tbl", 2, [0, 1]),
    "b_dict": ("int_float2.tbl", 2, [0, 1]),
    "c_dict": ("int_float.tbl", 2, [0]),
    "m_dict": ("aggregateoperator/groupby_int_1gb_0agg/input_null.tbl", 20, [0]),
    "n_dict": ("aggregateoperator/groupby_int_1gb_1agg/input_null.tbl", 20, [0]),
    "a_null": ("int_float_with_null.tbl", 2, None),
    "a_null_dict": ("int_float_with_null.tbl", 2, None),  # join_null_test.cpp:41-44 never encodes it
    "semi_a": ("joinoperators/semi_left.tbl", 2, None),
    "semi_b": ("joinoperators/semi_right.tbl", 2, None),
}


def scan(inp, col, cond, value):
    return ("scan", inp, col, cond, value)


def join(left, right, mode, cols):
    return ("join", left, right, mode, cols)


# (name, left, right, mode, column pair, expected table, needs strings)
CASES = [
    ("LeftJoin", "a", "b", "Left", (0, 0), "joinoperators/int_left_join.tbl"),
    ("InnerJoinIntFloat", "a", "o", "Inner", (0, 0), "joinoperators/int_float_inner.tbl"),
    ("InnerJoinFloatInt", "o", "a", "Inner", (0, 0), "joinoperators/float_int_inner.tbl"),
    ("InnerJoinIntDouble", "a", "p", "Inner", (0, 0), "joinoperators/int_double_inner.tbl"),
    ("InnerJoinDoubleInt", "p", "a", "Inner", (0, 0), "joinoperators/double_int_inner.tbl"),
    ("InnerJoinIntString", "a", "q", "Inner", (0, 0), "joinoperators/int_string_inner.tbl"),
    ("LeftJoinOnString", "c", "d", "Left", (1, 0), "joinoperators/string_left_join.tbl"),
    ("RightJoin", "a", "b", "Right", (0, 0), "joinoperators/int_right_join.tbl"),
    ("OuterJoin", "a", "b", "Outer", (0, 0), None),  # JoinHash is excluded from outer-join expectations
    ("InnerJoin", "a", "b", "Inner", (0, 0), "joinoperators/int_inner_join.tbl"),
    ("InnerJoinOnString", "c", "d", "Inner", (1, 0), "joinoperators/string_inner_join.tbl"),
    ("InnerRefJoin", scan("a", 0, "GreaterThanEquals", 0), scan("b", 0, "GreaterThanEquals", 0), "Inner", (0, 0),
     "joinoperators/int_inner_join.tbl"),
    ("InnerValueDictJoin", "a", "b_dict", "Inner", (0, 0), "joinoperators/int_inner_join.tbl"),
    ("InnerDictValueJoin", "a_dict", "b", "Inner", (0, 0), "joinoperators/int_inner_join.tbl"),
    ("InnerValueDictRefJoin", scan("a", 0, "GreaterThanEquals", 0), scan("b_dict", 0, "GreaterThanEquals", 0), "Inner",
     (0, 0), "joinoperators/int_inner_join.tbl"),
    ("InnerDictValueRefJoin", scan("a_dict", 0, "GreaterThanEquals", 0), scan("b", 0, "GreaterThanEquals", 0), "Inner",
     (0, 0), "joinoperators/int_inner_join.tbl"),
    ("InnerRefJoinFiltered", scan("a", 0, "GreaterThan", 1000), scan("b", 0, "GreaterThanEquals", 0), "Inner", (0, 0),
     "joinoperators/int_inner_join_filtered.tbl"),
    ("InnerDictJoin", "a_dict", "b_dict", "Inner", (0, 0), "joinoperators/int_inner_join.tbl"),
    ("InnerRefDictJoin", scan("a_dict", 0, "GreaterThanEquals", 0), scan("b_dict", 0, "GreaterThanEquals", 0), "Inner",
     (0, 0), "joinoperators/int_inner_join.tbl"),
    ("InnerRefDictJoinFiltered", scan("a_dict", 0, "GreaterThan", 1000), scan("b_dict", 0, "GreaterThanEquals", 0),
     "Inner", (0, 0), "joinoperators/int_inner_join_filtered.tbl"),
    ("InnerJoinBig", "c", "d", "Inner", (0, 1), "joinoperators/int_string_inner_join.tbl"),
    ("InnerRefJoinFilteredBig", scan("c", 0, "GreaterThanEquals", 0), scan("d", 1, "GreaterThanEquals", 6), "Inner",
     (0, 1), "joinoperators/int_string_inner_join_filtered.tbl"),
    ("JoinOnMixedValueAndDictionaryColumns", "c_dict", "b", "Inner", (0, 0), "joinoperators/int_inner_join.tbl"),
    ("JoinOnMixedValueAndReferenceColumns", scan("a", 0, "GreaterThanEquals", 0), "b", "Inner", (0, 0),
     "joinoperators/int_inner_join.tbl"),
    ("MultiJoinOnReferenceLeft",
     join(scan("f", 0, "GreaterThanEquals", 0), scan("g", 0, "GreaterThanEquals", 0), "Inner", (0, 0)),
     scan("h", 0, "GreaterThanEquals", 0), "Inner", (0, 0), "joinoperators/int_inner_multijoin_ref_ref_ref_left.tbl"),
    ("MultiJoinOnReferenceRight", scan("h", 0, "GreaterThanEquals", 0),
     join(scan("f", 0, "GreaterThanEquals", 0), scan("g", 0, "GreaterThanEquals", 0), "Inner", (0, 0)), "Inner", (0, 0),
     "joinoperators/int_inner_multijoin_ref_ref_ref_right.tbl"),
    ("MultiJoinOnReferenceLeftFiltered",
     join(scan("f", 0, "GreaterThan", 6), scan("g", 0, "GreaterThanEquals", 0), "Inner", (0, 0)),
     scan("h", 0, "GreaterThanEquals", 0), "Inner", (0, 0),
     "joinoperators/int_inner_multijoin_ref_ref_ref_left_filtered.tbl"),
    ("MultiJoinOnValue", join("f", "g", "Inner", (0, 0)), "h", "Inner", (0, 0),
     "joinoperators/int_inner_multijoin_val_val_val_left.tbl"),
    ("MultiJoinOnRefOuter", join("f", "g", "Left", (0, 0)), "h", "Inner", (0, 0),
     "joinoperators/int_inner_multijoin_val_val_val_leftouter.tbl"),
    ("MixHashAndNestedLoop", join("f", "g", "Left", (0, 0)), "h", "Inner", (0, 0),
     "joinoperators/int_inner_multijoin_nlj_hash.tbl"),
    ("RightJoinRefColumn", scan("a", 0, "GreaterThanEquals", 0), "b", "Right", (0, 0), "joinoperators/int_right_join.tbl"),
    ("LeftJoinRefColumn", "a", scan("b", 0, "GreaterThanEquals", 0), "Left", (0, 0), "joinoperators/int_left_join.tbl"),
    ("RightJoinEmptyRefColumn", scan("a", 0, "Equals", 0), "b", "Right", (0, 0), "joinoperators/int_join_empty.tbl"),
    ("LeftJoinEmptyRefColumn", "b", scan("b", 0, "Equals", 0), "Left", (0, 0), "joinoperators/int_join_empty_left.tbl"),
    # join_null_test.cpp
    ("InnerJoinWithNull", "a", "a_null", "Inner", (0, 0), "joinoperators/int_float_null_inner.tbl"),
    ("InnerJoinWithNullDict", "a_dict", "a_null_dict", "Inner", (0, 0), "joinoperators/int_float_null_inner.tbl"),
    ("InnerJoinWithNull2", "m", "n", "Inner", (0, 0), "joinoperators/int_inner_join_null.tbl"),
    ("InnerJoinWithNullDict2", "m_dict", "n_dict", "Inner", (0, 0), "joinoperators/int_inner_join_null.tbl"),
    ("InnerJoinWithNullRef2", scan("m", 1, "GreaterThanEquals", 0), scan("n", 1, "GreaterThanEquals", 0), "Inner",
     (0, 0), "joinoperators/int_inner_join_null_ref.tbl"),
    ("LeftJoinWithNullAsOuter", "a_null", "b", "Left", (0, 0), "joinoperators/int_left_join_null.tbl"),
    ("LeftJoinWithNullAsOuterDict", "a_null_dict", "b_dict", "Left", (0, 0), "joinoperators/int_left_join_null.tbl"),
    ("LeftJoinWithNullAsInner", "b", "a_null", "Left", (0, 0), "joinoperators/int_left_join_null_inner.tbl"),
    ("LeftJoinWithNullAsInnerDict", "b_dict", "a_null_dict", "Left", (0, 0),
     "joinoperators/int_left_join_null_inner.tbl"),
    ("RightJoinWithNullAsOuter", "b", "a_null", "Right", (0, 0), "joinoperators/int_right_join_null.tbl"),
    ("RightJoinWithNullAsOuterDict", "b_dict", "a_null_dict", "Right", (0, 0), "joinoperators/int_right_join_null.tbl"),
    ("RightJoinWithNullAsInner", "a_null", "b", "Right", (0, 0), "joinoperators/int_right_join_null_inner.tbl"),
    ("RightJoinWithNullAsInnerDict", "a_null_dict", "b_dict", "Right", (0, 0),
     "joinoperators/int_right_join_null_inner.tbl"),
    # join_semi_anti_test.cpp
    ("SemiJoin", "k", "a", "Semi", (0, 0), "int.tbl"),
    ("SemiJoinRefColumns", scan("k", 0, "GreaterThanEquals", 0), scan("a", 0, "GreaterThanEquals", 0), "Semi", (0, 0),
     "int.tbl"),
    ("SemiJoinBig", "semi_a", "semi_b", "Semi", (0, 0), "joinoperators/semi_result.tbl"),
    ("AntiJoin", "k", "a", "Anti", (0, 0), "joinoperators/anti_int4.tbl"),
    ("AntiJoinRefColumns", scan("k", 0, "GreaterThanEquals", 0), scan("a", 0, "GreaterThanEquals", 0), "Anti", (0, 0),
     "joinoperators/anti_int4.tbl"),
    ("AntiJoinBig", "semi_a", "semi_b", "Anti", (0, 0), "joinoperators/anti_result.tbl"),
]

CASE_IDS = [c[0] for c in CASES]


class BaseTables:
    def __init__(self, hy):
        self.hy = hy
        self._cache = {}

    def table(self, name):
        if name not in self._cache:
            f, chunk, enc = BASE[name]
            t = self.hy.load_table(tbl(f), chunk)
            if enc is not None:
                self.hy.encode_chunks(t, enc, self.hy.EncodingType.Dictionary)
            self._cache[name] = t
        return self._cache[name]


def uses_strings(hy, base, plan):
    if isinstance(plan, str):
        t = base.table(plan)
        return any(t.column_data_type(c) == hy.DataType.String for c in range(t.column_count()))
    if plan[0] == "scan":
        return uses_strings(hy, base, plan[1])
    return uses_strings(hy, base, plan[1]) or uses_strings(hy, base, plan[2])


def join_column_is_string(hy, base, case):
    _, left, right, _, cols, _ = case
    lt, rt = eval_oracle(hy, None, base, left, types_only=True), eval_oracle(hy, None, base, right, types_only=True)
    return lt[cols[0]] == hy.DataType.String or rt[cols[1]] == hy.DataType.String


def eval_oracle(hy, oracle, base, plan, types_only=False):
    if isinstance(plan, str):
        t = base.table(plan)
        return [t.column_data_type(c) for c in range(t.column_count())] if types_only else t
    if plan[0] == "scan":
        if types_only:
            return eval_oracle(hy, oracle, base, plan[1], True)
        inp = eval_oracle(hy, oracle, base, plan[1])
        return oracle.table_scan(inp, plan[2], getattr(hy.PredicateCondition, plan[3]), plan[4], [])
    _, left, right, mode, cols = plan
    if types_only:
        lt, rt = eval_oracle(hy, oracle, base, left, True), eval_oracle(hy, oracle, base, right, True)
        return lt + rt if mode not in ("Semi", "Anti") else lt
    out, _bits = oracle.join_hash(eval_oracle(hy, oracle, base, left), eval_oracle(hy, oracle, base, right),
                                  getattr(hy.JoinMode, mode), cols)
    return out


def eval_device(hy, base, plan):
    """Runs the plan through the device operators; returns the root operator."""
    if isinstance(plan, str):
        return wrap(hy, base.table(plan))
    if plan[0] == "scan":
        op = hy.TableScan(eval_device(hy, base, plan[1]), plan[2], getattr(hy.PredicateCondition, plan[3]), plan[4])
        op.execute()
        return op
    _, left, right, mode, cols = plan
    op = hy.JoinHash(eval_device(hy, base, left), eval_device(hy, base, right), getattr(hy.JoinMode, mode), cols,
                     hy.PredicateCondition.Equals)
    op.execute()
    return op
