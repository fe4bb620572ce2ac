"""TPC-H SF0.01 CUSTOMER / ORDERS / LINEITEM from the committed dbgen fixture (tests/golden/tpch_sf0.01.npz, made by
tests/golden/make_tpch_fixture.py) as host tables with the reference schema types (tpch_db_generator.cpp:20-27:
keys int, money and quantity float, flags and dates strings), chunked by 10,000 rows like tpch_test.cpp:56."""
import json
import os

import numpy as np

from helpers import GOLDEN

CHUNK = 10_000


def answers():
    return json.load(open(os.path.join(GOLDEN, "tpch_sf0.01_answers.json")))


def arrays():
    with np.load(os.path.join(GOLDEN, "tpch_sf0.01.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def tables(hy, encode=True):
    a = arrays()
    S, I, F = hy.DataType.String, hy.DataType.Int, hy.DataType.Float
    dec = lambda x: x.astype(str)
    orders = hy.Table.from_arrays([("o_orderkey", I, False), ("o_custkey", I, False), ("o_orderdate", S, False),
                                   ("o_shippriority", I, False)],
                                  [a["o_orderkey"], a["o_custkey"], dec(a["o_orderdate"]), a["o_shippriority"]], [],
                                  CHUNK)
    lineitem = hy.Table.from_arrays(
        [("l_orderkey", I, False), ("l_quantity", F, False), ("l_extendedprice", F, False), ("l_discount", F, False),
         ("l_tax", F, False), ("l_returnflag", S, False), ("l_linestatus", S, False), ("l_shipdate", S, False)],
        [a["l_orderkey"], a["l_quantity"], a["l_extendedprice"], a["l_discount"], a["l_tax"], dec(a["l_returnflag"]),
         dec(a["l_linestatus"]), dec(a["l_shipdate"])], [], CHUNK)
    if encode:
        hy.encode_all_chunks(lineitem, hy.EncodingType.Dictionary)
        hy.encode_all_chunks(orders, hy.EncodingType.Dictionary)
    return orders, lineitem


def customer_table(hy, encode=True):
    a = arrays()
    customer = hy.Table.from_arrays([("c_custkey", hy.DataType.Int, False), ("c_mktsegment", hy.DataType.String, False)],
                                    [a["c_custkey"], a["c_mktsegment"].astype(str)], [], CHUNK)
    if encode:
        hy.encode_all_chunks(customer, hy.EncodingType.Dictionary)
    return customer


Q1_GROUPBY = [5, 6]
Q1_AGGS = [(1, "Sum"), (2, "Sum"), (3, "Avg"), (None, "Count")]
Q6_SCANS = [(7, "GreaterThanEquals", "1994-01-01"), (7, "LessThan", "1995-01-01"), (3, "GreaterThanEquals", 0.05),
            (3, "LessThanEquals", 0.07001), (1, "LessThan", 24)]
