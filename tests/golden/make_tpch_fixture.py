"""Generates the TPC-H SF0.01 hot-path fixture (run here, where /root/reference exists; the outputs are committed).

1. oracle/_ref/dbgen_driver (the reference's vendored dbgen compiled by `make -C oracle ref`) prints ORDERS and
   LINEITEM exactly as the reference's TpchDbGenerator produces them (tpch_db_generator.cpp:203-236).
2. The columns the hot path touches are stored in tests/golden/tpch_sf0.01.npz (plain arrays, no pickle).
3. Known answers come from SQLite over the same rows, as the reference's own tpch_test.cpp:54-87 checks Hyrise
   against SQLite; queries are the reference texts (tpch_queries.cpp) or their hot-path parts. Written to
   tests/golden/tpch_sf0.01_answers.json.
"""
import json
import os
import sqlite3
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SF = "0.01"


def main():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True, capture_output=True)
    out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "dbgen_driver"), SF], check=True, capture_output=True,
                         text=True).stdout
    customers, orders, lines = [], [], []
    for row in out.splitlines():
        f = row.split("\t")
        if f[0] == "C":
            customers.append((int(f[1]), f[2]))
        elif f[0] == "O":
            orders.append((int(f[1]), int(f[2]), f[3], int(f[4])))
        else:
            lines.append((int(f[1]), float(f[2]), float(f[3]), float(f[4]), float(f[5]), f[6], f[7], f[8]))
    o = list(zip(*orders))
    li = list(zip(*lines))
    c = list(zip(*customers))
    arrays = {
        "c_custkey": np.array(c[0], np.int32), "c_mktsegment": np.array(c[1], "S10"),
        "o_orderkey": np.array(o[0], np.int32), "o_custkey": np.array(o[1], np.int32),
        "o_orderdate": np.array(o[2], "S10"), "o_shippriority": np.array(o[3], np.int32),
        "l_orderkey": np.array(li[0], np.int32), "l_quantity": np.array(li[1], np.float32),
        "l_extendedprice": np.array(li[2], np.float32), "l_discount": np.array(li[3], np.float32),
        "l_tax": np.array(li[4], np.float32), "l_returnflag": np.array(li[5], "S1"),
        "l_linestatus": np.array(li[6], "S1"), "l_shipdate": np.array(li[7], "S10"),
    }
    np.savez_compressed(os.path.join(HERE, "tpch_sf0.01.npz"), **arrays)

    db = sqlite3.connect(":memory:")
    db.execute("CREATE TABLE customer (c_custkey INT, c_mktsegment TEXT)")
    db.executemany("INSERT INTO customer VALUES (?,?)", customers)
    db.execute("CREATE TABLE orders (o_orderkey INT, o_custkey INT, o_orderdate TEXT, o_shippriority INT)")
    db.execute("CREATE TABLE lineitem (l_orderkey INT, l_quantity REAL, l_extendedprice REAL, l_discount REAL, "
               "l_tax REAL, l_returnflag TEXT, l_linestatus TEXT, l_shipdate TEXT)")
    db.executemany("INSERT INTO orders VALUES (?,?,?,?)", orders)
    # float32 values, widened exactly to double as Hyrise's float columns hand them to SQLite
    db.executemany("INSERT INTO lineitem VALUES (?,?,?,?,?,?,?,?)",
                   [(a, float(np.float32(b)), float(np.float32(c)), float(np.float32(d)), float(np.float32(e)), f, g,
                     h) for a, b, c, d, e, f, g, h in lines])
    q = lambda sql: db.execute(sql).fetchall()
    answers = {
        "sf": float(SF),
        "lineitem_rows": len(lines),
        "orders_rows": len(orders),
        "max_o_orderkey": q("SELECT max(o_orderkey) FROM orders")[0][0],
        "scan_l_quantity_lt_24": q("SELECT count(*) FROM lineitem WHERE l_quantity < 24")[0][0],
        "join_lineitem_orders_rows": q("SELECT count(*) FROM lineitem JOIN orders ON l_orderkey = o_orderkey")[0][0],
        "join_scan_lineitem_orders_rows": q("SELECT count(*) FROM lineitem JOIN orders ON l_orderkey = o_orderkey "
                                            "WHERE l_quantity < 24")[0][0],
        # TPC-H 6, reference text tpch_queries.cpp:206-210
        "q6_rows": q("SELECT count(*) FROM lineitem WHERE l_shipdate >= '1994-01-01' AND l_shipdate < '1995-01-01' "
                     "AND l_discount BETWEEN .06 - 0.01 AND .06 + 0.01001 AND l_quantity < 24")[0][0],
        "q6_revenue": q("SELECT sum(l_extendedprice*l_discount) FROM lineitem WHERE l_shipdate >= '1994-01-01' "
                        "AND l_shipdate < '1995-01-01' AND l_discount BETWEEN .06 - 0.01 AND .06 + 0.01001 "
                        "AND l_quantity < 24")[0][0],
        # TPC-H 1 group counts / sums, Hyrise's text filters l_shipdate <= '1998-12-01' (tpch_queries.cpp:36-44)
        "q1": [list(r) for r in q("SELECT l_returnflag, l_linestatus, count(*), sum(l_quantity), sum(l_extendedprice), "
                                  "avg(l_discount) FROM lineitem WHERE l_shipdate <= '1998-12-01' "
                                  "GROUP BY l_returnflag, l_linestatus ORDER BY l_returnflag, l_linestatus")],
        # TPC-H 1 in full (all eight aggregates), reference text tpch_queries.cpp:36-44; the arithmetic runs in SQLite's
        # double over the float32 values, so these pin the device results to a relative tolerance only
        "q1_full": [list(r) for r in q(
            "SELECT l_returnflag, l_linestatus, SUM(l_quantity), SUM(l_extendedprice), "
            "SUM(l_extendedprice*(1-l_discount)), SUM(l_extendedprice*(1-l_discount)*(1+l_tax)), AVG(l_quantity), "
            "AVG(l_extendedprice), AVG(l_discount), COUNT(*) FROM lineitem WHERE l_shipdate <= '1998-12-01' "
            "GROUP BY l_returnflag, l_linestatus ORDER BY l_returnflag, l_linestatus")],
        # TPC-H 3, reference text tpch_queries.cpp:101-106 (all groups, ordered as the query orders them)
        "q3": [list(r) for r in q(
            "SELECT l_orderkey, SUM(l_extendedprice*(1-l_discount)) as revenue, o_orderdate, o_shippriority "
            "FROM customer, orders, lineitem WHERE c_mktsegment = 'BUILDING' AND c_custkey = o_custkey "
            "AND l_orderkey = o_orderkey AND o_orderdate < '1995-03-15' AND l_shipdate > '1995-03-15' "
            "GROUP BY l_orderkey, o_orderdate, o_shippriority ORDER BY revenue DESC, o_orderdate, l_orderkey")],
        "customer_rows": len(customers),
    }
    with open(os.path.join(HERE, "tpch_sf0.01_answers.json"), "w") as fh:
        json.dump(answers, fh, indent=1)
    print(json.dumps(answers, indent=1))


if __name__ == "__main__":
    main()
