"""Timing of the widening rows (IS NULL, column-vs-column, LIKE, Validate, RunLength / FrameOfReference scanned
compressed, SIMD-BP128 dictionaries, unencoded string columns: comparisons, LIKE on value columns, string column
compares) through the drop-in operators on SF10-sized synthetic tables (60M rows in 65,536-row chunks; strings on 6M
rows). Wall time per operator call after warm-up, inputs HBM-resident (device mirrors built in the warm-up);
per-kernel device time comes from running this under `rocprofv3 --kernel-trace --stats`.

    python tools/bench_widen.py [--rows 60000000] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import importlib  # noqa: E402

hy = importlib.import_module("hyrise-1_amd")


def timed(make, steps):
    op = make()
    op.execute()  # warm-up: device mirrors, pools
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        op = make()
        op.execute()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, op.get_output().row_count()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=60_000_000)
    ap.add_argument("--like-rows", type=int, default=6_000_000)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    rng = np.random.default_rng(7)
    n, chunk = args.rows, 65_536
    a = rng.integers(1, 51, n).astype(np.int32)
    b = rng.integers(1, 51, n).astype(np.int32)
    nl = (rng.random(n) < 0.05).astype(np.uint8)
    t = hy.Table.from_arrays([("a", hy.DataType.Int, True), ("b", hy.DataType.Int, False)], [a, b], [nl, None], chunk)
    begin = rng.integers(0, 10, n).astype(np.uint32)
    end = np.where(rng.random(n) < 0.1, rng.integers(0, 10, n), hy.MAX_COMMIT_ID).astype(np.uint32)
    tids = np.zeros(n, np.uint32)
    at = 0
    for c in range(t.chunk_count()):
        k = t.get_chunk(c).size()
        t.get_chunk(c).set_mvcc_columns(tids[at:at + k], begin[at:at + k], end[at:at + k])
        at += k
    w = hy.TableWrapper(t)
    w.execute()
    lines = []

    def report(name, ms, rows_in, rows_out, bytes_per_row):
        line = {"op": name, "rows": rows_in, "matches": rows_out, "ms": round(ms, 3),
                "rows_per_s": rows_in / (ms / 1e3), "alg_GBps_wall": rows_in * bytes_per_row / (ms / 1e3) / 1e9,
                "alg_bytes_per_row": bytes_per_row}
        lines.append(line)
        print(json.dumps(line), flush=True)

    C = hy.PredicateCondition
    ms, m = timed(lambda: hy.TableScan(w, 0, C.IsNull, None), args.steps)
    report("IS NULL (value, int32, 5% NULL)", ms, n, m, 5 + 8 * m / n)
    ms, m = timed(lambda: hy.TableScan(w, 0, C.IsNotNull, None), args.steps)
    report("IS NOT NULL (value, int32)", ms, n, m, 5 + 8 * m / n)
    ms, m = timed(lambda: hy.TableScan(w, 0, C.LessThan, hy.ColumnParameter(1)), args.steps)
    report("a < b (column compare, int32 x int32)", ms, n, m, 9 + 8 * m / n)
    def validate():
        v = hy.Validate(w)
        v.set_transaction_context(hy.TransactionContext(1, 5))
        return v

    ms, m = timed(validate, args.steps)
    report("Validate (data input)", ms, n, m, 12 + 8 * m / n)

    for enc in ("RunLength", "FrameOfReference"):
        te = hy.Table.from_arrays([("a", hy.DataType.Int, False)], [np.sort(a)], [None], chunk)
        hy.encode_all_chunks(te, getattr(hy.EncodingType, enc))
        we = hy.TableWrapper(te)
        we.execute()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s = hy.TableScan(we, 0, C.LessThan, 24)  # first use: upload of the compressed arrays, no decode
        s.execute()
        torch.cuda.synchronize()
        report(f"{enc}: first scan incl. upload of the compressed arrays", (time.perf_counter() - t0) * 1e3, n,
               s.get_output().row_count(), 4)
        per_row = 12 / 60 if enc == "RunLength" else 2  # 50 runs per chunk x 12 B; u16 offsets
        ms, m = timed(lambda: hy.TableScan(we, 0, C.LessThan, 24), args.steps)
        report(f"{enc}: scan a < 24 in compressed form", ms, n, m, per_row + 8 * m / n)

    tb = hy.Table.from_arrays([("a", hy.DataType.Int, False)], [a], [None], chunk)
    hy.encode_all_chunks(tb, hy.EncodingType.Dictionary, hy.VectorCompressionType.SimdBp128)
    wb = hy.TableWrapper(tb)
    wb.execute()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s = hy.TableScan(wb, 0, C.LessThan, 24)  # first use: upload of the packed words + device decode to u8 ids
    s.execute()
    torch.cuda.synchronize()
    report("SIMD-BP128 dictionary: first scan incl. upload + hy_decode_simd_bp128", (time.perf_counter() - t0) * 1e3, n,
           s.get_output().row_count(), 6 / 8 + 1)
    ms, m = timed(lambda: hy.TableScan(wb, 0, C.LessThan, 24), args.steps)
    report("SIMD-BP128 dictionary: scan a < 24 on the id mirror", ms, n, m, 1 + 8 * m / n)

    nl_ = args.like_rows
    words = np.array([f"{p} {q}" for p in ("special", "regular", "pending", "express", "final")
                      for q in ("requests", "deposits", "packages", "accounts", "ideas")], dtype=object)
    strs = words[rng.integers(0, len(words), nl_)]
    ts = hy.Table([("s", hy.DataType.String, False)], hy.TableType.Data, chunk)
    for v in strs:
        ts.append([v])
    hy.encode_all_chunks(ts, hy.EncodingType.Dictionary)
    ws = hy.TableWrapper(ts)
    ws.execute()
    ms, m = timed(lambda: hy.TableScan(ws, 0, C.Like, "%special%requests%"), args.steps)
    report("LIKE '%special%requests%' (dictionary, u8 ids)", ms, nl_, m, 1 + 8 * m / nl_)
    ms, m = timed(lambda: hy.TableScan(ws, 0, C.NotLike, "%final%"), args.steps)
    report("NOT LIKE '%final%' (dictionary, u8 ids)", ms, nl_, m, 1 + 8 * m / nl_)

    # unencoded string columns (packed string arrays in HBM): a row's bytes + its 4-byte offset
    tu = hy.Table([("s", hy.DataType.String, False), ("t", hy.DataType.String, False)], hy.TableType.Data, chunk)
    strs2 = words[rng.integers(0, len(words), nl_)]
    for x, y in zip(strs, strs2):
        tu.append([x, y])
    wu = hy.TableWrapper(tu)
    wu.execute()
    avg = float(np.mean([len(x) for x in strs])) + 4
    for name, cond, v in (("= 'pending ideas'", C.Equals, "pending ideas"), ("< 'final'", C.LessThan, "final"),
                          ("LIKE '%special%requests%'", C.Like, "%special%requests%"),
                          ("LIKE 'reg_lar%'", C.Like, "reg_lar%"), ("NOT LIKE '%final%'", C.NotLike, "%final%")):
        ms, m = timed(lambda: hy.TableScan(wu, 0, cond, v), args.steps)
        report(f"unencoded string {name}", ms, nl_, m, avg + 8 * m / nl_)
    ms, m = timed(lambda: hy.TableScan(wu, 0, C.LessThan, hy.ColumnParameter(1)), args.steps)
    report("s < t (string column compare, unencoded)", ms, nl_, m, 2 * avg + 8 * m / nl_)


if __name__ == "__main__":
    main()
