"""The headline step through the drop-in operators (`python bench.py --through-operators`): what a Hyrise process
linking the library executes - TableScan::_on_execute then JoinHash::_on_execute (csrc/host/operators.cpp, the
reference constructors and output tables), not the C-ABI directly.

One step (SF --sf, chunks of --chunk rows, l_quantity dictionary-encoded, keys unencoded - the same database as the
C-ABI bench):
    scan = TableScan(lineitem, l_quantity < 24)        -> reference table, one lazy PosList per input chunk
    join = JoinHash(orders, scan, Inner, o_orderkey = l_orderkey)  -> reference table, one chunk per radix partition
and a synchronize of the operator stream (the outputs are produced asynchronously; their PosLists are copied to the
host only when host code reads them). The column chunks' HBM mirrors are created by the warmup steps, as they would be
by the first query over the tables. Rows/s counts the base rows consumed, as the C-ABI bench does.
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def main_operators(args):
    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    hy = importlib.import_module("hyrise-1_amd")
    synth = importlib.import_module("hyrise-1_amd.synth")
    torch.cuda.set_device(0)
    chunk = args.chunk
    okey, lines = synth.orders_numpy(args.sf)
    lkey, qty = synth.lineitem_numpy(okey, lines)
    del lines
    t0 = time.perf_counter()
    orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False)], [okey], [], chunk)
    lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, False), ("l_quantity", hy.DataType.Float, False)],
                                    [lkey, qty.astype(np.float32)], [], chunk)
    n_ord, n_li = len(okey), len(lkey)
    # kept for the output check (sampled partitions against the keys and the predicate)
    okey_h, lkey_h, qty_h = okey, lkey, qty.astype(np.int8)
    expected_matches = int(np.count_nonzero(qty < 24))
    del okey, lkey, qty
    hy.encode_columns(lineitem, [1], hy.EncodingType.Dictionary)
    setup_s = time.perf_counter() - t0
    print(f"operators: tables built and encoded in {setup_s:.1f} s", file=sys.stderr, flush=True)
    o, l = hy.TableWrapper(orders), hy.TableWrapper(lineitem)
    o.execute()
    l.execute()

    def step():
        scan = hy.TableScan(l, 1, hy.PredicateCondition.LessThan, 24)
        scan.execute()
        join = hy.JoinHash(o, scan, hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
        join.execute()
        hy.synchronize()
        return scan, join

    for _ in range(args.warmup):
        step()
    times, releases, drains, phases, pool = [], [], [], [], []
    scan = join = None
    hy.op_trace_enable(True)  # every step's operator phase split (host wall time), to attribute any outlier step
    hy.op_trace_take()
    kstats = []
    if getattr(args, "op_kernel_stats", False):  # per-step device time of every kernel (HIP events; no overlap)
        from bench import kernel_stats
        L = hy.capi.lib
    for _ in range(args.steps):
        if getattr(args, "op_kernel_stats", False):
            L.hy_kernel_stats_reset()
            L.hy_kernel_stats_enable(1)
        # the previous step's output tables (65,536 chunks at SF100) are released inside the timed step: the caller
        # drops them (their chunks are destroyed on the library's background thread, Table::~Table); release_ms is
        # that drop alone
        t0 = time.perf_counter()
        scan = join = None
        releases.append(time.perf_counter() - t0)
        scan, join = step()
        times.append(time.perf_counter() - t0)
        if getattr(args, "op_kernel_stats", False):
            L.hy_kernel_stats_enable(0)
            ks = kernel_stats(L)
            kstats.append({"device_ms": round(sum(k["ms_total"] for k in ks.values()), 3),
                           "top": sorted(((round(k["ms_total"], 3), n) for n, k in ks.items()), reverse=True)[:3]})
        # the background release of the previous step's chunks, finished outside the timed step (its CPU time ran
        # beside this step on another core): how long this thread then still waits for it
        t1 = time.perf_counter()
        hy.release_drain()
        drains.append(time.perf_counter() - t1)
        phases.append({f"{op}: {phase}": round(ms, 3) for op, phase, ms in hy.op_trace_take()})
        pool.append([round(b / 2**30, 2) for b in hy.pool_stats()] + [round(hy.device_memory()[0] / 2**30, 2)])
    hy.op_trace_enable(False)
    step_s = sum(times) / len(times)
    out = join.get_output()
    matches = scan.get_output().row_count()
    check = output_check(np, out, matches, expected_matches, okey_h, lkey_h, qty_h, chunk)
    line = {
        "metric": "rows/sec TableScan+JoinHash through the operators (TableScan/JoinHash::_on_execute), "
                  "TPC-H lineitem⋈orders",
        "value": round((n_li + n_ord) / step_s, 1), "unit": "rows/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 3),
        "ms_per_step_runs": [round(t * 1e3, 3) for t in times],
        "release_ms_runs": [round(t * 1e3, 3) for t in releases],
        "release_drain_ms_runs": [round(t * 1e3, 3) for t in drains],
        "phases_ms_runs": phases, "kernel_stats_runs": kstats or None, "pool_reserved_used_device_free_gib_runs": pool, "host_cpu_share": hy.host_cpu_share(),
        "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "int32", "data": "synthetic (seeded counter-based TPC-H-shaped columns)",
        "config": {"workload": "TableScan(l_quantity<24) -> JoinHash(orders, scan) via _on_execute", "sf": args.sf,
                   "lineitem_rows": n_li, "orders_rows": n_ord, "chunk_size": chunk, "scan_matches": matches,
                   "join_pairs": out.row_count(), "join_output_chunks": out.chunk_count(),
                   "setup_s": round(setup_s, 1), "parallelism": "single GPU"},
        "check": check,
    }
    print(json.dumps(line))


def output_check(np, out, matches, expected_matches, okey, lkey, qty, chunk):
    """The last step's outputs: the scan's row count against the predicate on the host columns, the join's pair count
    (every lineitem row has its order: pairs == matches), and 16 output chunks (radix partitions) spread over the
    output read back RowID by RowID - the build row's o_orderkey equals the probe row's l_orderkey, the probe row
    satisfies l_quantity < 24, and the partition's probe rows ascend within each referenced chunk (the join's probe
    order)."""
    ok_scan = matches == expected_matches
    ok_pairs = out.row_count() == expected_matches
    n_chunks = out.chunk_count()
    sample = sorted(set(int(x) for x in np.linspace(0, max(n_chunks - 1, 0), 16))) if n_chunks else []
    bad, pairs = 0, 0
    for c in sample:
        ch = out.get_chunk(c)
        b = ch.get_column(0).pos_list().reshape(-1, 2).astype(np.int64)  # orders RowIDs
        p = ch.get_column(1).pos_list().reshape(-1, 2).astype(np.int64)  # lineitem RowIDs
        brow, prow = b[:, 0] * chunk + b[:, 1], p[:, 0] * chunk + p[:, 1]
        bad += int(np.count_nonzero(okey[brow] != lkey[prow])) + int(np.count_nonzero(qty[prow] >= 24))
        pairs += len(prow)
    status = "ok" if ok_scan and ok_pairs and bad == 0 and pairs > 0 else "FAILED"
    return {"scan_matches": ok_scan, "join_pairs": ok_pairs, "sampled_partitions": len(sample), "pairs_checked": pairs,
            "mismatches": bad, "status": status}
