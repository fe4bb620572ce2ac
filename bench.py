"""Headline benchmark: rows/s of TableScan + JoinHash on TPC-H-shaped lineitem ⋈ orders (BASELINE.json metric).

One step = the reference's query shape, on data already resident in HBM:
    TableScan(lineitem, l_quantity < 24)            dictionary-encoded u8 attribute vectors, 100k-row chunks
    JoinHash(orders, <scan output>, o_orderkey = l_orderkey, Inner)   orders builds (smaller side), the scan's
                                                                       reference table probes
executed as the fused hy_scan_join_hash (the scan predicate runs inside the join's first radix pass; --unfused runs
the two C-ABI calls). Rows per step = |lineitem| + |orders| (base-table rows consumed). Everything runs through the
C-ABI (include/hyrise_amd.h) on buffers owned by torch (device memory only; the C-ABI never sees a torch type).

Multi-GPU (torchrun, one process per GPU): bench_dist.py - strong scaling by default (the SF database split over the
ranks), the scan fused into the distributed JoinHash's exchange partition, 8-byte records over one RCCL all-to-all
per side. --workload q1 / q3: bench_tpch.py (BASELINE.json configs[3] / configs[4] at N=1).
"""
import argparse
import ctypes
import importlib
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--sf", type=float, default=None,
                   help="TPC-H scale factor of the database (strong scaling) or per GPU (--scaling weak)")
    p.add_argument("--scaling", choices=["strong", "weak"], default=None,
                   help="N>1: strong (default; the --sf database split over the ranks, BASELINE.json's metric) or "
                        "weak (--sf per rank)")
    p.add_argument("--chunk", type=int, default=100_000)
    p.add_argument("--cpu-sf", type=float, default=10.0, help="scale factor of the bounded CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (RCCL; one GPU per rank) or gloo (host-staged exchange: rehearsal of N ranks on one GPU)")
    p.add_argument("--transport", choices=["capi", "torch"], default="capi",
                   help="N>1 over RCCL: the library's own communicator (default: hy_join_exchange_counts/records, the "
                        "C++ integration's path; in a torch process it binds torch's RCCL under the same soname) or "
                        "torch's all_to_all_single")
    p.add_argument("--workload", choices=["join", "q1", "q3", "scan", "join-only"], default="join",
                   help="join: the headline TableScan+JoinHash (BASELINE.json metric); q1: BASELINE config 4, "
                        "TPC-H 1 TableScan -> Projection -> Aggregate (8 aggregates) on one GPU; q3: BASELINE config 5 at N=1, "
                        "TPC-H 3 Scan -> Join -> Join -> Projection -> Aggregate (bench_tpch.py); scan: config 2, the "
                        "TableScan l_quantity<24 alone (SF10 default); join-only: config 3, JoinHash lineitem x orders "
                        "over all lineitem rows (SF10 default)")
    p.add_argument("--q1-fused", action="store_true",
                   help="q1: the TableScan fused into the aggregate (hy_agg_input.filter; agg_dense_vec) - the default")
    p.add_argument("--q1-poslist", action="store_true",
                   help="q1: the reference plan shape instead - TableScan to PosLists, the aggregate over them "
                        "(agg_dense_lanes through the RowIDs); A/B")
    p.add_argument("--q1-materialize", action="store_true",
                   help="q1: materialise the two arithmetic expressions with hy_projection before the aggregate "
                        "(the reference's plan shape) instead of evaluating them inside it (A/B)")
    p.add_argument("--op-kernel-stats", action="store_true",
                   help="--through-operators: record every step's per-kernel device time (HIP events)")
    p.add_argument("--through-operators", action="store_true",
                   help="time the headline step through TableScan / JoinHash::_on_execute (the drop-in operators, "
                        "bench_ops.py) instead of the C-ABI")
    p.add_argument("--unfused", action="store_true",
                   help="run TableScan and JoinHash as two C-ABI calls (hy_table_scan_row_ids, hy_join_hash) instead "
                        "of the fused hy_scan_join_hash (A/B of the fusion; single GPU)")
    p.add_argument("--no-plan", action="store_true",
                   help="call hy_scan_join_hash every step instead of executing a prepared plan (hy_scan_join_plan_*, "
                        "which stages the 11,444 chunk / predicate descriptors to HBM once); same kernels, A/B of the "
                        "per-call host staging")
    p.add_argument("--probe-gb", type=float, default=4.0, help="buffer size of the measured HBM roofline probe")
    p.add_argument("--join-trace", default=None,
                   help="debug: after the timed region run one traced step and write per-partition join phase "
                        "durations (us) to this .npz (hy_debug_set_join_trace)")
    args = p.parse_args()
    if args.sf is None:  # BASELINE.json: configs 2 and 3 are quoted at SF10, the others at SF100
        args.sf = 10.0 if args.workload in ("scan", "join-only") else 100.0
    return args


def main():
    args = parse()
    if args.through_operators:
        import bench_ops

        return bench_ops.main_operators(args)
    if args.workload in ("q1", "q3"):
        import bench_tpch

        return bench_tpch.main_q1(args) if args.workload == "q1" else bench_tpch.main_q3(args)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 or os.environ.get("HY_BENCH_DIST"):  # (env: rehearse at N = 1)
        import bench_dist

        return bench_dist.main_distributed(args)
    import torch

    hy = importlib.import_module("hyrise-1_amd")
    synth = importlib.import_module("hyrise-1_amd.synth")
    capi = hy.capi
    L = capi.lib

    world, rank = 1, 0  # N > 1: bench_dist.py
    torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    capi.check(L.hy_set_device(dev.index), "hy_set_device")
    # a stream of our own as torch's current stream (torch's work, the events and every C-ABI launch share it): the
    # prepared plan captures its launches into a hipGraph, which the legacy null stream does not allow
    torch.cuda.set_stream(torch.cuda.Stream())
    stream = torch.cuda.current_stream().cuda_stream
    chunk = args.chunk

    # ---------------- data (resident in HBM before timing) ----------------
    n_ord = synth.n_orders(args.sf)
    okey, lines = synth.orders_torch(args.sf, dev)
    lkey, qty = synth.lineitem_torch(okey, lines)
    del lines
    n_li = lkey.numel()
    vids, present = synth.dictionary_encode_small_domain(qty, chunk, 50)
    del qty
    present_h = present.cpu().numpy()
    n_lchunks = (n_li + chunk - 1) // chunk
    n_ochunks = (n_ord + chunk - 1) // chunk
    # pad buffers so 16-byte vector loads of the last chunk stay in bounds
    def padded(t, mult=64):
        extra = (-t.numel()) % mult
        return torch.cat([t, torch.zeros(extra, dtype=t.dtype, device=t.device)]) if extra else t

    vids = padded(vids.contiguous())
    lkey = padded(lkey.contiguous())
    okey = padded(okey.contiguous())
    torch.cuda.synchronize()

    # ---------------- scan descriptors: l_quantity < 24 on dictionary chunks ----------------
    # search value id = lower_bound(dictionary, 24) = number of distinct values < 24 in the chunk
    # (single_column_table_scan_impl.cpp:145-205: LessThan -> all if INVALID, none if 0, else vid < svid)
    scan_chunks = (capi.ScanChunk * n_lchunks)()
    for c in range(n_lchunks):
        size = min(chunk, n_li - c * chunk)
        dsize = int(present_h[c].sum())
        svid = int(present_h[c, :23].sum())
        sc = scan_chunks[c]
        sc.column.data = vids.data_ptr() + c * chunk
        sc.column.size = size
        sc.column.dictionary_size = dsize
        sc.column.kind = capi.HY_COL_DICT
        sc.column.vid_width = 1
        sc.search_vid = svid
        sc.op = capi.HY_OP_ALL if svid >= dsize else (capi.HY_OP_NONE if svid == 0 else capi.HY_OP_LT)
        sc.out_begin = c * chunk
    sizes = (ctypes.c_uint32 * n_lchunks)(*[min(chunk, n_li - c * chunk) for c in range(n_lchunks)])
    l_base, o_base = 0, 0
    chunk_ids = (ctypes.c_uint32 * n_lchunks)(*range(l_base, l_base + n_lchunks))
    ws_bytes = ctypes.c_size_t(0)
    capi.check(L.hy_table_scan_workspace_size(sizes, n_lchunks, ctypes.byref(ws_bytes)), "scan ws")
    scan_ws = torch.empty(ws_bytes.value, dtype=torch.uint8, device=dev)
    scan_rows = torch.empty(n_li * 2 + 64, dtype=torch.int32, device=dev)  # RowIDs (2 x u32)
    scan_counts = torch.empty(n_lchunks, dtype=torch.int32, device=dev)
    L.hy_table_scan_row_ids.restype = ctypes.c_int
    L.hy_table_scan_row_ids.argtypes = [ctypes.POINTER(capi.ScanChunk), ctypes.c_uint32, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]

    def run_scan():
        capi.check(L.hy_table_scan_row_ids(scan_chunks, n_lchunks, capi.HY_TYPE_FLOAT, None, chunk_ids,
                                           scan_rows.data_ptr(), scan_counts.data_ptr(), scan_ws.data_ptr(),
                                           ws_bytes.value, stream), "hy_table_scan_row_ids")

    # ---------------- join descriptors ----------------
    build_chunks = (capi.JoinChunk * n_ochunks)()
    for c in range(n_ochunks):
        size = min(chunk, n_ord - c * chunk)
        b = build_chunks[c]
        b.column.data = okey.data_ptr() + 4 * c * chunk
        b.column.size = size
        b.column.kind = capi.HY_COL_VALUE
        b.size = size
        b.chunk_id = o_base + c
        b.single_chunk = capi.HY_MIXED_CHUNKS
    referenced = (capi.ColumnChunk * n_lchunks)()
    for c in range(n_lchunks):
        r = referenced[c]
        r.data = lkey.data_ptr() + 4 * c * chunk
        r.size = min(chunk, n_li - c * chunk)
        r.kind = capi.HY_COL_VALUE
    build_side = capi.JoinSide(build_chunks, n_ochunks, capi.HY_TYPE_INT32, None, 0, 0, 0)
    radix_bits = L.hy_join_radix_bits(n_ord, 4)  # join_hash.cpp:640-668
    params = capi.JoinParams(capi.HY_JOIN_INNER, capi.HY_TYPE_INT32, radix_bits, 17)
    n_parts = 1 << radix_bits
    part_begin = torch.empty(n_parts, dtype=torch.int64, device=dev)
    part_count = torch.empty(n_parts, dtype=torch.int32, device=dev)
    state = {}

    import numpy as np
    jc_dtype = np.dtype(capi.JoinChunk)

    def probe_side_from_counts(counts_h):
        # the scan's output table: one chunk (PosList) per input chunk with >= 1 match (table_scan.cpp:99); built with
        # numpy so the host side of a step costs what the C++ operator's loop would, not a Python loop
        nz = np.nonzero(counts_h > 0)[0]
        pchunks = np.zeros(len(nz), jc_dtype)
        pchunks["pos_list"] = scan_rows.data_ptr() + 8 * chunk * nz.astype(np.uint64)
        pchunks["size"] = counts_h[nz]
        pchunks["chunk_id"] = np.arange(len(nz), dtype=np.uint32)
        pchunks["single_chunk"] = nz  # scan output chunk k references lineitem chunk nz[k] only
        side = capi.JoinSide(pchunks.ctypes.data_as(ctypes.POINTER(capi.JoinChunk)), len(nz), capi.HY_TYPE_INT32,
                             referenced, n_lchunks, 1, l_base)
        return side, pchunks, int(counts_h[nz].sum())

    def run_join(counts_h):
        side, keep, n_probe = probe_side_from_counts(counts_h)
        if "ws" not in state:
            wsb = ctypes.c_size_t(0)
            capi.check(L.hy_join_hash_workspace_size(ctypes.byref(build_side), ctypes.byref(side),
                                                     ctypes.byref(params), ctypes.byref(wsb)), "join ws")
            state["ws"] = torch.empty(wsb.value, dtype=torch.uint8, device=dev)
            state["out_b"] = torch.empty(2 * n_probe + 64, dtype=torch.int32, device=dev)
            state["out_p"] = torch.empty(2 * n_probe + 64, dtype=torch.int32, device=dev)
            state["cap"] = n_probe
        res = capi.JoinResult()
        capi.check(L.hy_join_hash(ctypes.byref(build_side), ctypes.byref(side), ctypes.byref(params),
                                  state["out_b"].data_ptr(), state["out_p"].data_ptr(), state["cap"],
                                  part_begin.data_ptr(), part_count.data_ptr(), ctypes.byref(res),
                                  state["ws"].data_ptr(), state["ws"].numel(), stream), "hy_join_hash")
        return n_probe, res.total_pairs

    # ---------------- fused TableScan -> JoinHash (hy_scan_join_hash): the scan predicate runs inside the join's
    # first radix pass over lineitem's chunks; the scan output (per-chunk offset lists) is written by the same pass ----
    probe_chunks = (capi.JoinChunk * n_lchunks)()
    for c in range(n_lchunks):
        pc = probe_chunks[c]
        pc.column = referenced[c]
        pc.size = referenced[c].size
        pc.chunk_id = l_base + c
        pc.single_chunk = capi.HY_MIXED_CHUNKS
    probe_data_side = capi.JoinSide(probe_chunks, n_lchunks, capi.HY_TYPE_INT32, None, 0, 0, 0)
    scan_off = torch.empty(n_li + 64, dtype=torch.int32, device=dev)
    scan_begin = torch.zeros(n_lchunks + 1, dtype=torch.int64, device=dev)
    pfilter = capi.JoinFilter(scan_chunks, capi.HY_TYPE_FLOAT, None, scan_off.data_ptr(), scan_begin.data_ptr())

    def run_fused_plan():
        # the prepared plan (hy_scan_join_plan_*): the same kernels as hy_scan_join_hash, descriptors staged once
        if "plan" not in state:
            plan = ctypes.c_void_p()
            capi.check(L.hy_scan_join_plan_create(ctypes.byref(build_side), None, ctypes.byref(probe_data_side),
                                                  ctypes.byref(pfilter), ctypes.byref(params), ctypes.byref(plan)),
                       "hy_scan_join_plan_create")
            state["plan"] = plan
            state["fcap"] = n_li + 64
            state["fout_b"] = torch.empty(2 * state["fcap"], dtype=torch.int32, device=dev)
            state["fout_p"] = torch.empty(2 * state["fcap"], dtype=torch.int32, device=dev)
        res = capi.JoinResult()
        st = L.hy_scan_join_plan_execute(state["plan"], state["fout_b"].data_ptr(), state["fout_p"].data_ptr(),
                                         state["fcap"], part_begin.data_ptr(), part_count.data_ptr(), ctypes.byref(res),
                                         stream)
        if st == capi.HY_ERR_CAPACITY:
            state["fcap"] = res.capacity_required + 64
            state["fout_b"] = torch.empty(2 * state["fcap"], dtype=torch.int32, device=dev)
            state["fout_p"] = torch.empty(2 * state["fcap"], dtype=torch.int32, device=dev)
            return run_fused_plan()
        capi.check(st, "hy_scan_join_plan_execute")
        return res.total_pairs

    def run_fused():
        if not args.no_plan:
            return run_fused_plan()
        if "fws" not in state:
            wsb = ctypes.c_size_t(0)
            capi.check(L.hy_scan_join_hash_workspace_size(ctypes.byref(build_side), None, ctypes.byref(probe_data_side),
                                                          ctypes.byref(pfilter), ctypes.byref(params),
                                                          ctypes.byref(wsb)), "fused ws")
            state["fws"] = torch.empty(wsb.value, dtype=torch.uint8, device=dev)
            state["fcap"] = n_li + 64  # pairs <= probe rows for the unique orders keys; HY_ERR_CAPACITY grows it
            state["fout_b"] = torch.empty(2 * state["fcap"], dtype=torch.int32, device=dev)
            state["fout_p"] = torch.empty(2 * state["fcap"], dtype=torch.int32, device=dev)
        res = capi.JoinResult()
        st = L.hy_scan_join_hash(ctypes.byref(build_side), None, ctypes.byref(probe_data_side), ctypes.byref(pfilter),
                                 ctypes.byref(params), state["fout_b"].data_ptr(), state["fout_p"].data_ptr(),
                                 state["fcap"], part_begin.data_ptr(), part_count.data_ptr(), ctypes.byref(res),
                                 state["fws"].data_ptr(), state["fws"].numel(), stream)
        if st == capi.HY_ERR_CAPACITY:
            state["fcap"] = res.capacity_required + 64
            state["fout_b"] = torch.empty(2 * state["fcap"], dtype=torch.int32, device=dev)
            state["fout_p"] = torch.empty(2 * state["fcap"], dtype=torch.int32, device=dev)
            return run_fused()
        capi.check(st, "hy_scan_join_hash")
        return res.total_pairs

    fused = not args.unfused and args.workload == "join"
    mode = args.workload  # "join" (headline), "scan" (config 2) or "join-only" (config 3)

    def run_join_only():
        # JoinHash lineitem ⋈ orders over every lineitem row (BASELINE.json configs[2]): data tables on both sides
        if "jws" not in state:
            wsb = ctypes.c_size_t(0)
            capi.check(L.hy_join_hash_workspace_size(ctypes.byref(build_side), ctypes.byref(probe_data_side),
                                                     ctypes.byref(params), ctypes.byref(wsb)), "join ws")
            state["jws"] = torch.empty(wsb.value, dtype=torch.uint8, device=dev)
            state["jcap"] = n_li + 64
            state["jout_b"] = torch.empty(2 * state["jcap"], dtype=torch.int32, device=dev)
            state["jout_p"] = torch.empty(2 * state["jcap"], dtype=torch.int32, device=dev)
        res = capi.JoinResult()
        capi.check(L.hy_join_hash(ctypes.byref(build_side), ctypes.byref(probe_data_side), ctypes.byref(params),
                                  state["jout_b"].data_ptr(), state["jout_p"].data_ptr(), state["jcap"],
                                  part_begin.data_ptr(), part_count.data_ptr(), ctypes.byref(res),
                                  state["jws"].data_ptr(), state["jws"].numel(), stream), "hy_join_hash")
        return n_li, res.total_pairs

    def step():
        if mode == "scan":  # the TableScan operator's step: RowIDs + per-chunk match counts to the host
            run_scan()
            return int(scan_counts.cpu().numpy().astype(np.int64).sum()), 0
        if mode == "join-only":
            return run_join_only()
        if fused:
            pairs = run_fused()
            return None, pairs  # scan matches are read once after the timed region (scan_begin[-1])
        run_scan()
        counts_h = scan_counts.cpu().numpy()  # D2H of per-chunk match counts (the output chunk layout)
        return run_join(counts_h)

    for _ in range(args.warmup):
        n_probe, pairs = step()
    torch.cuda.synchronize()

    # ---------------- timed region (per-kernel HIP-event timing off: its event records would sit in the step) -------
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n_probe, pairs = step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-kernel device times: the same K steps again with HIP events on the launch stream around every kernel
    L.hy_kernel_stats_reset()
    L.hy_kernel_stats_enable(1)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    L.hy_kernel_stats_enable(0)
    if fused:
        n_probe = int(scan_begin[-1].item())
    if args.join_trace:
        import numpy as np
        trace = torch.zeros(5 * (1 << radix_bits), dtype=torch.int64, device=dev)
        L.hy_debug_set_join_trace.argtypes = [ctypes.c_void_p]
        L.hy_debug_set_join_trace(trace.data_ptr())
        step()
        torch.cuda.synchronize()
        L.hy_debug_set_join_trace(None)
        t = trace.view(-1, 5).cpu().numpy().astype(np.float64) / 100.0  # 100 MHz device clock -> us
        np.savez(args.join_trace, stamps_us=t, out_pairs=part_count.cpu().numpy())
    g_li, g_ord, g_probe, g_pairs = n_li, n_ord, n_probe, int(pairs)
    check = None
    if mode == "scan":  # config 2: every chunk's count and every RowID of the timed step's output
        thr = [256 if scan_chunks[c].op == capi.HY_OP_ALL else (0 if scan_chunks[c].op == capi.HY_OP_NONE
               else scan_chunks[c].search_vid) for c in range(n_lchunks)]
        check = verify_scan(torch, chunk, vids, n_li, thr, scan_rows, scan_counts)
        if check["status"] != "ok":
            raise SystemExit(f"scan output check failed: {check}")
    if mode == "join-only":  # config 3: the headline's join properties with every lineitem row as a probe row
        check = verify_headline(torch, L, stream, chunk, okey, lkey, vids, n_li, [256] * n_lchunks,
                                (state["jout_b"], state["jout_p"], None, None), part_begin, part_count, radix_bits,
                                g_pairs)
        if check["status"] != "ok":
            raise SystemExit(f"join-only output check failed: {check}")
    if mode == "join":  # pin the timed output at its full size (every pair, partition and scan offset)
        thr = []
        for c in range(n_lchunks):
            op_ = scan_chunks[c].op
            thr.append(256 if op_ == capi.HY_OP_ALL else (0 if op_ == capi.HY_OP_NONE else scan_chunks[c].search_vid))
        if fused:
            outs = (state["fout_b"], state["fout_p"], scan_off, scan_begin)
        else:
            outs = (state["out_b"], state["out_p"], None, None)
        check = verify_headline(torch, L, stream, chunk, okey, lkey, vids, n_li, thr, outs, part_begin, part_count,
                                radix_bits, g_pairs)
        if check["status"] != "ok":
            raise SystemExit(f"headline output check failed: {check}")

    # ---------------- per-kernel device time (HIP events on the launch stream) ----------------
    nk = ctypes.c_uint32(0)
    L.hy_kernel_stats_collect(ctypes.byref(nk))
    L.hy_kernel_stats_get.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
    kernels = {}
    for i in range(nk.value):
        name, launches, total, units = ctypes.c_char_p(), ctypes.c_uint64(), ctypes.c_double(), ctypes.c_uint64()
        L.hy_kernel_stats_get(i, ctypes.byref(name), ctypes.byref(launches), ctypes.byref(total), ctypes.byref(units))
        kernels[name.value.decode()] = {"launches": launches.value, "ms_total": total.value}

    K = args.steps
    # algorithmic bytes: scan 1 B/row read + 4 B/match written (chunk offsets; 8 B RowIDs on the
    # unfused path); JoinHash 4 B/build row + 4 B/probe row read + 16 B/pair written. Partition passes are overhead:
    # for them the table lists the bytes each kernel must move (records 8 B, digit bytes 1 B), not algorithmic bytes.
    recv_build, recv_probe = n_ord, n_probe
    scan_out_b = 4 if fused else 8
    e2e_bytes = n_li * 1 + n_probe * scan_out_b + n_ord * 4 + n_probe * 4 + int(pairs) * 16
    if mode == "scan":
        e2e_bytes = n_li * 1 + n_probe * 8  # u8 value ids read, 8-byte RowIDs written
    elif mode == "join-only":
        e2e_bytes = n_ord * 4 + n_li * 4 + int(pairs) * 16
    if fused and "part1_mask.probe" in kernels:  # match-bit pass (HY_FILTER_COMPACT=0)
        moved = {
            "part1_mask.probe": n_li * 5 + n_li // 8,  # predicate ids + keys read, one match bit per row written
            "part1_spread.probe": n_li * 4 + n_li // 8 + n_probe * (8 + 4 + 1),  # keys + bits; records, offsets, digit
            "part2_hist.probe": n_probe * 1,
            "part2_scatter.probe": n_probe * 16,
        }
    elif fused:  # compact -> spread (default)
        moved = {
            "part1_compact.probe": n_li * 5 + n_probe * 8,
            "part1_spread.probe": n_probe * 8 + n_probe * (8 + 4 + 1),
            "part2_hist.probe": n_probe * 1,
            "part2_scatter.probe": n_probe * 16,
        }
    else:
        moved = {
            "scan_dict": n_li * 1 + n_probe * 8,
            "part1_hist.probe": n_probe * (8 + 4),
            "part1_scatter.probe": n_probe * (8 + 4 + 8),
            "part2_hist.probe": n_probe * 8,
            "part2_scatter.probe": n_probe * 16,
        }
    if mode == "scan":
        moved = {"scan_dict": n_li * 1 + n_probe * 8}
    elif mode == "join-only":
        moved = {"part1_hist.probe": n_li * 4, "part1_scatter.probe": n_li * (4 + 8 + 1),
                 "part2_hist.probe": n_li * 1, "part2_scatter.probe": n_li * 16}
    moved.update({
        "part1_hist.build": n_ord * 4,
        "part1_scatter.build": n_ord * (4 + 8 + 1),
        "part2_hist.build": n_ord * (1 if fused else 8),
        "part2_scatter.build": n_ord * 16,
        # the join kernel's algorithmic bytes exactly as 8(d) counts JoinHash
        "join_partition": recv_build * 4 + recv_probe * 4 + int(pairs) * 16,
    })
    # the partition join is join_partition plus the list kernels it defers partitions to (more probe records than one
    # pass, more build rows than one LDS table): one logical kernel for the roofline, launched once per step
    deferred = [k for k in ("join_partition_multi", "join_partition_skewed") if k in kernels]
    if "join_partition" in kernels and deferred:
        jp = kernels["join_partition"]
        jp["includes"] = {k: round(kernels[k]["ms_total"] / max(kernels[k]["launches"], 1), 4) for k in deferred}
        for k in deferred:
            jp["ms_total"] += kernels.pop(k)["ms_total"]
    for k, v in kernels.items():
        per_launch_ms = v["ms_total"] / max(v["launches"], 1)
        v["ms_per_launch"] = per_launch_ms
        if k in moved:
            launches_per_step = v["launches"] / K
            v["bytes_per_launch"] = moved[k] / launches_per_step
            v["achieved_GBps"] = v["bytes_per_launch"] / (per_launch_ms * 1e-3) / 1e9
    step_s = elapsed / K
    value = (g_li + (0 if mode == "scan" else g_ord)) / step_s
    peak, probe = measured_roofline(L, capi, torch, dev, stream, args.probe_gb)
    dom = max((k for k in kernels if k in moved), key=lambda k: kernels[k]["ms_total"])
    dk = kernels[dom]
    e2e_gbps = e2e_bytes / step_s / 1e9
    # SURVEY 8(d) asks for both fractions: the read side alone (column bytes in) and read + write
    e2e_read = n_li * 1 + n_ord * 4 + n_probe * 4
    if mode == "scan":
        e2e_read = n_li * 1
    elif mode == "join-only":
        e2e_read = n_ord * 4 + n_li * 4
    # headline roofline: the whole step's algorithmic bytes over its time, against the HBM bandwidth measured in this
    # run; the dominant kernel's own line follows (its rocprofv3 average is in profiles/)
    roofline = {"bound": "hbm", "scope": "end-to-end step (TableScan + JoinHash, algorithmic bytes of SURVEY 8(d))",
                "achieved": round(e2e_gbps, 1), "peak": round(peak, 1), "unit": "GB/s",
                "frac": round(e2e_gbps / peak, 4), "alg_bytes_per_step": e2e_bytes, "traffic": None,
                "frac_read_only": round(e2e_read / step_s / 1e9 / peak, 4), "alg_read_bytes_per_step": e2e_read,
                "peak_source": "measured in this run (hy_stream_bandwidth_probe, best of read / copy)",
                "frac_of_spec_8000": round(e2e_gbps / HBM_PEAK_GBPS, 4)}
    traffic, traffic_src = committed_traffic_step(args.sf, chunk, world, fused, mode)
    if traffic is not None:
        roofline["traffic"] = round(traffic)
        roofline["traffic_source"] = traffic_src
    # the contract's `roofline`: the dominant kernel among those whose bytes SURVEY 8(d) defines (join_partition =
    # JoinHash: 4 B/build row + 4 B/probe row + 16 B/pair; scan_dict = TableScan), algorithmic bytes per launch over
    # its average launch duration (HIP events on its stream, a timing pass outside the timed region), against the
    # MI355X spec peak (MI355X_MICROARCH.md); traffic = its PMC bytes per launch from the committed rocprofv3 summary
    alg_kernels = [k for k in ("join_partition", "scan_dict") if k in kernels and "achieved_GBps" in kernels[k]]
    adom = max(alg_kernels, key=lambda k: kernels[k]["ms_total"]) if alg_kernels else dom
    ak = kernels[adom]
    k_traffic, k_src = committed_traffic(adom, args.sf, chunk, world, mode, fused)
    kernel_roofline = {"bound": "hbm", "kernel": adom, "achieved": round(ak["achieved_GBps"], 1),
                       "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(ak["achieved_GBps"] / HBM_PEAK_GBPS, 4),
                       "traffic": round(k_traffic) if k_traffic is not None else None,
                       "traffic_source": k_src, "ms_per_launch": round(ak["ms_per_launch"], 4),
                       "bytes_per_launch": ak["bytes_per_launch"], "peak_measured": round(peak, 1),
                       "frac_of_measured_peak": round(ak["achieved_GBps"] / peak, 4),
                       "peak_source": "MI355X_MICROARCH.md HBM3E spec; peak_measured: this run's stream probe"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # (config 3's sample is half the scale factor: its join takes every lineitem row, ~2x the headline's)
        cpu = cpu_baseline(hy, synth, args.cpu_sf / (2 if mode == "join-only" else 1), chunk, mode=mode)

    if rank == 0:
        line = {
            "metric": "rows/sec TableScan+JoinHash, TPC-H SF100 lineitem⋈orders, 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling or "strong",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded counter-based TPC-H-shaped columns, resident in HBM)",
            "config": {"workload": f"TableScan(l_quantity<24, dictionary u8) -> JoinHash(orders ⋈ scan, "
                                   f"o_orderkey=l_orderkey, radix_bits={radix_bits})",
                       "path": ("fused hy_scan_join_hash" + ("" if args.no_plan else " (prepared plan)")) if fused
                       else "hy_table_scan_row_ids + hy_join_hash",
                       "sf_total": args.sf, "lineitem_rows": g_li, "orders_rows": g_ord, "chunk_size": chunk,
                       "scan_matches": g_probe, "join_pairs": g_pairs,
                       "parallelism": "single GPU"},
            "roofline": kernel_roofline,
            "roofline_e2e": roofline,
            "hbm_probe": probe,
            "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in kernels.items()},
            "cpu_baseline": cpu,
            "check": check,
        }
        if mode == "scan":  # BASELINE.json configs[1]
            line["metric"] = "rows/sec TableScan lineitem.l_quantity<24, dictionary-encoded, one MI355X"
            line["config"] = {"workload": "TableScan(l_quantity<24, dictionary u8) alone (BASELINE.json configs[1])",
                              "path": "hy_table_scan_row_ids + per-chunk counts to the host", "sf": args.sf,
                              "lineitem_rows": g_li, "chunk_size": chunk, "scan_matches": g_probe,
                              "parallelism": "single GPU"}
            line["roofline_e2e"]["scope"] = "TableScan step (1 B/row value ids read + 8 B/match RowIDs written)"
        elif mode == "join-only":  # BASELINE.json configs[2]
            line["metric"] = "rows/sec JoinHash lineitem⋈orders on l_orderkey, one MI355X"
            line["config"] = {"workload": f"JoinHash(orders ⋈ lineitem, o_orderkey=l_orderkey, radix_bits={radix_bits}) "
                                          f"over every lineitem row (BASELINE.json configs[2])",
                              "path": "hy_join_hash (data tables on both sides)", "sf": args.sf,
                              "lineitem_rows": g_li, "orders_rows": g_ord, "chunk_size": chunk, "join_pairs": g_pairs,
                              "parallelism": "single GPU"}
            line["roofline_e2e"]["scope"] = "JoinHash step (SURVEY 8(d): 4 B/build row + 4 B/probe row + 16 B/pair)"
        print(json.dumps(line))


def verify_scan(torch, chunk, vids, n_li, thr, scan_rows, scan_counts):
    """Config 2's TableScan output at its full size: per chunk the match count, and every RowID {chunk, offset} of the
    matches (vid < search value id of their chunk, single_column_table_scan_impl.cpp:145-205) in row order, chunk c's
    written from c * chunk on (its out_begin)."""
    dev = vids.device
    n_chunks = len(thr)
    sizes = torch.tensor([min(chunk, n_li - c * chunk) for c in range(n_chunks)], dtype=torch.int64, device=dev)
    t = torch.repeat_interleave(torch.tensor(thr, dtype=torch.int32, device=dev), sizes)
    match = torch.nonzero(vids[:n_li].to(torch.int32) < t).flatten()
    del t
    c = match // chunk
    first = torch.searchsorted(match, torch.arange(0, n_li, chunk, device=dev))
    counts = torch.diff(torch.cat([first, torch.tensor([match.numel()], device=dev)]))
    res = {"chunk_counts": bool(torch.equal(scan_counts[:n_chunks].to(torch.int64), counts))}
    pos = c * chunk + (torch.arange(match.numel(), device=dev) - first[c])
    rows = scan_rows.view(-1, 2)[pos].to(torch.int64)
    res["row_ids"] = bool(torch.equal(rows[:, 0], c) and torch.equal(rows[:, 1], match % chunk))
    res["status"] = "ok" if all(res.values()) else "MISMATCH"
    res["matches_checked"] = int(match.numel())
    return res


def verify_headline(torch, L, stream, chunk, okey, lkey, vids, n_li, thr, outs, part_begin, part_count, bits, pairs):
    """Checks the timed step's output at its full size on the device (after the timed region). For an INNER join with
    unique build keys these properties determine the reference's output exactly (join_hash.cpp:362-455, 829-855):
      * every pair's o_orderkey[build RowID] == l_orderkey[probe RowID];
      * the probe rows of all pairs are exactly the scan matches (every lineitem row's order exists);
      * partition p's range holds only probe keys with murmur2(key, 17) & (2^bits - 1) == p;
      * probe RowIDs ascend within each partition (the reference's probe order);
      * the partitions' ranges tile the output buffer without gaps or overlap;
      * fused path: the scan output offsets are the rows with vid < search_vid of their chunk (table_scan.cpp:78-164,
        single_column_table_scan_impl.cpp:145-205), chunk by chunk."""
    dev = okey.device
    ob_t, op_t, scan_off, scan_begin = outs
    ob = ob_t[: 2 * pairs].view(-1, 2).to(torch.int64)
    op = op_t[: 2 * pairs].view(-1, 2).to(torch.int64)
    bidx = ob[:, 0] * chunk + ob[:, 1]
    pidx = op[:, 0] * chunk + op[:, 1]
    del ob, op
    res = {}
    res["keys_equal"] = bool(torch.equal(okey[bidx], lkey[pidx]))
    del bidx
    sizes = torch.tensor([min(chunk, n_li - c * chunk) for c in range(len(thr))], dtype=torch.int64, device=dev)
    t = torch.repeat_interleave(torch.tensor(thr, dtype=torch.int32, device=dev), sizes)
    match = torch.nonzero(vids[:n_li].to(torch.int32) < t).flatten()
    del t
    res["probe_rows_are_scan_matches"] = bool(match.numel() == pairs and torch.equal(torch.sort(pidx).values, match))
    if scan_off is not None:
        n_m = int(scan_begin[-1].item())
        res["scan_offsets"] = bool(n_m == match.numel() and
                                   torch.equal(scan_off[:n_m].to(torch.int64), match % chunk))
        starts = torch.searchsorted(match, torch.arange(0, n_li, chunk, device=dev))
        res["scan_chunk_begins"] = bool(torch.equal(scan_begin[:-1], starts))
    del match
    n_parts = 1 << bits
    cnt = part_count[:n_parts].to(torch.int64)
    beg = part_begin[:n_parts].to(torch.int64)
    order = torch.argsort(beg[cnt > 0])
    pids = torch.nonzero(cnt > 0).flatten()[order]
    cs = cnt[pids]
    res["ranges_tile_output"] = bool(int(cs.sum()) == pairs and
                                     torch.equal(beg[pids], torch.cumsum(cs, 0) - cs))
    pid = torch.repeat_interleave(pids, cs)  # partition of each output slot
    h = torch.empty(pairs, dtype=torch.int32, device=dev)
    keys = lkey[pidx].contiguous()
    st = L.hy_murmur2(keys.data_ptr(), pairs, 4, 17, h.data_ptr(), stream)
    res["partition_ids"] = bool(st == 0 and torch.equal(h.to(torch.int64) & (n_parts - 1), pid))
    same = pid[1:] == pid[:-1]
    res["probe_order_within_partitions"] = bool(torch.all((pidx[1:] > pidx[:-1]) | ~same))
    torch.cuda.synchronize()
    res["status"] = "ok" if all(v for k, v in res.items()) else "MISMATCH"
    res["pairs_checked"] = pairs
    return res


def kernel_stats(L):
    """Per-kernel launches and total device ms of the timed region (HIP events on the launch stream)."""
    nk = ctypes.c_uint32(0)
    L.hy_kernel_stats_collect(ctypes.byref(nk))
    L.hy_kernel_stats_get.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
    out = {}
    for i in range(nk.value):
        name, launches, total, units = ctypes.c_char_p(), ctypes.c_uint64(), ctypes.c_double(), ctypes.c_uint64()
        L.hy_kernel_stats_get(i, ctypes.byref(name), ctypes.byref(launches), ctypes.byref(total), ctypes.byref(units))
        out[name.value.decode()] = {"launches": launches.value, "ms_total": total.value}
    return out


# bench.py's kernel-table names -> the HIP kernel function names rocprofv3 reports (a list: the kernel-table entry
# times several launches as one - the two-pass TableScan's count and write kernels - and its traffic is their sum;
# older summaries name the one-pass scan_kernel)
ROCPROF_NAME = {"scan_dict": [["scan_count_kernel", "scan_write_kernel"], ["scan_kernel"]],
                "scan_value": [["scan_count_kernel", "scan_write_kernel"], ["scan_kernel"]]}


def summary_files(mode, sf, fused):
    """The committed PMC summaries of one bench configuration, newest round last (tools/profile_round.sh names them
    rNN_rocprof_<workload>_summary.json; FETCH_SIZE x2 + WRITE_SIZE as the MI355X guide prescribes)."""
    here = os.path.dirname(os.path.abspath(__file__))
    if mode == "join":
        pats = [f"r*_rocprof_sf{sf:g}_fused_summary.json"] if fused else [f"r*_rocprof_sf{sf:g}_summary.json"]
    else:
        pats = [f"r*_rocprof_{mode.replace('-', '')}_sf{sf:g}_summary.json"]
    files = [f for pat in pats for f in glob.glob(os.path.join(here, "profiles", pat))]
    return here, sorted(files, key=os.path.basename)


def committed_traffic(kernel, sf, chunk, world, mode="join", fused=True):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary of this configuration. The counters need
    their own rocprofv3 passes, so they are not re-collected here; the summary named in traffic_source is the
    evidence. None if no summary matches (other scale factor or N>1)."""
    if world != 1 or chunk != 100_000:
        return None, None
    here, files = summary_files(mode, sf, fused)
    for f in reversed(files):
        with open(f) as fh:
            ks = json.load(fh).get("kernels", {})
        for names in ROCPROF_NAME.get(kernel, [[kernel]]):
            if all("hbm_bytes_per_launch" in ks.get(n, {}) for n in names):
                return sum(ks[n]["hbm_bytes_per_launch"] for n in names), os.path.relpath(f, here)
    return None, None


def measured_roofline(L, capi, torch, dev, stream, gb):
    """HBM bandwidth measured in this run with the library's streaming read and copy kernels (best of 5 each, 16-B
    nontemporal accesses): the denominator of roofline.frac."""
    n = int(gb * 1e9) // 16 * 16
    src = torch.empty(n // 4, dtype=torch.int32, device=dev).fill_(1)
    dst = torch.empty(n // 4, dtype=torch.int32, device=dev)
    out = {}
    for name, mode, traffic in (("read", capi.HY_PROBE_READ, n), ("copy", capi.HY_PROBE_COPY, 2 * n)):
        best = 0.0
        for _ in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            capi.check(L.hy_stream_bandwidth_probe(src.data_ptr(), dst.data_ptr(), n, mode, stream), "probe")
            e1.record()
            torch.cuda.synchronize()
            best = max(best, traffic / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        out[name + "_GBps"] = round(best, 1)
    del src, dst
    out["bytes"] = n
    return max(out["read_GBps"], out["copy_GBps"]), out


def committed_traffic_step(sf, chunk, world, fused, mode="join"):
    """HBM bytes per step (all kernels) from the newest committed PMC summary of this configuration. None if no
    summary matches."""
    if world != 1 or chunk != 100_000:
        return None, None
    here, files = summary_files(mode, sf, fused)
    for f in reversed(files):
        with open(f) as fh:
            d = json.load(fh)
        if "hbm_bytes_per_step" in d:
            return d["hbm_bytes_per_step"], os.path.relpath(f, here)
    return None, None


def host_cpu():
    """(threads to use, CPU model): the CPUs this process may run on, capped by OMP_NUM_THREADS (the GPU box's share
    of a larger machine)."""
    n = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        n = min(n, int(os.environ["OMP_NUM_THREADS"]))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return max(1, n), model


def cpu_baseline(hy, synth, sf, chunk, runs=5, mode="join"):
    """The oracle (CPU restatement of the reference operators with the reference's per-chunk / per-partition jobs)
    on a bounded sample of the same workload: TableScan(l_quantity < 24) on dictionary-encoded lineitem, then
    JoinHash(orders, scan output) - or, for config 2 (mode "scan"), the TableScan alone, and for config 3 ("join-only")
    JoinHash(orders, lineitem) over every lineitem row. Median of `runs` warm runs on all host cores of this process,
    and on 1 core at a fifth of the sample."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import helpers

    oracle = helpers.load_oracle()
    threads, model = host_cpu()
    out = {"unit": "rows/s", "kind": "port", "cpu_model": model, "nproc": os.cpu_count(),
           "cores_note": "all cores this process may use: the GPU box grants one GPU's share of a larger machine "
                         "(OMP_NUM_THREADS, 16 per GPU); nproc counts the whole machine"}
    for label, n_threads, sample_sf in (("all_cores", threads, sf), ("one_core", 1, sf / 5)):
        okey, lines = synth.orders_numpy(sample_sf)
        lkey, qty = synth.lineitem_numpy(okey, lines)
        orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False)], [okey], [], chunk)
        lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, False),
                                         ("l_quantity", hy.DataType.Float, False)],
                                        [lkey, qty.astype(np.float32)], [], chunk)
        hy.encode_all_chunks(lineitem, hy.EncodingType.Dictionary)
        oracle.set_threads(n_threads)
        times = []
        scan = join = None
        for _ in range(runs + 1):  # the first run warms caches and allocators
            t0 = time.perf_counter()
            if mode != "join-only":
                scan = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24, [])
            if mode != "scan":
                join, _bits = oracle.join_hash(orders, lineitem if mode == "join-only" else scan, hy.JoinMode.Inner,
                                               (0, 0))
            times.append(time.perf_counter() - t0)
        oracle.set_threads(1)
        med = sorted(times[1:])[len(times[1:]) // 2]
        rows = lineitem.row_count() + (0 if mode == "scan" else orders.row_count())
        what = {"join": f"scan {scan.row_count() if scan else 0} matches, join {join.row_count() if join else 0} pairs",
                "scan": f"scan {scan.row_count() if scan else 0} matches",
                "join-only": f"join {join.row_count() if join else 0} pairs"}[mode]
        out[label] = {"value": round(rows / med, 1), "cores": n_threads, "median_s": round(med, 3),
                      "runs_s": [round(t, 3) for t in times[1:]],
                      "sample": f"SF{sample_sf:g}: {lineitem.row_count()} lineitem + {orders.row_count()} orders "
                                f"rows, {what}"}
        del orders, lineitem, scan, join
    out["value"], out["cores"] = out["all_cores"]["value"], out["all_cores"]["cores"]
    out["sample"] = out["all_cores"]["sample"] + f"; median of {runs}"
    return out


if __name__ == "__main__":
    main()
