"""TPC-H 3 on one GPU (BASELINE.json configs[4] at N=1): `python bench.py --workload q3`.

One step is the reference's plan for tpch_queries.cpp:101-106, on columns resident in HBM, through the C-ABI:

    TableScan(customer, c_mktsegment = 'BUILDING')                       hy_table_scan_row_ids (dictionary u8)
    JoinHash(<customer scan>, TableScan(orders, o_orderdate < 1995-03-15), c_custkey = o_custkey)
                                                                          hy_scan_join_hash: the orders scan runs
                                                                          inside the join's first partition pass
    JoinHash(<that join>, TableScan(lineitem, l_shipdate > 1995-03-15), o_orderkey = l_orderkey)
                                                                          hy_scan_join_hash, same fusion
    Projection(l_orderkey, o_orderdate, o_shippriority, l_extendedprice * (1 - l_discount))   hy_projection x 4
    Aggregate(GROUP BY l_orderkey, o_orderdate, o_shippriority; SUM(revenue))                  hy_aggregate

The builds are the smaller inputs (the reference's swap rule, join_hash.cpp:55-76; checked after the run), radix bits
come from the build input's row count (join_hash.cpp:640-668), so the step reads the customer scan's per-chunk counts
and each join's partition bounds back to the host, as the operators would. A join's output chunks are its non-empty
radix partitions in ascending order (write_output_columns). The second join's build side dereferences the first join's
orders PosLists (the orders columns of the join output); the customer columns are not read after the first join
(the reference's column pruning). ORDER BY / LIMIT (Sort) is outside the hot path.

Dates are int32 days in per-chunk dictionaries (u16 value ids, the reference's default Dictionary encoding; ISO date
strings order like their days), c_mktsegment is a u8 dictionary of its five codes, keys are unencoded int32 columns.
Rows/s counts the base rows consumed (customer + orders + lineitem). The result is checked against torch on the same
columns: match and pair counts, group count and every sampled group's SUM exactly (an order's revenue is a sum of
<= 7 float products, exact in double).
"""
import ctypes
import glob
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
INVALID_VALUE_ID = 0xFFFFFFFF


def dict_predicate(capi, lb, ub, dict_size, cond):
    """(op, search_vid) for a dictionary chunk, from lower_bound / upper_bound value ids of the constant
    (single_column_table_scan_impl.cpp:145-205 via operators.cpp dictionary_predicate; INVALID when at the end)."""
    lb = INVALID_VALUE_ID if lb >= dict_size else lb
    ub = INVALID_VALUE_ID if ub >= dict_size else ub
    svid = ub if cond in ("LessThanEquals", "GreaterThan") else lb
    one = dict_size == 1
    if cond == "Equals":
        all_, none = svid != ub and one, svid == ub
    elif cond in ("LessThan", "LessThanEquals"):
        all_, none = svid == INVALID_VALUE_ID, svid == 0
    else:
        all_, none = svid == 0, svid == INVALID_VALUE_ID
    if all_:
        return capi.HY_OP_ALL, svid
    if none:
        return capi.HY_OP_NONE, svid
    return {"Equals": capi.HY_OP_EQ, "LessThan": capi.HY_OP_LT, "LessThanEquals": capi.HY_OP_LT}.get(
        cond, capi.HY_OP_GE), svid


class DictColumn:
    """A chunked integer column dictionary-encoded per chunk on the device (vids u8 / u16 by dictionary size)."""

    def __init__(self, torch, synth, capi, values, chunk, lo, domain, dict_values=None):
        """values: integer codes in [lo, lo + domain); the dictionary holds the codes themselves (int32), or
        dict_values[code - lo] (e.g. float32 values whose order is the codes' order)."""
        vids, present = synth.dictionary_encode_chunks(values, chunk, lo, domain)
        n = values.numel()
        self.n_chunks = present.shape[0]
        self.sizes = [min(chunk, n - c * chunk) for c in range(self.n_chunks)]
        dsize = present.sum(dim=1)
        # dictionaries: dict[c, rank] = lo + value index, one row of `domain` int32 per chunk
        rank = torch.cumsum(present.to(torch.int32), dim=1) - 1
        rows, js = torch.nonzero(present, as_tuple=True)
        dv = (torch.arange(lo, lo + domain, dtype=torch.int32, device=values.device) if dict_values is None
              else dict_values.to(values.device))
        self.dicts = torch.zeros(self.n_chunks, domain, dtype=dv.dtype, device=values.device)
        self.dicts[rows, rank[rows, js].long()] = dv[js]
        self.cum = torch.cumsum(present.to(torch.int64), dim=1).cpu().numpy()  # cum[c, j] = #values <= lo + j
        self.dsize = dsize.cpu().numpy()
        self.lo, self.domain = lo, domain
        wide = self.dsize > 0xFF
        self.v16 = torch.cat([vids.to(torch.int16), torch.zeros(64, dtype=torch.int16, device=values.device)])
        self.v8 = torch.cat([vids.to(torch.uint8), torch.zeros(64, dtype=torch.uint8, device=values.device)]) \
            if not wide.all() else None
        self.desc = (capi.ColumnChunk * self.n_chunks)()
        for c in range(self.n_chunks):
            d = self.desc[c]
            w = 2 if wide[c] else 1
            d.data = (self.v16.data_ptr() + 2 * c * chunk) if w == 2 else (self.v8.data_ptr() + c * chunk)
            d.size = self.sizes[c]
            d.kind, d.vid_width = capi.HY_COL_DICT, w
            d.dictionary = self.dicts.data_ptr() + 4 * domain * c
            d.dictionary_size = int(self.dsize[c])

    def scan_chunks(self, capi, cond, value):
        arr = (capi.ScanChunk * self.n_chunks)()
        j = value - self.lo
        for c in range(self.n_chunks):
            lb = int(self.cum[c, j - 1]) if 0 < j <= self.domain else (0 if j <= 0 else int(self.dsize[c]))
            ub = int(self.cum[c, j]) if 0 <= j < self.domain else (0 if j < 0 else int(self.dsize[c]))
            s = arr[c]
            s.column = self.desc[c]
            s.op, s.search_vid = dict_predicate(capi, lb, ub, int(self.dsize[c]), cond)
        return arr


def value_chunks(capi, t, chunk, width):
    n = t.numel() - 64
    n_chunks = (n + chunk - 1) // chunk
    arr = (capi.ColumnChunk * n_chunks)()
    for c in range(n_chunks):
        arr[c].data = t.data_ptr() + width * c * chunk
        arr[c].size = min(chunk, n - c * chunk)
        arr[c].kind = capi.HY_COL_VALUE
    return arr


def data_side(capi, cols, value_type):
    arr = (capi.JoinChunk * len(cols))()
    for c in range(len(cols)):
        arr[c].column = cols[c]
        arr[c].size = cols[c].size
        arr[c].chunk_id = c
        arr[c].single_chunk = capi.HY_MIXED_CHUNKS
    side = capi.JoinSide(arr, len(cols), value_type, None, 0, 0, 0)
    side._keep = arr
    return side


def expr_column(capi, col, vtype):
    return capi.ExprNode(capi.HY_EXPR_COLUMN, vtype, 0, col, 0)


def main_q3(args):
    import numpy as np
    import torch

    if int(os.environ.get("WORLD_SIZE", "1")) > 1 or os.environ.get("HY_BENCH_DIST"):
        # N ranks: the distributed plan through the JoinHash radix shuffle (bench_q3_dist.py)
        import bench_q3_dist

        return bench_q3_dist.main_q3_dist(args)
    # one GPU (N > 1 returned above: the plan through the JoinHash radix shuffle)
    world = 1
    sys.path.insert(0, ROOT)
    hy = importlib.import_module("hyrise-1_amd")
    synth = importlib.import_module("hyrise-1_amd.synth")
    capi = hy.capi
    L = capi.lib
    torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    capi.check(L.hy_set_device(dev.index), "hy_set_device")
    stream = torch.cuda.current_stream().cuda_stream
    chunk = args.chunk
    D = synth.DATE_1995_03_15
    I32, F32 = capi.HY_TYPE_INT32, capi.HY_TYPE_FLOAT

    # ---------------- data ----------------
    cols = synth.q3_columns(args.sf, dev)
    n_cust, n_ord, n_li = (cols[k].numel() for k in ("c_custkey", "o_orderkey", "l_orderkey"))
    # expected result (torch on the same columns)
    seg_ok = cols["c_mktsegment"] == 1  # BUILDING
    o_date_ok = cols["o_orderdate"] < D
    o_ok = o_date_ok & seg_ok[cols["o_custkey"].long() - 1]
    l_date_ok = cols["l_shipdate"] > D
    l_ok = l_date_ok & o_ok[cols["l_order_index"]]
    exp = {"customer_matches": int(seg_ok.sum()), "orders_matches": int(o_date_ok.sum()),
           "lineitem_matches": int(l_date_ok.sum()), "join1_pairs": int(o_ok.sum()), "join2_pairs": int(l_ok.sum())}
    rev = cols["l_extendedprice"] * (1 - cols["l_discount"])  # float32, as the projection computes it
    order_rev = torch.zeros(n_ord, dtype=torch.float64, device=dev).index_add_(
        0, cols["l_order_index"][l_ok], rev[l_ok].to(torch.float64))
    order_hit = torch.zeros(n_ord, dtype=torch.bool, device=dev)
    order_hit[cols["l_order_index"][l_ok]] = True
    exp["groups"] = int(order_hit.sum())
    del seg_ok, o_date_ok, o_ok, l_date_ok, l_ok, rev
    n_ord_g, n_li_g = n_ord, n_li

    def padded(t):
        return torch.cat([t.contiguous(), torch.zeros(64, dtype=t.dtype, device=t.device)])

    seg = DictColumn(torch, synth, capi, cols["c_mktsegment"], chunk, 0, 5)
    odate = DictColumn(torch, synth, capi, cols["o_orderdate"], chunk, synth.DATE_1992_01_01,
                       synth.DATE_1998_08_02 - synth.DATE_1992_01_01 + 1)
    ship = DictColumn(torch, synth, capi, cols["l_shipdate"], chunk, synth.DATE_1992_01_01,
                      synth.DATE_1998_08_02 + 121 - synth.DATE_1992_01_01 + 1)
    ckey, ocust, okey = padded(cols["c_custkey"]), padded(cols["o_custkey"]), padded(cols["o_orderkey"])
    oprio, lkey = padded(cols["o_shippriority"]), padded(cols["l_orderkey"])
    price, disc = padded(cols["l_extendedprice"]), padded(cols["l_discount"])
    del cols
    torch.cuda.synchronize()
    ckey_c, ocust_c, okey_c = (value_chunks(capi, t, chunk, 4) for t in (ckey, ocust, okey))
    oprio_c, lkey_c, price_c, disc_c = (value_chunks(capi, t, chunk, 4) for t in (oprio, lkey, price, disc))
    n_cc, n_oc, n_lc = len(ckey_c), len(okey_c), len(lkey_c)

    # ---------------- operators' fixed descriptors ----------------
    cscan = seg.scan_chunks(capi, "Equals", 1)
    for c in range(n_cc):
        cscan[c].out_begin = c * chunk
    c_ids = (ctypes.c_uint32 * n_cc)(*range(n_cc))
    wsb = ctypes.c_size_t(0)
    capi.check(L.hy_table_scan_workspace_size((ctypes.c_uint32 * n_cc)(*seg.sizes), n_cc, ctypes.byref(wsb)), "ws")
    c_ws = torch.empty(max(16, wsb.value), dtype=torch.uint8, device=dev)
    c_rows = torch.empty(2 * n_cust + 64, dtype=torch.int32, device=dev)
    c_counts = torch.empty(n_cc, dtype=torch.int32, device=dev)
    L.hy_table_scan_row_ids.restype = ctypes.c_int
    L.hy_table_scan_row_ids.argtypes = [ctypes.POINTER(capi.ScanChunk), ctypes.c_uint32, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]

    orders_side = data_side(capi, ocust_c, I32)
    li_side = data_side(capi, lkey_c, I32)
    # The orders / lineitem scans feed only their join: the fused operator returns their per-chunk match counts and
    # not their PosLists (hy_join_filter.out_offsets NULL), so a join side's first pass writes records for the rows
    # that pass the prefilter only. HY_Q3_SCAN_POSLISTS=1 materialises the scans' PosLists as well (A/B).
    scan_poslists = os.environ.get("HY_Q3_SCAN_POSLISTS") == "1"
    o_off = torch.empty(n_ord + 64, dtype=torch.int32, device=dev) if scan_poslists else None
    o_begin = torch.zeros(n_oc + 1, dtype=torch.int64, device=dev)
    ofilter = capi.JoinFilter(odate.scan_chunks(capi, "LessThan", D), I32, None,
                              o_off.data_ptr() if scan_poslists else None, o_begin.data_ptr())
    l_off = torch.empty(n_li + 64, dtype=torch.int32, device=dev) if scan_poslists else None
    l_begin = torch.zeros(n_lc + 1, dtype=torch.int64, device=dev)
    lfilter = capi.JoinFilter(ship.scan_chunks(capi, "GreaterThan", D), I32, None,
                              l_off.data_ptr() if scan_poslists else None, l_begin.data_ptr())
    jc_dtype = np.dtype(capi.JoinChunk)
    cc_dtype = np.dtype(capi.ColumnChunk)
    state = {"ws": {}, "cap": {}}

    def workspace(key, query):
        if key not in state["ws"]:
            b = ctypes.c_size_t(0)
            capi.check(query(ctypes.byref(b)), "workspace size")
            state["ws"][key] = torch.empty(max(16, b.value), dtype=torch.uint8, device=dev)
        return state["ws"][key]

    def out_pairs(tag, cap):
        if state["cap"].get(tag, (0,))[0] < cap:
            state["cap"][tag] = (cap, torch.empty(2 * cap, dtype=torch.int32, device=dev),
                                 torch.empty(2 * cap, dtype=torch.int32, device=dev))
        return state["cap"][tag]

    def ref_side(pos_base, begins, counts, single, referenced, n_referenced):
        """A reference input's join side: chunk k = PosList pos_base + 8 * begins[k] of counts[k] RowIDs."""
        arr = np.zeros(len(counts), jc_dtype)
        arr["pos_list"] = pos_base + 8 * begins.astype(np.uint64)
        arr["size"] = counts
        arr["chunk_id"] = np.arange(len(counts), dtype=np.uint32)
        arr["single_chunk"] = single
        side = capi.JoinSide(arr.ctypes.data_as(ctypes.POINTER(capi.JoinChunk)), len(counts), I32, referenced,
                             n_referenced, 1, 0)
        side._keep = arr
        return side

    def join(tag, build, probe, pfilter, bits, cap_hint):
        params = capi.JoinParams(capi.HY_JOIN_INNER, I32, bits, 17)
        ws = workspace((tag, bits, build.n_chunks), lambda b: L.hy_scan_join_hash_workspace_size(
            ctypes.byref(build), None, ctypes.byref(probe), ctypes.byref(pfilter), ctypes.byref(params), b))
        pb = torch.empty(1 << bits, dtype=torch.int64, device=dev)
        pc = torch.empty(1 << bits, dtype=torch.int32, device=dev)
        while True:
            cap, ob, op = out_pairs(tag, cap_hint)
            res = capi.JoinResult()
            st = L.hy_scan_join_hash(ctypes.byref(build), None, ctypes.byref(probe), ctypes.byref(pfilter),
                                     ctypes.byref(params), ob.data_ptr(), op.data_ptr(), cap, pb.data_ptr(),
                                     pc.data_ptr(), ctypes.byref(res), ws.data_ptr(), ws.numel(), stream)
            if st != capi.HY_ERR_CAPACITY:
                capi.check(st, "hy_scan_join_hash " + tag)
                break
            cap_hint = res.capacity_required + 64
        pb_h, pc_h = pb.cpu().numpy(), pc.cpu().numpy()
        nz = np.nonzero(pc_h)[0]
        return ob, op, pb_h[nz], pc_h[nz].astype(np.uint32), res.total_pairs

    proj_cols = (capi.AggColumn * 5)()
    for j, (vt, g, ch) in enumerate([(I32, 1, lkey_c), (I32, 0, odate.desc), (I32, 0, oprio_c), (F32, 1, price_c),
                                     (F32, 1, disc_c)]):
        proj_cols[j].value_type, proj_cols[j].pos_group, proj_cols[j].chunks, proj_cols[j].n_chunks = vt, g, ch, len(ch)
    programs = [[expr_column(capi, 0, I32)], [expr_column(capi, 1, I32)], [expr_column(capi, 2, I32)],
                [expr_column(capi, 3, F32), capi.ExprNode(capi.HY_EXPR_VALUE, I32, 0, 0, 1),
                 expr_column(capi, 4, F32), capi.ExprNode(capi.HY_EXPR_SUB, F32, F32, 0, 0),
                 capi.ExprNode(capi.HY_EXPR_MUL, F32, F32, 0, 0)]]
    programs = [(capi.ExprNode * len(p))(*p) for p in programs]
    prog_ptrs = (ctypes.c_void_p * len(programs))(*[ctypes.addressof(p) for p in programs])
    prog_lens = (ctypes.c_uint32 * len(programs))(*[len(p) for p in programs])
    groupby = (ctypes.c_int32 * 3)(0, 1, 2)
    agg_defs = (capi.AggDef * 1)(capi.AggDef(capi.HY_AGG_SUM, 3))
    agg_params = capi.AggParams(groupby, 3, agg_defs, 1, 0)

    trace_q3 = os.environ.get("HY_Q3_TRACE") is not None  # host wall time per operator (each ends synchronised)

    def mark(label, t=[0.0]):
        if trace_q3:
            now = time.perf_counter()
            if label != "start":
                print(f"[q3] {label} {1e3 * (now - t[0]):.3f} ms", file=sys.stderr)
            t[0] = now

    def step():
        mark("start")
        # TableScan(customer, c_mktsegment = 'BUILDING'): its output's chunk layout decides the join's build input
        capi.check(L.hy_table_scan_row_ids(cscan, n_cc, I32, None, c_ids, c_rows.data_ptr(), c_counts.data_ptr(),
                                           c_ws.data_ptr(), c_ws.numel(), stream), "customer scan")
        cc = c_counts.cpu().numpy()
        nz = np.nonzero(cc)[0]
        c_match = int(cc.sum())
        build1 = ref_side(c_rows.data_ptr(), nz.astype(np.uint64) * chunk, cc[nz].astype(np.uint32),
                          nz.astype(np.uint32), ckey_c, n_cc)
        j1b, j1p, b1, n1, pairs1 = join("j1", build1, orders_side, ofilter, L.hy_join_radix_bits(c_match, 4),
                                        n_ord // 4 + 64)
        mark("customer scan + join 1")
        build2 = ref_side(j1p.data_ptr(), b1, n1, capi.HY_MIXED_CHUNKS, okey_c, n_oc)
        j2b, j2p, b2, n2, pairs2 = join("j2", build2, li_side, lfilter, L.hy_join_radix_bits(pairs1, 4),
                                        n_li // 32 + 64)
        mark("join 2")
        # Projection over the join output (chunks = non-empty partitions; PosList groups: orders, lineitem)
        k = len(n2)
        sizes_np = np.ascontiguousarray(n2, dtype=np.uint32)
        pls_np = np.concatenate([j2b.data_ptr() + 8 * b2.astype(np.uint64), j2p.data_ptr() + 8 * b2.astype(np.uint64)])
        sizes = sizes_np.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        pls = pls_np.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p))
        pin = capi.AggInput(k, sizes, pls, 2, proj_cols, 5)
        pws = workspace(("proj", k), lambda b: L.hy_projection_workspace_size(ctypes.byref(pin), b))
        if state.get("proj_rows", 0) < pairs2:
            state["proj_rows"] = pairs2
            state["proj"] = torch.empty(4, pairs2 + 64, dtype=torch.int32, device=dev)
        proj = state["proj"]
        # the four SELECT-list expressions in one launch (the reference's Projection evaluates them per chunk)
        outs = (ctypes.c_void_p * 4)(*[proj[j].data_ptr() for j in range(4)])
        capi.check(L.hy_projection_multi(ctypes.byref(pin), prog_ptrs, prog_lens, 4, outs, None, pws.data_ptr(),
                                         pws.numel(), stream), "hy_projection_multi")
        mark("projection")
        # Aggregate over the projection's output (a data table with the join output's chunking)
        rb = np.concatenate([[0], np.cumsum(n2.astype(np.int64))])[:-1].astype(np.uint64)
        acols = (capi.AggColumn * 4)()
        keep = []
        for j, vt in enumerate([I32, I32, I32, F32]):
            ch = np.zeros(max(1, k), cc_dtype)
            ch["data"][:k] = proj[j].data_ptr() + 4 * rb
            ch["size"][:k] = n2
            ch["kind"] = capi.HY_COL_VALUE
            keep.append(ch)
            acols[j].value_type, acols[j].pos_group, acols[j].n_chunks = vt, -1, k
            acols[j].chunks = ch.ctypes.data_as(ctypes.POINTER(capi.ColumnChunk))
        ain = capi.AggInput(k, sizes, None, 0, acols, 4)
        if "layout" not in state:
            lay = capi.AggLayout()
            capi.check(L.hy_aggregate_layout(ctypes.byref(ain), ctypes.byref(agg_params), ctypes.byref(lay)), "layout")
            state["layout"] = lay
        words = state["layout"].words
        aws = workspace(("agg", k, pairs2, agg_params.group_bound), lambda b: L.hy_aggregate_workspace_size(
            ctypes.byref(ain), ctypes.byref(agg_params), b))
        if state.get("agg_cap", 0) < pairs2 + 1:
            state["agg_cap"] = pairs2 + 1
            state["agg_out"] = torch.empty((pairs2 + 1) * words, dtype=torch.int64, device=dev)
        ng = ctypes.c_uint64(0)
        while True:
            st = L.hy_aggregate(ctypes.byref(ain), ctypes.byref(agg_params), state["agg_out"].data_ptr(),
                                state["agg_cap"], ctypes.byref(ng), aws.data_ptr(), aws.numel(), stream)
            if st != capi.HY_ERR_GROUP_BOUND:
                break
            agg_params.group_bound = ng.value  # more groups than the table was sized for: grow it
            aws = workspace(("agg", k, pairs2, ng.value), lambda b: L.hy_aggregate_workspace_size(
                ctypes.byref(ain), ctypes.byref(agg_params), b))
        capi.check(st, "hy_aggregate")
        mark("aggregate")
        return {"customer_matches": c_match, "join1_pairs": int(pairs1), "join2_pairs": int(pairs2),
                "groups": int(ng.value)}

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        got = step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-kernel device times: K more steps with HIP events around every launch (kept out of the timed region)
    L.hy_kernel_stats_reset()
    L.hy_kernel_stats_enable(1)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    L.hy_kernel_stats_enable(0)
    got["orders_matches"] = int(o_begin[-1].item())
    got["lineitem_matches"] = int(l_begin[-1].item())
    local_groups = got["groups"]

    # ---------------- check ----------------
    lay = state["layout"]
    rec = state["agg_out"].view(-1, lay.words)[:local_groups].cpu().numpy().view(np.uint64)
    ok = got == exp
    # the reference's swap rule kept the builds on the smaller inputs
    ok &= got["customer_matches"] <= got["orders_matches"] and got["join1_pairs"] <= got["lineitem_matches"]
    # every group: its revenue (decoded exactly once, hy_agg_float_sums) equals the order's revenue summed in float64
    # by torch (<= 7 float products per order: exact), keyed by the inverse of the dbgen sparse order key
    order_rev_h = order_rev.cpu().numpy()
    w = lay.agg_word[0]
    rec = np.ascontiguousarray(rec)
    sums = np.zeros(rec.shape[0], dtype=np.float64)
    capi.check(L.hy_agg_float_sums(rec.ctypes.data, rec.shape[0], lay.words, w, lay.agg_limbs[0], lay.agg_emin[0],
                                   sums.ctypes.data), "hy_agg_float_sums")
    keys = rec[:, 0].astype(np.uint32).view(np.int32).astype(np.int64)
    oi = ((keys >> 5) << 3) + (keys & 7) - 1  # inverse of the dbgen sparse order key
    groups_ok = bool(rec.shape[0] == 0 or (np.all((oi >= 0) & (oi < order_rev_h.size)) and
                                            np.array_equal(sums, order_rev_h[oi])))
    ok &= groups_ok
    if not ok:
        raise SystemExit(f"q3 result mismatch: {got} vs {exp}")

    from bench import kernel_stats, measured_roofline, host_cpu  # noqa: E402  (shared helpers)

    kernels = kernel_stats(L)
    K = args.steps
    step_s = elapsed / K
    # algorithmic bytes (SURVEY.md 8(d) per operator): scans 1 B (u8 vids) / 2 B (u16 vids) per row read + output
    # (8 B RowIDs customer, 4 B offsets for the fused scans); JoinHash 4 B per build row + 4 B per probe row + 16 B
    # per pair; Projection per row 2 RowIDs + 4 x 4 B read... (16 + 20) in, 16 out; Aggregate per row 16 B in
    n_ord, n_li = n_ord_g, n_li_g
    cm, om, lm = got["customer_matches"], got["orders_matches"], got["lineitem_matches"]
    p1, p2 = got["join1_pairs"], got["join2_pairs"]
    alg = {"scans": n_cust * 1 + cm * 8 + n_ord * 2 + om * 4 + n_li * 2 + lm * 4,
           "join1": cm * 4 + om * 4 + p1 * 16, "join2": p1 * 4 + lm * 4 + p2 * 16,
           "projection": p2 * (16 + 20 + 16), "aggregate": p2 * 16}
    e2e = sum(alg.values())
    peak, probe = measured_roofline(L, capi, torch, dev, stream, args.probe_gb)
    for v in kernels.values():
        v["ms_per_launch"] = v["ms_total"] / max(v["launches"], 1)
    dom = max(kernels, key=lambda k: kernels[k]["ms_total"])
    roofline = {"bound": "hbm", "scope": "end-to-end step (algorithmic bytes of SURVEY 8(d) per operator)",
                "achieved": round(e2e / step_s / 1e9, 1), "peak": round(peak, 1), "unit": "GB/s",
                "frac": round(e2e / step_s / 1e9 / peak, 4), "alg_bytes_per_step": e2e, "alg_bytes": alg,
                "traffic": None, "peak_source": "measured in this run (hy_stream_bandwidth_probe, best of read / copy)",
                "dominant_kernel": dom, "dominant_ms_per_step": round(kernels[dom]["ms_total"] / K, 4)}
    cpu = None if args.no_cpu_baseline else cpu_baseline_q3(hy, synth, args.cpu_sf, chunk, host_cpu)
    line = {
        "metric": "rows/sec TPC-H 3 (Scan -> JoinHash -> JoinHash -> Projection -> Aggregate), 1/2/4/8 MI355X",
        "value": round((n_cust + n_ord + n_li) / step_s, 1), "unit": "rows/s", "n_gpus": world, "steps": K,
        "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 3), "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None, "dtype": "int32/f32", "data": "synthetic (seeded counter-based TPC-H-shaped columns, "
                                                           "resident in HBM)",
        "config": {"workload": "TPC-H 3 (tpch_queries.cpp:101-106) without ORDER BY/LIMIT", "sf": args.sf,
                   "customer_rows": n_cust, "orders_rows": n_ord, "lineitem_rows": n_li, "chunk_size": chunk, "scan_poslists": scan_poslists,
                   **got, "parallelism": "single GPU"},
        "check": {"ok": bool(ok), "expected": exp, "groups_checked": int(rec.shape[0]), "groups_equal": groups_ok},
        "roofline": roofline,
        "hbm_probe": probe,
        "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                    for k, v in kernels.items()},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line))


def cpu_baseline_q3(hy, synth, sf, chunk, host_cpu, runs=5):
    """The oracle's Q3 operator chain (same plan, the reference's per-chunk / per-partition jobs) on a bounded sample
    of the same synthetic columns (dictionary-encoded like the reference default). Median of `runs` on all host cores
    of this process at SF `sf`, and on one core at a fifth of it."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import helpers

    oracle = helpers.load_oracle()
    threads, model = host_cpu()
    I, F = hy.DataType.Int, hy.DataType.Float
    P, A, O, V = (hy.PQPColumnExpression.from_table, hy.ArithmeticExpression, hy.ArithmeticOperator,
                  hy.ValueExpression)
    D = synth.DATE_1995_03_15
    cond = hy.PredicateCondition
    out = {"unit": "rows/s", "kind": "port", "cpu_model": model, "nproc": os.cpu_count()}
    for label, n_threads, sample_sf in (("all_cores", threads, sf), ("one_core", 1, sf / 5)):
        c = {k: v.numpy() for k, v in synth.q3_columns(sample_sf, "cpu").items()}
        customer = hy.Table.from_arrays([("c_custkey", I, False), ("c_mktsegment", I, False)],
                                        [c["c_custkey"], c["c_mktsegment"]], [], chunk)
        orders = hy.Table.from_arrays([("o_orderkey", I, False), ("o_custkey", I, False), ("o_orderdate", I, False),
                                       ("o_shippriority", I, False)],
                                      [c["o_orderkey"], c["o_custkey"], c["o_orderdate"], c["o_shippriority"]], [],
                                      chunk)
        lineitem = hy.Table.from_arrays([("l_orderkey", I, False), ("l_extendedprice", F, False),
                                         ("l_discount", F, False), ("l_shipdate", I, False)],
                                        [c["l_orderkey"], c["l_extendedprice"], c["l_discount"], c["l_shipdate"]], [],
                                        chunk)
        del c
        for t in (customer, orders, lineitem):
            hy.encode_all_chunks(t, hy.EncodingType.Dictionary)

        def run():
            cs = oracle.table_scan(customer, 1, cond.Equals, 1, [])
            os_ = oracle.table_scan(orders, 2, cond.LessThan, D, [])
            ls = oracle.table_scan(lineitem, 3, cond.GreaterThan, D, [])
            j1, _ = oracle.join_hash(cs, os_, hy.JoinMode.Inner, (0, 1))
            j2, _ = oracle.join_hash(j1, ls, hy.JoinMode.Inner, (2, 0))
            p = oracle.projection(j2, [P(j2, 6), P(j2, 4), P(j2, 5),
                                       A(O.Multiplication, P(j2, 7), A(O.Subtraction, V(1), P(j2, 8)))])
            return oracle.aggregate(p, [hy.AggregateColumnDefinition(3, hy.AggregateFunction.Sum)], [0, 1, 2])

        rows = customer.row_count() + orders.row_count() + lineitem.row_count()
        oracle.set_threads(n_threads)
        times = []
        for _ in range(runs + 1):  # the first run warms caches and allocators
            t0 = time.perf_counter()
            agg = run()
            times.append(time.perf_counter() - t0)
        oracle.set_threads(1)
        med = sorted(times[1:])[len(times[1:]) // 2]
        out[label] = {"value": round(rows / med, 1), "cores": n_threads, "median_s": round(med, 3),
                      "runs_s": [round(t, 3) for t in times[1:]],
                      "sample": f"SF{sample_sf:g}: {customer.row_count()} customer + {orders.row_count()} orders + "
                                f"{lineitem.row_count()} lineitem rows, {agg.row_count()} groups"}
        del customer, orders, lineitem, agg
    out["value"], out["cores"] = out["all_cores"]["value"], out["all_cores"]["cores"]
    out["sample"] = out["all_cores"]["sample"] + f"; median of {runs}"
    return out


# TPC-H 1 (tpch_queries.cpp:36-44): SELECT list over the scan, by aggregate-input column index
Q1_AGGS = [("SUM", 2), ("SUM", 3), ("SUM", 4), ("SUM", 5), ("AVG", 2), ("AVG", 3), ("AVG", 6), ("COUNT", -1)]


def main_q1(args):
    """BASELINE.json configs[3] on one GPU: TPC-H 1 with all eight aggregates on the reference schema's types.

    One step:
        TableScan(lineitem, l_shipdate <= 1998-09-02)          hy_table_scan_row_ids (dictionary u16 dates)
        Projection(l_extendedprice * (1 - l_discount), l_extendedprice * (1 - l_discount) * (1 + l_tax)) fused into
        Aggregate(GROUP BY l_returnflag, l_linestatus; SUM(l_quantity), SUM(l_extendedprice), SUM(disc_price),
                  SUM(charge), AVG(l_quantity), AVG(l_extendedprice), AVG(l_discount), COUNT(*))   hy_aggregate
    The reference's Projection materialises all seven SELECT-list inputs into a data table (projection.cpp:52-85)
    that the Aggregate then reads; here the two arithmetic expressions are expression columns of hy_aggregate,
    evaluated (in float, as the reference computes them) in the aggregation kernel, and every column is read through
    the scan's PosLists once - nothing is materialised. --q1-materialize runs the two hy_projection launches first
    instead (A/B). Float SUM/AVG are exact (rounded once); every sum is checked for equality with the correctly
    rounded exact sum of the same float32 values (gsum), counts exactly."""
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    sys.path.insert(0, ROOT)
    hy = importlib.import_module("hyrise-1_amd")
    synth = importlib.import_module("hyrise-1_amd.synth")
    capi = hy.capi
    L = capi.lib
    dist = None
    if world > 1:  # multi-GPU Aggregate: chunk ranges per rank, partial records all-gathered and merged exactly
        import torch.distributed as dist

        if args.dist_backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    xdev = dev if (dist is None or args.dist_backend == "nccl") else torch.device("cpu")
    capi.check(L.hy_set_device(dev.index), "hy_set_device")
    stream = torch.cuda.current_stream().cuda_stream
    chunk = args.chunk
    I32, F32 = capi.HY_TYPE_INT32, capi.HY_TYPE_FLOAT
    D = synth.DATE_1998_09_02

    cols = synth.q1_columns(args.sf, dev)
    n = cols["l_shipdate"].numel()  # rows of the whole table (all ranks)
    # expected results (torch, same columns)
    print(f"q1: {n} lineitem rows generated", file=sys.stderr, flush=True)
    mask = cols["l_shipdate"] <= D
    gkey = torch.where(mask, cols["l_returnflag"] * 2 + cols["l_linestatus"], -1)
    price, disc, tax = cols["l_extendedprice"], cols["l_discount"], cols["l_tax"]
    dp = price * (1 - disc)  # float32, as the projection computes it
    ch = dp * (1 + tax)
    # per-group masked reductions (a 6-slot index_add_ would be 6e8 contended float64 atomics)
    sel = [gkey == g for g in range(6)]

    def gsum(v):
        """Per group the correctly rounded double of the EXACT sum of the float32 values v: every value is an integer
        mantissa times a power of two, so the int64 sums of the mantissas per (group, exponent) are exact (at most 2^30
        rows x 2^24 per bucket), and one Python integer per group combines them; int / int rounds correctly."""
        bits = v.contiguous().view(torch.int32)
        e = (bits >> 23) & 0xFF
        assert not bool((e == 0xFF).any()), "non-finite value"
        m = ((bits & 0x7FFFFF) | torch.where(e > 0, 1 << 23, 0)).to(torch.int64)
        m = torch.where(bits < 0, -m, m)
        key = gkey.to(torch.int64) * 256 + torch.clamp(e, min=1).to(torch.int64)  # subnormals: exponent of e = 1
        keep = gkey >= 0
        buckets = torch.zeros(6 * 256, dtype=torch.int64, device=v.device).index_add_(0, key[keep], m[keep])
        b = buckets.view(6, 256).cpu().tolist()
        return [sum(int(x) << (ex - 1) for ex, x in enumerate(row) if x) / (1 << 149) for row in b]

    exp = {"count": [int(m.sum()) for m in sel], "qty": gsum(cols["l_quantity"]), "price": gsum(price),
           "disc_price": gsum(dp), "charge": gsum(ch), "disc": gsum(disc)}
    n_match_exp = int(mask.sum())
    del mask, gkey, dp, ch, sel
    print("q1: expected results computed", file=sys.stderr, flush=True)
    # this rank's shard: global chunks [rank * C / N, (rank + 1) * C / N) (strong scaling over the SF database)
    n_chunks_g = (n + chunk - 1) // chunk
    c_lo, c_hi = rank * n_chunks_g // world, (rank + 1) * n_chunks_g // world
    row_lo, row_hi = c_lo * chunk, min(n, c_hi * chunk)
    if world > 1:
        cols = {k: v[row_lo:row_hi].contiguous() for k, v in cols.items()}
        torch.cuda.empty_cache()
    n_local = row_hi - row_lo
    price, disc, tax = cols["l_extendedprice"], cols["l_discount"], cols["l_tax"]
    codes = lambda v, scale: torch.round(v.to(torch.float64) * scale).to(torch.int32)
    ship = DictColumn(torch, synth, capi, cols["l_shipdate"], chunk, synth.DATE_1992_01_01,
                      synth.DATE_1998_08_02 + 121 - synth.DATE_1992_01_01 + 1)
    rf = DictColumn(torch, synth, capi, cols["l_returnflag"], chunk, 0, 3)
    ls = DictColumn(torch, synth, capi, cols["l_linestatus"], chunk, 0, 2)
    qty = DictColumn(torch, synth, capi, codes(cols["l_quantity"], 1), chunk, 1, 50,
                     torch.arange(1, 51, dtype=torch.float32))
    dsc = DictColumn(torch, synth, capi, codes(disc, 100), chunk, 0, 11,
                     (torch.arange(11, dtype=torch.float64) / 100).to(torch.float32))
    tx = DictColumn(torch, synth, capi, codes(tax, 100), chunk, 0, 9,
                    (torch.arange(9, dtype=torch.float64) / 100).to(torch.float32))
    price_t = torch.cat([price.contiguous(), torch.zeros(64, dtype=torch.float32, device=dev)])
    del cols, price, disc, tax
    torch.cuda.synchronize()
    price_c = value_chunks(capi, price_t, chunk, 4)
    n_chunks = len(price_c)

    scan = ship.scan_chunks(capi, "LessThanEquals", D)
    for c in range(n_chunks):
        scan[c].out_begin = c * chunk
    ids = (ctypes.c_uint32 * n_chunks)(*range(n_chunks))
    wsb = ctypes.c_size_t(0)
    capi.check(L.hy_table_scan_workspace_size((ctypes.c_uint32 * n_chunks)(*ship.sizes), n_chunks,
                                              ctypes.byref(wsb)), "scan ws")
    scan_ws = torch.empty(max(16, wsb.value), dtype=torch.uint8, device=dev)
    rows_t = torch.empty(2 * n_local + 64, dtype=torch.int32, device=dev)
    counts_t = torch.empty(n_chunks, dtype=torch.int32, device=dev)
    L.hy_table_scan_row_ids.restype = ctypes.c_int
    L.hy_table_scan_row_ids.argtypes = [ctypes.POINTER(capi.ScanChunk), ctypes.c_uint32, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    proj_cols = (capi.AggColumn * 3)()
    for j, (vt, chs) in enumerate([(F32, price_c), (F32, dsc.desc), (F32, tx.desc)]):
        proj_cols[j].value_type, proj_cols[j].pos_group, proj_cols[j].chunks, proj_cols[j].n_chunks = vt, 0, chs, \
            n_chunks
    N = capi.ExprNode
    one = N(capi.HY_EXPR_VALUE, I32, 0, 0, 1)
    disc_price = [N(capi.HY_EXPR_COLUMN, F32, 0, 0, 0), one, N(capi.HY_EXPR_COLUMN, F32, 0, 1, 0),
                  N(capi.HY_EXPR_SUB, F32, F32, 0, 0), N(capi.HY_EXPR_MUL, F32, F32, 0, 0)]
    charge = disc_price + [one, N(capi.HY_EXPR_COLUMN, F32, 0, 2, 0), N(capi.HY_EXPR_ADD, F32, F32, 0, 0),
                           N(capi.HY_EXPR_MUL, F32, F32, 0, 0)]
    programs = [(N * len(p))(*p) for p in (disc_price, charge)]
    proj_out = torch.empty(2, n + 64, dtype=torch.float32, device=dev) if args.q1_materialize else None
    agg_cols = (capi.AggColumn * 8)()
    ref_cols = {0: (I32, rf.desc, 3), 1: (I32, ls.desc, 2), 2: (F32, qty.desc, 0), 3: (F32, price_c, 0),
                6: (F32, dsc.desc, 0), 7: (F32, tx.desc, 0)}
    for j, (vt, chs, dom) in ref_cols.items():
        agg_cols[j].value_type, agg_cols[j].pos_group, agg_cols[j].chunks = vt, 0, chs
        agg_cols[j].n_chunks, agg_cols[j].domain = n_chunks, dom
    # expression columns 4 and 5 over the aggregate input's columns 3 (price), 6 (discount), 7 (tax)
    col = lambda j: N(capi.HY_EXPR_COLUMN, F32, 0, j, 0)
    agg_dp = [col(3), one, col(6), N(capi.HY_EXPR_SUB, F32, F32, 0, 0), N(capi.HY_EXPR_MUL, F32, F32, 0, 0)]
    agg_ch = agg_dp + [one, col(7), N(capi.HY_EXPR_ADD, F32, F32, 0, 0), N(capi.HY_EXPR_MUL, F32, F32, 0, 0)]
    agg_programs = [(N * len(p))(*p) for p in (agg_dp, agg_ch)]
    groupby = (ctypes.c_int32 * 2)(0, 1)
    defs = (capi.AggDef * len(Q1_AGGS))(*[capi.AggDef(getattr(capi, "HY_AGG_" + f), col) for f, col in Q1_AGGS])
    params = capi.AggParams(groupby, 2, defs, len(Q1_AGGS), 64)
    cc_dtype = np.dtype(capi.ColumnChunk)
    state = {}

    # fused plan (default): the TableScan's predicate evaluated inside the aggregate over the data chunks
    fused_scan = not (args.q1_poslist or args.q1_materialize)
    if fused_scan:
        data_cols = (capi.AggColumn * 8)()
        for j, (vt, chs, dom) in ref_cols.items():
            data_cols[j].value_type, data_cols[j].pos_group, data_cols[j].chunks = vt, -1, chs
            data_cols[j].n_chunks, data_cols[j].domain = n_chunks, dom
        for j, prog in ((4, agg_programs[0]), (5, agg_programs[1])):
            data_cols[j].value_type, data_cols[j].pos_group, data_cols[j].n_chunks = F32, -1, 0
            data_cols[j].program, data_cols[j].n_nodes = prog, len(prog)
        all_sizes = (ctypes.c_uint32 * n_chunks)(*ship.sizes)
        fin = capi.AggInput(n_chunks, all_sizes, None, 0, data_cols, 8)
        fin.filter, fin.filter_value_type, fin.filter_constant = scan, I32, None

    def step_fused():
        if "ws" not in state:
            b = ctypes.c_size_t(0)
            capi.check(L.hy_aggregate_workspace_size(ctypes.byref(fin), ctypes.byref(params), ctypes.byref(b)), "ws")
            state["ws"] = torch.empty(b.value, dtype=torch.uint8, device=dev)
            lay = capi.AggLayout()
            capi.check(L.hy_aggregate_layout(ctypes.byref(fin), ctypes.byref(params), ctypes.byref(lay)), "layout")
            state["layout"] = lay
            state["out"] = torch.empty(64 * lay.words, dtype=torch.int64, device=dev)
        ng = ctypes.c_uint64(0)
        capi.check(L.hy_aggregate(ctypes.byref(fin), ctypes.byref(params), state["out"].data_ptr(), 64,
                                  ctypes.byref(ng), state["ws"].data_ptr(), state["ws"].numel(), stream),
                   "hy_aggregate (fused scan)")
        return ng

    def step():
        if fused_scan:
            ng = step_fused()
            return merge_or_local(ng, None)
        capi.check(L.hy_table_scan_row_ids(scan, n_chunks, I32, None, ids, rows_t.data_ptr(), counts_t.data_ptr(),
                                           scan_ws.data_ptr(), scan_ws.numel(), stream), "scan")
        cnt = counts_t.cpu().numpy()
        nz = np.nonzero(cnt)[0]
        k = len(nz)
        sizes_np = np.ascontiguousarray(cnt[nz], dtype=np.uint32)
        pls_np = (rows_t.data_ptr() + 8 * chunk * nz.astype(np.uint64)).astype(np.uint64)
        sizes = sizes_np.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        pls = pls_np.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p))
        keep = []
        if args.q1_materialize:
            pin = capi.AggInput(k, sizes, pls, 1, proj_cols, 3)
            if "pws" not in state:
                b = ctypes.c_size_t(0)
                capi.check(L.hy_projection_workspace_size(ctypes.byref(pin), ctypes.byref(b)), "proj ws")
                state["pws"] = torch.empty(max(16, b.value), dtype=torch.uint8, device=dev)
            pws = state["pws"]
            for j, prog in enumerate(programs):
                capi.check(L.hy_projection(ctypes.byref(pin), prog, len(prog), proj_out[j].data_ptr(), None,
                                           pws.data_ptr(), pws.numel(), stream), "hy_projection")
            rb = np.concatenate([[0], np.cumsum(sizes_np.astype(np.int64))])[:-1].astype(np.uint64)
            for j in (4, 5):  # the projection's columns: data chunks aligned with the scan output's chunks
                chs = np.zeros(max(1, k), cc_dtype)
                chs["data"][:k] = proj_out[j - 4].data_ptr() + 4 * rb
                chs["size"][:k] = sizes_np
                chs["kind"] = capi.HY_COL_VALUE
                keep.append(chs)
                agg_cols[j].value_type, agg_cols[j].pos_group, agg_cols[j].n_chunks = F32, -1, k
                agg_cols[j].chunks = chs.ctypes.data_as(ctypes.POINTER(capi.ColumnChunk))
                agg_cols[j].program, agg_cols[j].n_nodes = None, 0
        else:
            for j, prog in ((4, agg_programs[0]), (5, agg_programs[1])):
                agg_cols[j].value_type, agg_cols[j].pos_group, agg_cols[j].n_chunks = F32, -1, 0
                agg_cols[j].program, agg_cols[j].n_nodes = prog, len(prog)
        ain = capi.AggInput(k, sizes, pls, 1, agg_cols, 8)
        if "ws" not in state:
            b = ctypes.c_size_t(0)
            capi.check(L.hy_aggregate_workspace_size(ctypes.byref(ain), ctypes.byref(params), ctypes.byref(b)), "ws")
            state["ws"] = torch.empty(b.value, dtype=torch.uint8, device=dev)
            lay = capi.AggLayout()
            capi.check(L.hy_aggregate_layout(ctypes.byref(ain), ctypes.byref(params), ctypes.byref(lay)), "layout")
            state["layout"] = lay
            state["out"] = torch.empty(64 * lay.words, dtype=torch.int64, device=dev)
        ng = ctypes.c_uint64(0)
        capi.check(L.hy_aggregate(ctypes.byref(ain), ctypes.byref(params), state["out"].data_ptr(), 64,
                                  ctypes.byref(ng), state["ws"].data_ptr(), state["ws"].numel(), stream),
                   "hy_aggregate")
        return merge_or_local(ng, int(sizes_np.sum()))

    def merge_or_local(ng, n_match):
        """This rank's groups (one GPU), or the all-gathered and merged groups of every rank. n_match None: the
        fused scan's matches, counted from the records' rows words after the timed steps."""
        if world == 1:
            state["records"] = None
            return n_match, ng.value
        # all-gather of the ranks' partial records (64 x words each, groups count in front) and the exact merge
        words = state["layout"].words
        buf = torch.empty(1 + 64 * words, dtype=torch.int64, device=dev)
        buf[0] = int(ng.value)
        buf[1:] = state["out"][:64 * words]
        buf = buf.to(xdev)
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf)
        host = [np.ascontiguousarray(t.cpu().numpy().view(np.uint64)) for t in parts]
        ptrs = (ctypes.POINTER(ctypes.c_uint64) * world)(*[h[1:].ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
                                                           for h in host])
        ngs = (ctypes.c_uint64 * world)(*[int(h[0]) for h in host])
        bases = (ctypes.c_uint64 * world)(*[min(n, (r * n_chunks_g // world) * chunk) for r in range(world)])
        merged = np.zeros((64, words), np.uint64)
        n_out = ctypes.c_uint64()
        capi.check(L.hy_aggregate_merge(ctypes.byref(params), ctypes.byref(state["layout"]), ptrs, ngs, bases, world,
                                        merged.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 64,
                                        ctypes.byref(n_out)), "hy_aggregate_merge")
        state["records"] = merged[:n_out.value]
        return n_match, n_out.value

    print("q1: columns encoded, running", file=sys.stderr, flush=True)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n_match, n_groups = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-kernel device times: K more steps with HIP events around every launch (kept out of the timed region)
    L.hy_kernel_stats_reset()
    L.hy_kernel_stats_enable(1)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    L.hy_kernel_stats_enable(0)
    if dist is not None:  # max over ranks; scan matches summed over ranks
        t = torch.tensor([elapsed], dtype=torch.float64, device=xdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        if n_match is not None:  # (fused scan: counted from the merged records below)
            m = torch.tensor([n_match], dtype=torch.int64, device=xdev)
            dist.all_reduce(m, op=dist.ReduceOp.SUM)
            n_match = int(m.item())

    # ---- check ----
    lay = state["layout"]
    if state["records"] is not None:
        rec = state["records"]
    else:
        rec = state["out"].view(-1, lay.words)[:n_groups].cpu().numpy().view(np.uint64)
    if fused_scan:  # the scan's matches = the groups' rows (every matching row is in exactly one group)
        n_match = int(sum(int(r[5]) for r in rec))

    def fsum(r, a):
        w = lay.agg_word[a]
        limbs = (ctypes.c_uint64 * lay.agg_limbs[a])(*[int(x) for x in r[w + 2:w + 2 + lay.agg_limbs[a]]])
        out = ctypes.c_double(0)
        capi.check(L.hy_agg_float_sum(limbs, lay.agg_limbs[a], lay.agg_emin[a], int(r[w + 1]), ctypes.byref(out)))
        return out.value

    ok = n_match == n_match_exp and n_groups == sum(1 for c in exp["count"] if c)
    groups = {}
    for r in rec:
        g = int(r[0]) * 2 + int(r[1])
        rows = int(r[5])
        vals = {"sum_qty": fsum(r, 0), "sum_base_price": fsum(r, 1), "sum_disc_price": fsum(r, 2),
                "sum_charge": fsum(r, 3), "count_order": rows}
        vals["avg_qty"], vals["avg_price"] = vals["sum_qty"] / rows, vals["sum_base_price"] / rows
        vals["avg_disc"] = fsum(r, 6) / rows
        # every float sum is the correctly rounded exact sum (aggregate.cpp:168-179 adds sequentially in double; the
        # device accumulates exactly and rounds once): compared for equality
        ok &= rows == exp["count"][g] and vals["sum_qty"] == exp["qty"][g]
        ok &= vals["sum_base_price"] == exp["price"][g] and vals["sum_disc_price"] == exp["disc_price"][g]
        ok &= vals["sum_charge"] == exp["charge"][g] and fsum(r, 6) == exp["disc"][g]
        groups["ANR"[int(r[0])] + "FO"[int(r[1])]] = vals
    if not ok:
        raise SystemExit(f"q1 result mismatch: {groups} vs {exp}")
    if rank != 0:
        dist.destroy_process_group()
        return

    from bench import kernel_stats, measured_roofline, host_cpu  # noqa: E402  (shared helpers)

    kernels = kernel_stats(L)
    K = args.steps
    step_s = elapsed / K
    # algorithmic bytes, independent of the path: scan 2 B/row (u16 date vids) + 8 B/match RowID;
    # aggregate (with its projection) per match: RowID 8 B + returnflag, linestatus, quantity, discount, tax vids 1 B
    # each + price 4 B = 17 B. Per kernel: the bytes that kernel must move on the path taken.
    # SURVEY 8(d)'s definition: the encoded widths of the 7 referenced columns, ~11 B/row (l_shipdate u16 vids for every
    # row, then returnflag, linestatus, quantity, discount, tax u8 vids + extendedprice 4 B per matching row); the
    # PosList the unfused plan writes and re-reads (8 B per match each way) is overhead, reported beside it
    e2e_parts = {"scan": n * 2, "aggregate": n_match * 9}
    overhead = {} if fused_scan else {"pos_list_write": n_match * 8, "pos_list_read": n_match * 8}
    alg = {"scan_dict": n * 2 + n_match * 8, "projection": n_match * (17 + 18), "agg_dense_span": n_match * 24,
           "agg_dense_fused": n_match * 17}
    # agg_dense_lanes reads per matching row the 9 B of columns, plus its 8-B RowID on the PosList plan
    alg["agg_dense_lanes"] = n * 2 + n_match * 9 if fused_scan else n_match * 17
    alg["agg_dense_vec"] = n * 2 + n_match * 9  # (data input: the fused plan only)
    e2e = sum(e2e_parts.values())
    for k, v in kernels.items():
        v["ms_per_launch"] = v["ms_total"] / max(v["launches"], 1)
        if k in alg:
            v["alg_bytes_per_step"] = alg[k]
            v["achieved_GBps"] = alg[k] / (v["ms_total"] / K * 1e-3) / 1e9
    peak, probe = measured_roofline(L, capi, torch, dev, stream, args.probe_gb)
    dom = max(kernels, key=lambda k: kernels[k]["ms_total"])
    roofline = {"bound": "hbm", "scope": "end-to-end step (algorithmic bytes of SURVEY 8(d) per operator)",
                "achieved": round(e2e / step_s / 1e9, 1), "peak": round(peak, 1), "unit": "GB/s",
                "frac": round(e2e / step_s / 1e9 / peak, 4), "alg_bytes_per_step": e2e, "alg_bytes": e2e_parts,
                "traffic": None, "peak_source": "measured in this run (hy_stream_bandwidth_probe, best of read / copy)",
                "dominant_kernel": dom, "dominant_ms_per_step": round(kernels[dom]["ms_total"] / K, 4),
                "overhead_bytes_per_step": overhead,
                "frac_incl_overhead": round((e2e + sum(overhead.values())) / step_s / 1e9 / peak, 4)}
    # the contract's `roofline`: the dominant kernel, its SURVEY 8(d) bytes per launch over its average launch time,
    # against the MI355X spec peak; traffic = its PMC bytes per launch from the committed rocprofv3 summary
    kroof = None
    if "alg_bytes_per_step" in kernels.get(dom, {}):
        kd = kernels[dom]
        per_launch = kd["alg_bytes_per_step"] * K / max(kd["launches"], 1)
        ach = per_launch / (kd["ms_per_launch"] * 1e-3) / 1e9
        traffic, src = None, None
        here = os.path.dirname(os.path.abspath(__file__))
        for f in reversed(sorted(glob.glob(os.path.join(here, "profiles", f"r*_rocprof_q1_sf{args.sf:g}_summary.json")))):
            with open(f) as fh:
                kk = json.load(fh).get("kernels", {}).get(dom, {})
            if "hbm_bytes_per_launch" in kk and args.chunk == 100_000 and world == 1:
                traffic, src = kk["hbm_bytes_per_launch"], os.path.relpath(f, here)
                break
        kroof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": 8000.0, "unit": "GB/s",
                 "frac": round(ach / 8000.0, 4), "traffic": round(traffic) if traffic is not None else None,
                 "traffic_source": src, "ms_per_launch": round(kd["ms_per_launch"], 4),
                 "bytes_per_launch": per_launch, "peak_measured": round(peak, 1),
                 "frac_of_measured_peak": round(ach / peak, 4)}
    # the reference Aggregate runs ~1e6 rows/s per core: a tenth of --cpu-sf keeps the sample near 10-30 s
    cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline_q1(hy, synth, args.cpu_sf / 10, chunk,
                                                                            host_cpu)
    line = {
        "metric": "rows/sec TableScan+Projection+Aggregate, TPC-H 1 on lineitem (BASELINE.json configs[3])",
        "value": round(n / step_s, 1), "unit": "rows/s", "n_gpus": world, "steps": K, "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 3), "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak", "vs_baseline": None,
        "dtype": "f32 (exact sums)", "data": "synthetic (seeded counter-based TPC-H-shaped columns, resident in HBM)",
        "config": {"workload": "TPC-H 1 (tpch_queries.cpp:36-44) without ORDER BY: scan l_shipdate <= 1998-09-02, "
                               "8 aggregates GROUP BY l_returnflag, l_linestatus", "sf": args.sf, "lineitem_rows": n,
                   "chunk_size": chunk, "scan_matches": n_match, "groups": n_groups,
                   "path": "TableScan fused into the aggregate (hy_agg_input.filter)" if fused_scan else
                   ("hy_table_scan_row_ids -> hy_projection x2 -> hy_aggregate" if args.q1_materialize else
                    "hy_table_scan_row_ids -> hy_aggregate with expression columns"),
                   "parallelism": "single GPU" if world == 1 else
                   f"chunk-sharded x{world}: per-rank scan + aggregate, all-gather of partial records, exact merge "
                   f"(hy_aggregate_merge)"},
        "check": {"ok": bool(ok), "groups": groups},
        "roofline": kroof or roofline,
        "roofline_e2e": roofline,
        "hbm_probe": probe,
        "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                    for k, v in kernels.items()},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline_q1(hy, synth, sf, chunk, host_cpu, runs=5):
    """The oracle's TPC-H 1 chain (TableScan -> Projection of the seven SELECT-list inputs -> Aggregate, the
    reference's plan and per-chunk jobs) on a bounded sample of the same columns, dictionary-encoded like the reference
    default. Median of `runs` on all host cores of this process at SF `sf`, and on one core at a fifth of it."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import helpers

    oracle = helpers.load_oracle()
    threads, model = host_cpu()
    I, F = hy.DataType.Int, hy.DataType.Float
    P, A, O, V = (hy.PQPColumnExpression.from_table, hy.ArithmeticExpression, hy.ArithmeticOperator,
                  hy.ValueExpression)
    out = {"unit": "rows/s", "kind": "port", "cpu_model": model, "nproc": os.cpu_count()}
    for label, n_threads, sample_sf in (("all_cores", threads, sf), ("one_core", 1, sf / 5)):
        print(f"q1 cpu baseline: {label} SF{sample_sf:g}", file=sys.stderr, flush=True)
        c = {k: v.numpy() for k, v in synth.q1_columns(sample_sf, "cpu").items()}
        names = ["l_returnflag", "l_linestatus", "l_quantity", "l_extendedprice", "l_discount", "l_tax", "l_shipdate"]
        types = [I, I, F, F, F, F, I]
        t = hy.Table.from_arrays([(nm, ty, False) for nm, ty in zip(names, types)], [c[nm] for nm in names], [],
                                 chunk)
        del c
        hy.encode_all_chunks(t, hy.EncodingType.Dictionary)
        aggs = [hy.AggregateColumnDefinition(None if col < 0 else col, getattr(hy.AggregateFunction, f.capitalize()))
                for f, col in Q1_AGGS]

        def run():
            s = oracle.table_scan(t, 6, hy.PredicateCondition.LessThanEquals, synth.DATE_1998_09_02, [])
            dp = A(O.Multiplication, P(s, 3), A(O.Subtraction, V(1), P(s, 4)))
            p = oracle.projection(s, [P(s, 0), P(s, 1), P(s, 2), P(s, 3), dp,
                                      A(O.Multiplication, dp, A(O.Addition, V(1), P(s, 5))), P(s, 4)])
            return oracle.aggregate(p, aggs, [0, 1])

        oracle.set_threads(n_threads)
        times = []
        for _ in range(runs + 1):
            t0 = time.perf_counter()
            agg = run()
            times.append(time.perf_counter() - t0)
        oracle.set_threads(1)
        med = sorted(times[1:])[len(times[1:]) // 2]
        out[label] = {"value": round(t.row_count() / med, 1), "cores": n_threads, "median_s": round(med, 3),
                      "runs_s": [round(x, 3) for x in times[1:]],
                      "sample": f"SF{sample_sf:g}: {t.row_count()} lineitem rows, {agg.row_count()} groups"}
        del t, agg
    out["value"], out["cores"] = out["all_cores"]["value"], out["all_cores"]["cores"]
    out["sample"] = out["all_cores"]["sample"] + f"; median of {runs}"
    return out
