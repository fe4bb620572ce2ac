"""TPC-H 3 on N GPUs through the distributed JoinHash's radix shuffle (BASELINE.json configs[4]).

Every rank holds contiguous chunk ranges of customer, orders and lineitem (strong scaling: the SF database split over
the ranks; no co-partitioning is assumed - lineitem's shard is independent of the orders shard). One step is the
reference's plan (tpch_queries.cpp:101-106) distributed:

    A  TableScan(customer shard, c_mktsegment = 'BUILDING') -> the matches' c_custkey        hy_table_scan_row_ids +
                                                                                           hy_projection
       all_gather of those keys (3M at SF100: the small dimension side is broadcast)
    B  JoinHash(<all customer matches>, TableScan(orders shard, o_orderdate < 1995-03-15))  hy_scan_join_hash, local:
       c_custkey = o_custkey; the orders scan runs inside the join's first radix pass         every orders row is on
                                                                                           this rank
       all_reduce of the join's pairs -> radix bits of the next join from its GLOBAL build size (join_hash.cpp:640-668)
    C  step 1 of the distributed JoinHash o_orderkey = l_orderkey:
         build: the join-B output (PosLists into this rank's orders) dereferenced, hy_scan_join_exchange_partition
                -> 8-byte records {o_orderkey, orders row}; carried: o_orderdate, o_shippriority in record order
                (hy_exchange_record_row_ids + hy_projection)
         probe: lineitem shard with TableScan(l_shipdate > 1995-03-15) fused, -> records {l_orderkey, lineitem row};
                carried: l_extendedprice * (1 - l_discount) (the projection's expression, evaluated by the row's owner)
       exchange: all_gather of the bucket counts, one all_to_all per array (RCCL over xGMI with --dist-backend nccl)
    D  step 2 on the receiver: hy_exchange_records_localize (payload := position in the receive buffer, probe keys
       saved), hy_join_exchange_join_rows over the rank's radix partitions with uniform 64k-row chunks over the receive
       buffers, Projection(l_orderkey, o_orderdate, o_shippriority, revenue) through the join's PosLists into the
       received arrays, Aggregate(GROUP BY l_orderkey, o_orderdate, o_shippriority; SUM(revenue)) - local: every row
       of an l_orderkey is in the partition the rank owns, so the ranks' groups are disjoint and their union is the
       single-node result.

Timing: barrier + synchronize around K steps, the max over ranks; rows = customer + orders + lineitem of the whole
database. The result is checked against torch on the full columns (every rank regenerates them for the check).
"""
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
RECV_CHUNK = 65536  # rows per chunk of the receive-side tables (the received records' positions map to RowIDs)


def _value_chunks(capi, t, n, chunk, width):
    n_chunks = (n + chunk - 1) // chunk
    arr = (capi.ColumnChunk * max(1, n_chunks))()
    for c in range(n_chunks):
        arr[c].data = t.data_ptr() + width * c * chunk
        arr[c].size = min(chunk, n - c * chunk)
        arr[c].kind = capi.HY_COL_VALUE
    return arr, n_chunks


def _layout(n, chunk):
    sizes = [chunk] * (n // chunk) + ([n % chunk] if n % chunk else [])
    return np.ascontiguousarray(np.asarray(sizes, dtype=np.uint32))


class Q3Rank:
    """One rank's shard of TPC-H 3's tables and the C-ABI calls of its steps (a torch device holds the buffers)."""

    def __init__(self, hy, torch, synth, cols, chunk, dev, stream):
        import bench_tpch as bt

        self.hy, self.capi, self.L, self.torch = hy, hy.capi, hy.capi.lib, torch
        self.chunk, self.dev, self.stream = chunk, dev, stream
        capi = self.capi
        I32 = capi.HY_TYPE_INT32
        D = synth.DATE_1995_03_15
        pad = lambda t: torch.cat([t.contiguous(), torch.zeros(64, dtype=t.dtype, device=dev)])
        self.seg = bt.DictColumn(torch, synth, capi, cols["c_mktsegment"], chunk, 0, 5)
        self.odate = bt.DictColumn(torch, synth, capi, cols["o_orderdate"], chunk, synth.DATE_1992_01_01,
                                   synth.DATE_1998_08_02 - synth.DATE_1992_01_01 + 1)
        self.ship = bt.DictColumn(torch, synth, capi, cols["l_shipdate"], chunk, synth.DATE_1992_01_01,
                                  synth.DATE_1998_08_02 + 121 - synth.DATE_1992_01_01 + 1)
        self.ckey, self.ocust, self.okey = (pad(cols[k]) for k in ("c_custkey", "o_custkey", "o_orderkey"))
        self.oprio, self.lkey = pad(cols["o_shippriority"]), pad(cols["l_orderkey"])
        self.price, self.disc = pad(cols["l_extendedprice"]), pad(cols["l_discount"])
        self.ckey_c, self.ocust_c, self.okey_c = (bt.value_chunks(capi, t, chunk, 4)
                                                  for t in (self.ckey, self.ocust, self.okey))
        self.oprio_c, self.lkey_c, self.price_c, self.disc_c = (bt.value_chunks(capi, t, chunk, 4)
                                                                for t in (self.oprio, self.lkey, self.price, self.disc))
        self.n_cust, self.n_ord, self.n_li = (cols[k].numel() for k in ("c_custkey", "o_orderkey", "l_orderkey"))
        self.n_cc, self.n_oc, self.n_lc = len(self.ckey_c), len(self.okey_c), len(self.lkey_c)
        self.o_layout = np.ascontiguousarray([c.size for c in self.okey_c], dtype=np.uint32)
        self.l_layout = np.ascontiguousarray([c.size for c in self.lkey_c], dtype=np.uint32)
        # fixed descriptors
        self.cscan = self.seg.scan_chunks(capi, "Equals", 1)
        for c in range(self.n_cc):
            self.cscan[c].out_begin = c * chunk
        self.c_ids = (ctypes.c_uint32 * max(1, self.n_cc))(*range(self.n_cc))
        self.c_rows = torch.empty(2 * self.n_cust + 64, dtype=torch.int32, device=dev)
        self.c_counts = torch.empty(max(1, self.n_cc), dtype=torch.int32, device=dev)
        self.orders_side = bt.data_side(capi, self.ocust_c, I32)
        self.li_side = bt.data_side(capi, self.lkey_c, I32)
        self.o_off = torch.empty(self.n_ord + 64, dtype=torch.int32, device=dev)
        self.o_begin = torch.zeros(self.n_oc + 1, dtype=torch.int64, device=dev)
        self.ofilter = capi.JoinFilter(self.odate.scan_chunks(capi, "LessThan", D), I32, None, self.o_off.data_ptr(),
                                       self.o_begin.data_ptr())
        self.l_off = torch.empty(self.n_li + 64, dtype=torch.int32, device=dev)
        self.l_begin = torch.zeros(self.n_lc + 1, dtype=torch.int64, device=dev)
        self.lfilter = capi.JoinFilter(self.ship.scan_chunks(capi, "GreaterThan", D), I32, None,
                                       self.l_off.data_ptr(), self.l_begin.data_ptr())
        self._ws = {}
        self.stats = {}

    # ---- small helpers ----
    def _buf(self, key, n, dtype):
        t = self._ws.get(key)
        if t is None or t.numel() < n or t.dtype != dtype:
            t = self.torch.empty(max(n, 16), dtype=dtype, device=self.dev)
            self._ws[key] = t
        return t

    def _workspace(self, key, query):
        b = ctypes.c_size_t(0)
        self.capi.check(query(ctypes.byref(b)), f"workspace size {key}")
        return self._buf(("ws", key if isinstance(key, str) else key[0]), b.value, self.torch.uint8)

    def _project(self, agg_input, programs, n, dtypes, tag):
        """hy_projection of each program over agg_input into new arrays of n rows."""
        capi, L = self.capi, self.L
        ws = self._workspace(("proj", tag), lambda b: L.hy_projection_workspace_size(ctypes.byref(agg_input), b))
        outs = []
        for j, prog in enumerate(programs):
            out = self._buf((tag, j), n + 64, dtypes[j])
            if n:
                capi.check(L.hy_projection(ctypes.byref(agg_input), prog, len(prog), out.data_ptr(), None,
                                           ws.data_ptr(), ws.numel(), self.stream), "hy_projection " + tag)
            outs.append(out[:n])
        return outs

    def _col(self, vtype, group, chunks, n_chunks):
        c = self.capi.AggColumn()
        c.value_type, c.pos_group, c.chunks, c.n_chunks = vtype, group, chunks, n_chunks
        return c

    def _prog(self, nodes):
        return (self.capi.ExprNode * len(nodes))(*nodes)

    def _colref(self, i, vtype):
        return self.capi.ExprNode(self.capi.HY_EXPR_COLUMN, vtype, 0, i, 0)

    # ---- A: customer scan -> keys of the matches (scan order) ----
    def customer_keys(self):
        capi, L, torch = self.capi, self.L, self.torch
        I32 = capi.HY_TYPE_INT32
        ws = self._workspace("cscan", lambda b: L.hy_table_scan_workspace_size(
            (ctypes.c_uint32 * max(1, self.n_cc))(*self.seg.sizes), self.n_cc, b))
        if self.n_cc:
            capi.check(L.hy_table_scan_row_ids(self.cscan, self.n_cc, I32, None, self.c_ids, self.c_rows.data_ptr(),
                                               self.c_counts.data_ptr(), ws.data_ptr(), ws.numel(), self.stream),
                       "customer scan")
        cc = self.c_counts[: self.n_cc].cpu().numpy().astype(np.int64)
        nz = np.nonzero(cc)[0]
        n = int(cc.sum())
        sizes = np.ascontiguousarray(cc[nz], dtype=np.uint32)
        pls = np.ascontiguousarray(self.c_rows.data_ptr() + 8 * self.chunk * nz.astype(np.uint64))
        cols = (capi.AggColumn * 1)(self._col(I32, 0, self.ckey_c, self.n_cc))
        ain = capi.AggInput(len(nz), sizes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                            pls.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p)), 1, cols, 1)
        ain._keep = (sizes, pls, cols)
        (keys,) = self._project(ain, [self._prog([self._colref(0, I32)])], n, [torch.int32], "ckeys")
        self.stats["customer_matches"] = n
        return keys

    # ---- B: JoinHash(all customer matches, orders shard with its scan fused), local ----
    def join1(self, cust_keys):
        capi, L, torch = self.capi, self.L, self.torch
        I32 = capi.HY_TYPE_INT32
        n_b = cust_keys.numel()
        gk = self._buf("gk", n_b + 64, torch.int32)
        gk[:n_b].copy_(cust_keys)
        gk_c, n_gc = _value_chunks(capi, gk, n_b, RECV_CHUNK, 4)
        arr = (capi.JoinChunk * max(1, n_gc))()
        for c in range(n_gc):
            arr[c].column, arr[c].size, arr[c].chunk_id = gk_c[c], gk_c[c].size, c
            arr[c].single_chunk = capi.HY_MIXED_CHUNKS
        build = capi.JoinSide(arr, n_gc, I32, None, 0, 0, 0)
        bits = L.hy_join_radix_bits(n_b, 4)
        params = capi.JoinParams(capi.HY_JOIN_INNER, I32, bits, 17)
        ws = self._workspace(("j1", bits, n_gc), lambda b: L.hy_scan_join_hash_workspace_size(
            ctypes.byref(build), None, ctypes.byref(self.orders_side), ctypes.byref(self.ofilter), ctypes.byref(params),
            b))
        pb = self._buf(("j1pb", bits), 1 << bits, torch.int64)
        pc = self._buf(("j1pc", bits), 1 << bits, torch.int32)
        cap = self.stats.get("j1cap", self.n_ord // 4 + 64)
        while True:
            ob, op = self._buf("j1b", 2 * cap, torch.int32), self._buf("j1p", 2 * cap, torch.int32)
            res = capi.JoinResult()
            st = L.hy_scan_join_hash(ctypes.byref(build), None, ctypes.byref(self.orders_side),
                                     ctypes.byref(self.ofilter), ctypes.byref(params), ob.data_ptr(), op.data_ptr(),
                                     cap, pb.data_ptr(), pc.data_ptr(), ctypes.byref(res), ws.data_ptr(), ws.numel(),
                                     self.stream)
            if st != capi.HY_ERR_CAPACITY:
                capi.check(st, "join 1")
                break
            cap = self.stats["j1cap"] = res.capacity_required + 64
        pb_h, pc_h = pb[: 1 << bits].cpu().numpy(), pc[: 1 << bits].cpu().numpy()
        nz = np.nonzero(pc_h)[0]
        self.j1 = (op, pb_h[nz], pc_h[nz].astype(np.uint32))
        self.stats["join1_pairs"] = int(res.total_pairs)
        self.stats["orders_matches"] = int(self.o_begin[self.n_oc].item())
        return int(res.total_pairs)

    # ---- C: step 1 of the distributed join, both sides, with the carried columns ----
    def partition2(self, bits, world):
        capi, L, torch = self.capi, self.L, self.torch
        I32, F32 = capi.HY_TYPE_INT32, capi.HY_TYPE_FLOAT
        self.params2 = capi.JoinParams(capi.HY_JOIN_INNER, I32, bits, 17)
        self.nb_total = 1 << L.hy_join_exchange_bucket_bits(bits, world)
        op, begins, counts = self.j1
        arr = np.zeros(len(counts), np.dtype(capi.JoinChunk))
        arr["pos_list"] = op.data_ptr() + 8 * begins.astype(np.uint64)
        arr["size"] = counts
        arr["chunk_id"] = np.arange(len(counts), dtype=np.uint32)
        arr["single_chunk"] = capi.HY_MIXED_CHUNKS
        build = capi.JoinSide(arr.ctypes.data_as(ctypes.POINTER(capi.JoinChunk)), len(counts), I32, self.okey_c,
                              self.n_oc, 1, 0)
        out = []
        for tag, side, filt, n_max in (("b", build, None, int(counts.sum())), ("p", self.li_side, self.lfilter,
                                                                               self.n_li)):
            fp = ctypes.byref(filt) if filt is not None else None
            ws = self._workspace(("x" + tag, len(counts) if tag == "b" else 0), lambda b: L.hy_scan_join_exchange_partition_workspace_size(
                ctypes.byref(side), fp, ctypes.byref(self.params2), world, b))
            recs = self._buf("xrec" + tag, n_max + 64, torch.int64)
            cnt = (ctypes.c_uint64 * self.nb_total)()
            capi.check(L.hy_scan_join_exchange_partition(ctypes.byref(side), fp, ctypes.byref(self.params2), 0, world,
                                                         0, recs.data_ptr(), cnt, ws.data_ptr(), ws.numel(),
                                                         self.stream), "exchange partition " + tag)
            cnt = np.frombuffer(cnt, np.uint64).astype(np.int64).copy()
            n = int(cnt.sum())
            # the carried columns, evaluated by the rows' owner in record order
            rows = self._buf("xrid" + tag, 2 * n + 64, torch.int32)
            layout = self.o_layout if tag == "b" else self.l_layout
            if n:
                capi.check(L.hy_exchange_record_row_ids(recs.data_ptr(), n, 8, 0, layout.ctypes.data, layout.size,
                                                        rows.data_ptr(), self.stream), "record row ids")
            sizes = np.array([n], np.uint32)
            pls = np.array([rows.data_ptr()], np.uint64)
            if tag == "b":
                cols = (capi.AggColumn * 2)(self._col(I32, 0, self.odate.desc, self.n_oc),
                                            self._col(I32, 0, self.oprio_c, self.n_oc))
                progs = [self._prog([self._colref(0, I32)]), self._prog([self._colref(1, I32)])]
                dts = [torch.int32, torch.int32]
            else:
                cols = (capi.AggColumn * 2)(self._col(F32, 0, self.price_c, self.n_lc),
                                            self._col(F32, 0, self.disc_c, self.n_lc))
                N = capi.ExprNode
                progs = [self._prog([self._colref(0, F32), N(capi.HY_EXPR_VALUE, I32, 0, 0, 1), self._colref(1, F32),
                                     N(capi.HY_EXPR_SUB, F32, F32, 0, 0), N(capi.HY_EXPR_MUL, F32, F32, 0, 0)])]
                dts = [torch.float32]
            ain = capi.AggInput(1, sizes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                pls.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p)), 1, cols, 2)
            attrs = self._project(ain, progs, n, dts, "x" + tag)
            out.append(([recs[:n]] + attrs, cnt))
        self.stats["lineitem_matches"] = int(self.l_begin[self.n_lc].item())
        return out

    # ---- D: step 2 on the receiver, projection, aggregate ----
    def join2(self, bcols, bmat, pcols, pmat, rank, world):
        capi, L, torch = self.capi, self.L, self.torch
        I32, F32 = capi.HY_TYPE_INT32, capi.HY_TYPE_FLOAT
        import importlib as il

        hd = il.import_module("hyrise-1_amd.dist")
        brec, odate_r, oprio_r = bcols
        prec, rev_r = pcols
        n_b, n_p = brec.numel(), prec.numel()
        lkey_r = self._buf("lkey_r", n_p + 64, torch.int32)
        capi.check(L.hy_exchange_records_localize(brec.data_ptr(), n_b, 8, None, None, self.stream), "localize b")
        capi.check(L.hy_exchange_records_localize(prec.data_ptr(), n_p, 8, lkey_r.data_ptr(), None, self.stream),
                   "localize p")
        first, last = hd.owned_buckets(self.nb_total, rank, world)
        nb = last - first
        bc = np.ascontiguousarray(bmat, dtype=np.uint64)
        pc = np.ascontiguousarray(pmat, dtype=np.uint64)
        bcp, pcp = (m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)) for m in (bc, pc))
        bl, pl = _layout(n_b, RECV_CHUNK), _layout(n_p, RECV_CHUNK)
        blp = bl.ctypes.data if bl.size else None
        plp = pl.ctypes.data if pl.size else None
        ws = self._workspace(("j2", n_b, n_p), lambda b: L.hy_join_exchange_join_rows_workspace_size(
            bcp, pcp, world, nb, ctypes.byref(self.params2), blp, bl.size, plp, pl.size, b))
        bits = self.params2.radix_bits
        n_parts = nb << (bits - L.hy_join_exchange_bucket_bits(bits, world))
        pbeg = self._buf("j2pb", max(1, n_parts), torch.int64)
        pcnt = self._buf("j2pc", max(1, n_parts), torch.int32)
        cap = max(16, n_p + 16)
        while True:
            ob, op = self._buf("j2b", 2 * cap, torch.int32), self._buf("j2p", 2 * cap, torch.int32)
            res = capi.JoinResult()
            st = L.hy_join_exchange_join_rows(brec.data_ptr(), bcp, prec.data_ptr(), pcp, world, first, nb,
                                              ctypes.byref(self.params2), blp, bl.size, plp, pl.size, ob.data_ptr(),
                                              op.data_ptr(), cap, pbeg.data_ptr(), pcnt.data_ptr(), ctypes.byref(res),
                                              ws.data_ptr(), ws.numel(), self.stream)
            if st != capi.HY_ERR_CAPACITY:
                capi.check(st, "join 2")
                break
            cap = res.capacity_required + 16
        pairs = int(res.total_pairs)
        pb_h, pc_h = pbeg[:n_parts].cpu().numpy(), pcnt[:n_parts].cpu().numpy()
        nz = np.nonzero(pc_h)[0]
        k = len(nz)
        sizes = np.ascontiguousarray(pc_h[nz], dtype=np.uint32)
        b2 = pb_h[nz].astype(np.uint64)
        pls = np.ascontiguousarray(np.concatenate([ob.data_ptr() + 8 * b2, op.data_ptr() + 8 * b2]))
        # the received tables: uniform RECV_CHUNK-row chunks over the received arrays
        lk_c, n1 = _value_chunks(capi, lkey_r, n_p, RECV_CHUNK, 4)
        od_c, n2 = _value_chunks(capi, odate_r, n_b, RECV_CHUNK, 4)
        op_c, _ = _value_chunks(capi, oprio_r, n_b, RECV_CHUNK, 4)
        rv_c, _ = _value_chunks(capi, rev_r, n_p, RECV_CHUNK, 4)
        cols = (capi.AggColumn * 4)(self._col(I32, 1, lk_c, n1), self._col(I32, 0, od_c, n2),
                                    self._col(I32, 0, op_c, n2), self._col(F32, 1, rv_c, n1))
        ain = capi.AggInput(k, sizes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                            pls.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p)), 2, cols, 4)
        ain._keep = (sizes, pls, cols, lk_c, od_c, op_c, rv_c)
        progs = [self._prog([self._colref(j, t)]) for j, t in enumerate((I32, I32, I32, F32))]
        proj = self._project(ain, progs, pairs, [torch.int32, torch.int32, torch.int32, torch.float32], "proj2")
        # Aggregate over the projection's output (a data table with the join output's chunking)
        rb = np.concatenate([[0], np.cumsum(sizes.astype(np.int64))])[:-1].astype(np.uint64)
        acols = (capi.AggColumn * 4)()
        keep = []
        cc_dtype = np.dtype(capi.ColumnChunk)
        for j, vt in enumerate([I32, I32, I32, F32]):
            ch = np.zeros(max(1, k), cc_dtype)
            ch["data"][:k] = proj[j].data_ptr() + 4 * rb
            ch["size"][:k] = sizes
            ch["kind"] = capi.HY_COL_VALUE
            keep.append(ch)
            acols[j].value_type, acols[j].pos_group, acols[j].n_chunks = vt, -1, k
            acols[j].chunks = ch.ctypes.data_as(ctypes.POINTER(capi.ColumnChunk))
        agg_in = capi.AggInput(k, sizes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), None, 0, acols, 4)
        groupby = (ctypes.c_int32 * 3)(0, 1, 2)
        agg_defs = (capi.AggDef * 1)(capi.AggDef(capi.HY_AGG_SUM, 3))
        prm = capi.AggParams(groupby, 3, agg_defs, 1, self.stats.get("group_bound", 0))
        if "layout" not in self.stats:
            lay = capi.AggLayout()
            capi.check(L.hy_aggregate_layout(ctypes.byref(agg_in), ctypes.byref(prm), ctypes.byref(lay)), "layout")
            self.stats["layout"] = lay
        words = self.stats["layout"].words
        agg_out = self._buf("agg_out", (pairs + 1) * words, torch.int64)
        ng = ctypes.c_uint64(0)
        while True:
            aws = self._workspace(("agg", k, pairs, prm.group_bound), lambda b: L.hy_aggregate_workspace_size(
                ctypes.byref(agg_in), ctypes.byref(prm), b))
            st = L.hy_aggregate(ctypes.byref(agg_in), ctypes.byref(prm), agg_out.data_ptr(), pairs + 1,
                                ctypes.byref(ng), aws.data_ptr(), aws.numel(), self.stream)
            if st != capi.HY_ERR_GROUP_BOUND:
                break
            prm.group_bound = self.stats["group_bound"] = ng.value
        capi.check(st, "hy_aggregate")
        self.stats["join2_pairs"] = pairs
        self.stats["groups"] = int(ng.value)
        self.agg = agg_out
        return int(ng.value)

    def group_records(self):
        lay = self.stats["layout"]
        return self.agg.view(-1, lay.words)[: self.stats["groups"]].cpu().numpy().view(np.uint64)


def shard_q3(cols, chunk, rank, world):
    """Rank r's contiguous chunk ranges of each table (independently per table)."""
    out = {}
    for prefix, keys in (("c_", ("c_custkey", "c_mktsegment")),
                         ("o_", ("o_orderkey", "o_custkey", "o_orderdate", "o_shippriority")),
                         ("l_", ("l_orderkey", "l_shipdate", "l_extendedprice", "l_discount"))):
        n = cols[keys[0]].numel()
        n_chunks = (n + chunk - 1) // chunk
        lo, hi = min(n, rank * n_chunks // world * chunk), min(n, (rank + 1) * n_chunks // world * chunk)
        for k in keys:
            out[k] = cols[k][lo:hi].contiguous()
    return out


def q3_step(ranks, rank_ids, world, gather_keys, allreduce_sum, exchange):
    """One distributed TPC-H 3 step for the given rank objects (one per process, or all of them when the ranks are
    simulated in one process): the collectives are callables so that the same plan runs over torch.distributed and
    in-process. Returns the local group counts."""
    keys = [r.customer_keys() for r in ranks]
    all_keys = gather_keys(keys)
    pairs1 = [r.join1(all_keys) for r in ranks]
    # the reference's formula on the GLOBAL build size; at least one bit per doubling of the ranks (tiny inputs: the
    # formula may give 0 bits, one partition, which the exchange cannot split)
    bits2 = max(ranks[0].L.hy_join_radix_bits(allreduce_sum(sum(pairs1)), 4), max(1, (world - 1).bit_length()))
    parts = [r.partition2(bits2, world) for r in ranks]
    recv = exchange(parts)  # per local rank: ((build cols, bmat), (probe cols, pmat))
    return [r.join2(b[0], b[1], p[0], p[1], rid, world) for r, rid, (b, p) in zip(ranks, rank_ids, recv)]


def run_in_process(hy, torch, synth, cols, chunk, world, dev, stream):
    """All N ranks of the distributed plan in one process on one GPU (tests): exchanges are device copies."""
    hd = importlib.import_module("hyrise-1_amd.dist")
    ranks = [Q3Rank(hy, torch, synth, shard_q3(cols, chunk, r, world), chunk, dev, stream) for r in range(world)]

    def exchange(parts):
        out = []
        for side in (0, 1):
            per_rank = hd.exchange_columns_in_process([p[side][0] for p in parts], [p[side][1] for p in parts])
            out.append(per_rank)
        return [((out[0][r][0], out[0][r][1]), (out[1][r][0], out[1][r][1])) for r in range(world)]

    q3_step(ranks, list(range(world)), world, lambda ks: torch.cat(ks), lambda x: x, exchange)
    return ranks


def main_q3_dist(args):
    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    hy = importlib.import_module("hyrise-1_amd")
    synth = importlib.import_module("hyrise-1_amd.synth")
    hd = importlib.import_module("hyrise-1_amd.dist")
    capi = hy.capi
    L = capi.lib
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    nccl = args.dist_backend == "nccl"
    if nccl:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group("gloo")
    dev = torch.device("cuda", torch.cuda.current_device())
    xdev = dev if nccl else torch.device("cpu")
    capi.check(L.hy_set_device(dev.index), "hy_set_device")
    stream = torch.cuda.current_stream().cuda_stream
    chunk = args.chunk
    D = synth.DATE_1995_03_15

    # the whole database (every rank regenerates it: the expected result), then this rank's shard
    cols = synth.q3_columns(args.sf, dev)
    n_cust, n_ord, n_li = (cols[k].numel() for k in ("c_custkey", "o_orderkey", "l_orderkey"))
    seg_ok = cols["c_mktsegment"] == 1
    o_date_ok = cols["o_orderdate"] < D
    o_ok = o_date_ok & seg_ok[cols["o_custkey"].long() - 1]
    l_date_ok = cols["l_shipdate"] > D
    l_ok = l_date_ok & o_ok[cols["l_order_index"]]
    exp = {"customer_matches": int(seg_ok.sum()), "orders_matches": int(o_date_ok.sum()),
           "lineitem_matches": int(l_date_ok.sum()), "join1_pairs": int(o_ok.sum()), "join2_pairs": int(l_ok.sum())}
    rev = cols["l_extendedprice"] * (1 - cols["l_discount"])
    order_rev = torch.zeros(n_ord, dtype=torch.float64, device=dev).index_add_(
        0, cols["l_order_index"][l_ok], rev[l_ok].to(torch.float64))
    order_hit = torch.zeros(n_ord, dtype=torch.bool, device=dev)
    order_hit[cols["l_order_index"][l_ok]] = True
    exp["groups"] = int(order_hit.sum())
    del seg_ok, o_date_ok, o_ok, l_date_ok, l_ok, rev, order_hit
    shard = shard_q3(cols, chunk, rank, world)
    del cols
    torch.cuda.empty_cache()
    r = Q3Rank(hy, torch, synth, shard, chunk, dev, stream)
    del shard
    torch.cuda.synchronize()

    def gather_keys(keys):
        (k,) = keys
        n = torch.tensor([k.numel()], dtype=torch.int64, device=xdev)
        ns = [torch.empty_like(n) for _ in range(world)]
        dist.all_gather(ns, n)
        ns = [int(x.item()) for x in ns]
        m = max(ns)
        buf = torch.zeros(max(1, m), dtype=torch.int32, device=xdev)
        buf[: k.numel()].copy_(k)
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf)
        return torch.cat([p[:c] for p, c in zip(parts, ns)]).to(dev)

    def allreduce_sum(x):
        t = torch.tensor([x], dtype=torch.int64, device=xdev)
        dist.all_reduce(t)
        return int(t.item())

    def exchange(parts):
        (p,) = parts
        out = []
        for cols_, cnt in p:
            got, mat = hd.exchange_columns(dist, [c.to(xdev) for c in cols_], cnt, rank, world)
            out.append(([g.to(dev) for g in got], mat))
        return [tuple(out)]

    def step():
        q3_step([r], [rank], world, gather_keys, allreduce_sum, exchange)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
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
    t = torch.tensor([elapsed], dtype=torch.float64, device=xdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    keys = ["orders_matches", "lineitem_matches", "join2_pairs", "groups"]
    v = torch.tensor([r.stats[k] for k in keys], dtype=torch.int64, device=xdev)
    dist.all_reduce(v)
    got = {k: int(x) for k, x in zip(keys, v.tolist())}
    got["customer_matches"] = allreduce_sum(r.stats["customer_matches"])
    got["join1_pairs"] = allreduce_sum(r.stats["join1_pairs"])
    # every local group: its key's order, and its SUM exactly (the order's revenue is a sum of <= 7 float products,
    # exact in double); a sample of 2000 per rank
    rec = r.group_records()
    lay = r.stats["layout"]
    ok = got == exp
    rng = np.random.default_rng(3 + rank)
    sample = rng.choice(rec.shape[0], size=min(2000, rec.shape[0]), replace=False) if rec.shape[0] else []
    order_rev_h = order_rev.cpu().numpy()
    w = lay.agg_word[0]
    for g in sample:
        row = rec[g]
        key = int(np.int32(np.uint32(row[0])))
        oi = ((key >> 5) << 3) + (key & 7) - 1  # inverse of the dbgen sparse order key
        limbs = (ctypes.c_uint64 * lay.agg_limbs[0])(*[int(x) for x in row[w + 2:w + 2 + lay.agg_limbs[0]]])
        s = ctypes.c_double(0)
        capi.check(L.hy_agg_float_sum(limbs, lay.agg_limbs[0], lay.agg_emin[0], int(row[w + 1]), ctypes.byref(s)))
        ok &= s.value == order_rev_h[oi]
    okt = torch.tensor([1 if ok else 0], dtype=torch.int64, device=xdev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    ok = bool(okt.item())
    if not ok:
        raise SystemExit(f"q3 (distributed) result mismatch on rank {rank}: {got} vs {exp}")
    from bench import kernel_stats  # noqa: E402

    kernels = kernel_stats(L)
    if rank == 0:
        K = args.steps
        step_s = elapsed / K
        line = {
            "metric": "rows/sec TPC-H 3 (Scan -> JoinHash -> JoinHash -> Projection -> Aggregate), 1/2/4/8 MI355X",
            "value": round((n_cust + n_ord + n_li) / step_s, 1), "unit": "rows/s", "n_gpus": world, "steps": K,
            "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "int32/f32",
            "data": "synthetic (seeded counter-based TPC-H-shaped columns, resident in HBM)",
            "config": {"workload": "TPC-H 3 (tpch_queries.cpp:101-106) without ORDER BY/LIMIT", "sf": args.sf,
                       "customer_rows": n_cust, "orders_rows": n_ord, "lineitem_rows": n_li, "chunk_size": chunk,
                       **got, "parallelism": f"chunk-sharded x{world}: customer matches all-gathered (broadcast join "
                                             f"with the local orders), orders ⋈ lineitem through the "
                                             f"{'RCCL' if nccl else 'gloo'} radix shuffle with the projection's "
                                             f"columns carried, GROUP BY l_orderkey local after the shuffle"},
            "check": {"ok": ok, "expected": exp, "sampled_groups_rank0": len(sample)},
            "kernels_rank0": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v_.items()}
                              for k, v_ in kernels.items()},
            "cpu_baseline": None,
        }
        print(json.dumps(line))
    dist.destroy_process_group()


def _selftest(world, sf, chunk, out_path):
    """Runs the distributed plan with `world` ranks simulated on GPU 0 and saves every rank's groups (keys and the
    exactly rounded SUM) and join sizes to out_path (.npz). torch is imported before the library, so that both use
    one HIP runtime (tests/test_dist_q3_gpu.py runs this in a child process)."""
    import torch

    sys.path.insert(0, ROOT)
    hy = importlib.import_module("hyrise-1_amd")
    synth = importlib.import_module("hyrise-1_amd.synth")
    capi, L = hy.capi, hy.capi.lib
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    capi.check(L.hy_set_device(0), "hy_set_device")
    stream = torch.cuda.current_stream().cuda_stream
    cols = synth.q3_columns(sf, dev)
    cols.pop("l_order_index")
    ranks = run_in_process(hy, torch, synth, cols, chunk, world, dev, stream)
    torch.cuda.synchronize()
    keys, sums, owner = [], [], []
    for i, r in enumerate(ranks):
        lay = r.stats["layout"]
        w = lay.agg_word[0]
        for row in r.group_records():
            keys.append([int(np.int32(np.uint32(row[j]))) for j in range(3)])
            limbs = (ctypes.c_uint64 * lay.agg_limbs[0])(*[int(x) for x in row[w + 2:w + 2 + lay.agg_limbs[0]]])
            s = ctypes.c_double(0)
            capi.check(L.hy_agg_float_sum(limbs, lay.agg_limbs[0], lay.agg_emin[0], int(row[w + 1]), ctypes.byref(s)))
            sums.append(s.value)
            owner.append(i)
    np.savez(out_path, keys=np.array(keys, np.int64).reshape(-1, 3), sums=np.array(sums, np.float64),
             owner=np.array(owner, np.int64), join1=sum(r.stats["join1_pairs"] for r in ranks),
             join2=sum(r.stats["join2_pairs"] for r in ranks))


if __name__ == "__main__":
    if len(sys.argv) == 6 and sys.argv[1] == "--selftest":
        _selftest(int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
    else:
        raise SystemExit("usage: bench_q3_dist.py --selftest WORLD SF CHUNK OUT.npz (the bench runs through bench.py)")
