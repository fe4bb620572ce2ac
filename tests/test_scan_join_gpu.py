"""Fused TableScan -> JoinHash (hy_scan_join_hash) against the oracle's TableScan followed by its JoinHash on the scan
output (reference table_scan.cpp:78-164 then join_hash.cpp:49-858 + write_output_columns :564-613): the scan's
per-chunk offset lists, and every partition's build / probe PosLists RowID for RowID, for value and dictionary
predicate columns, NULLs in the predicate and join columns, filters on either or both sides and every join mode."""
import ctypes
import zlib

import numpy as np
import pytest

import device_tables as dt
from helpers import wrap

pytestmark = pytest.mark.gpu


def orders_lineitem(rng, n_orders, key_nulls):
    i = np.arange(1, n_orders + 1, dtype=np.int64)
    okey = (((i >> 3) << 5) + (i & 7)).astype(np.int32)  # dbgen sparse order keys (build.c)
    okey = np.concatenate([okey, okey[rng.integers(0, n_orders, n_orders // 9)]])  # duplicate build keys
    lkey = np.repeat(okey[:n_orders], rng.integers(1, 8, n_orders))
    lkey = np.concatenate([lkey, rng.integers(-500, 0, lkey.size // 40).astype(np.int32)])  # unmatched probe rows
    rng.shuffle(lkey)
    lkey = lkey.astype(np.int32)
    qty = rng.integers(1, 51, lkey.size).astype(np.float32)
    qty_nulls = (rng.random(lkey.size) < 0.02).astype(np.uint8)
    lkey_nulls = (rng.random(lkey.size) < 0.03).astype(np.uint8) if key_nulls else None
    ostatus = rng.integers(0, 10, okey.size).astype(np.int32)
    return okey, ostatus, lkey, lkey_nulls, qty, qty_nulls


def run_fused(hy, build, bfilt, probe, pfilt, params, cap):
    capi, L = hy.capi, hy.capi.lib
    wsb = ctypes.c_size_t()
    bf = ctypes.byref(bfilt) if bfilt is not None else None
    pf = ctypes.byref(pfilt) if pfilt is not None else None
    capi.check(L.hy_scan_join_hash_workspace_size(ctypes.byref(build), bf, ctypes.byref(probe), pf,
                                                  ctypes.byref(params), ctypes.byref(wsb)), "ws")
    ws = capi.DeviceArray(np.zeros(wsb.value, np.uint8))
    ob, op = capi.DeviceArray(np.zeros(cap * 2, np.uint32)), capi.DeviceArray(np.zeros(cap * 2, np.uint32))
    n_parts = 1 << params.radix_bits
    pbeg, pcnt = capi.DeviceArray(np.zeros(n_parts, np.uint64)), capi.DeviceArray(np.zeros(n_parts, np.uint32))
    res = capi.JoinResult()
    capi.check(L.hy_scan_join_hash(ctypes.byref(build), bf, ctypes.byref(probe), pf, ctypes.byref(params), ob.ptr,
                                   op.ptr, cap, pbeg.ptr, pcnt.ptr, ctypes.byref(res), ws.ptr, wsb.value, None),
               "hy_scan_join_hash")
    ob, op = ob.fetch().reshape(-1, 2), op.fetch().reshape(-1, 2)
    return [(ob[b:b + c], op[b:b + c]) for b, c in zip(pbeg.fetch().astype(np.int64), pcnt.fetch().astype(np.int64))]


class Filter:
    """hy_join_filter for `column cond value` on a DeviceColumn, with its output buffers."""

    def __init__(self, capi, col, cond, value, offsets=True, rows=False):
        self.chunks = col.scan_chunks(cond, value)
        self.const = col.constant(value)
        n = max(16, col.values.size)
        self.out = capi.DeviceArray(np.zeros(n, np.uint32))
        self.begin = capi.DeviceArray(np.zeros(col.n_chunks + 1, np.uint64))
        # out_row_ids: the scan's PosLists as RowIDs (pre-filled with a pattern no RowID of the scan takes)
        self.rows = capi.DeviceArray(np.full(n * 2, 0xDEADBEEF, np.uint32)) if rows else None
        self.f = capi.JoinFilter(self.chunks, dt.HY_TYPES[col.values.dtype], self.const.ctypes.data,
                                 self.out.ptr.value if offsets else None, self.begin.ptr.value,
                                 out_row_ids=self.rows.ptr.value if rows else None)

    def scan_output(self):
        beg = self.begin.fetch().astype(np.int64)
        if self.rows is not None:  # the offsets of the RowIDs, whose chunk ids must name their chunk
            rows = self.rows.fetch().reshape(-1, 2)
            for c in range(beg.size - 1):
                assert (rows[beg[c]:beg[c + 1], 0] == c).all(), f"out_row_ids chunk {c}: chunk ids"
            return [rows[beg[c]:beg[c + 1], 1] for c in range(beg.size - 1)]
        off = self.out.fetch()
        return [off[beg[c]:beg[c + 1]] for c in range(beg.size - 1)]


def check_scan(expected_scan, filt):
    """The fused scan's per-chunk offset lists equal the TableScan output chunks (chunks with >= 1 match)."""
    got = [(c, o) for c, o in enumerate(filt.scan_output()) if o.size]
    assert len(got) == expected_scan.chunk_count()
    for k, (c, offs) in enumerate(got):
        pl = expected_scan.get_chunk(k).get_column(0).pos_list()
        assert (pl[:, 0] == c).all(), f"scan output chunk {k}"
        assert np.array_equal(pl[:, 1], offs), f"scan output chunk {k}: offsets differ"


def check_join(expected, parts, build_cols, probe_first, semi_anti):
    """Partition p's PosLists equal output chunk k of the oracle's JoinHash (non-empty partitions, ascending)."""
    nonempty = [(b, p) for b, p in parts if p.shape[0]]
    assert len(nonempty) == expected.chunk_count()
    for k, (b, p) in enumerate(nonempty):
        ch = expected.get_chunk(k)
        pcol = 0 if (probe_first or semi_anti) else build_cols
        assert np.array_equal(ch.get_column(pcol).pos_list(), p), f"partition chunk {k}: probe RowIDs"
        if not semi_anti:
            bcol = (ch.column_count() - build_cols) if probe_first else 0
            assert np.array_equal(ch.get_column(bcol).pos_list(), b), f"partition chunk {k}: build RowIDs"


@pytest.mark.parametrize("mode", ["Inner", "Left", "Right", "Semi", "Anti"])
@pytest.mark.parametrize("qty_enc,key_enc,key_nulls", [("Dictionary", "Unencoded", False),
                                                       ("Unencoded", "Unencoded", True),
                                                       ("Dictionary", "Dictionary", True)])
@pytest.mark.parametrize("build_filter", [False, True])
@pytest.mark.parametrize("bloom", [False, True])
def test_scan_join_matches_operators(hy, oracle, monkeypatch, mode, qty_enc, key_enc, key_nulls, build_filter, bloom):
    monkeypatch.setenv("HY_JOIN_BLOOM", "1" if bloom else "0")  # probe-side Bloom prefilter (INNER / SEMI only)
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(repr((mode, qty_enc, key_enc, key_nulls, build_filter)).encode()))
    okey, ostatus, lkey, lkey_nulls, qty, qty_nulls = orders_lineitem(rng, 40_000, key_nulls)
    lchunk, ochunk = 9_000, 7_000
    lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, key_nulls), ("l_quantity", hy.DataType.Float, True)],
                                    [lkey, qty], [lkey_nulls, qty_nulls], lchunk)
    orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False), ("o_status", hy.DataType.Int, False)],
                                  [okey, ostatus], [], ochunk)
    scan_l = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24.0, [])
    left = oracle.table_scan(orders, 1, hy.PredicateCondition.GreaterThanEquals, 3, []) if build_filter else orders
    jm = getattr(hy.JoinMode, mode)
    expected, bits = oracle.join_hash(left, scan_l, jm, (0, 0))

    lk = dt.DeviceColumn(capi, lkey, lkey_nulls, lchunk, key_enc)
    lq = dt.DeviceColumn(capi, qty, qty_nulls, lchunk, qty_enc)
    ok = dt.DeviceColumn(capi, okey, None, ochunk, "Unencoded")
    os_ = dt.DeviceColumn(capi, ostatus, None, ochunk, "Dictionary")
    lf = Filter(capi, lq, "LessThan", 24.0)
    of = Filter(capi, os_, "GreaterThanEquals", 3) if build_filter else None
    # the reference's swap rule on the scan outputs' row counts (join_hash.cpp:55-76)
    swapped = mode in ("Left", "Semi", "Anti") or left.row_count() > scan_l.row_count()
    o_side, l_side = dt.join_side(capi, ok), dt.join_side(capi, lk)
    o_f, l_f = (of.f if of else None), lf.f
    params = capi.JoinParams({"Inner": 0, "Left": 1, "Right": 2, "Semi": 5, "Anti": 6}[mode], capi.HY_TYPE_INT32, bits,
                             17)
    cap = okey.size * 3 + lkey.size + 16
    if swapped:  # the scan output (left input's role after the swap: build = right input)
        parts = run_fused(hy, l_side, l_f, o_side, o_f, params, cap)
    else:
        parts = run_fused(hy, o_side, o_f, l_side, l_f, params, cap)
    check_scan(scan_l, lf)
    if of is not None:
        check_scan(left, of)
    check_join(expected, parts, 2, swapped, mode in ("Semi", "Anti"))


@pytest.mark.parametrize("mode", ["Inner", "Left", "Semi"])
@pytest.mark.parametrize("bloom", ["0", "1"])
@pytest.mark.parametrize("build_filter", [False, True])
def test_scan_join_counts_only(hy, oracle, monkeypatch, mode, bloom, build_filter):
    """out_offsets NULL with out_chunk_begin set: the join output and the scans' per-chunk match counts only (no scan
    PosLists). part1_compact then writes records for the rows taking part alone (after the prefilter), while the
    scan's counts still include the matches the prefilter drops."""
    monkeypatch.setenv("HY_JOIN_BLOOM", bloom)
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(repr(("counts_only", mode, bloom, build_filter)).encode()))
    okey, ostatus, lkey, lkey_nulls, qty, qty_nulls = orders_lineitem(rng, 40_000, True)
    lchunk, ochunk = 9_000, 7_000
    lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, True), ("l_quantity", hy.DataType.Float, True)],
                                    [lkey, qty], [lkey_nulls, qty_nulls], lchunk)
    orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False), ("o_status", hy.DataType.Int, False)],
                                  [okey, ostatus], [], ochunk)
    scan_l = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24.0, [])
    left = oracle.table_scan(orders, 1, hy.PredicateCondition.GreaterThanEquals, 3, []) if build_filter else orders
    expected, bits = oracle.join_hash(left, scan_l, getattr(hy.JoinMode, mode), (0, 0))
    lk = dt.DeviceColumn(capi, lkey, lkey_nulls, lchunk, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, lchunk, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, ochunk, "Unencoded")
    os_ = dt.DeviceColumn(capi, ostatus, None, ochunk, "Dictionary")
    lf = Filter(capi, lq, "LessThan", 24.0, offsets=False)
    of = Filter(capi, os_, "GreaterThanEquals", 3, offsets=False) if build_filter else None
    swapped = mode in ("Left", "Semi") or left.row_count() > scan_l.row_count()
    o_side, l_side = dt.join_side(capi, ok), dt.join_side(capi, lk)
    params = capi.JoinParams({"Inner": 0, "Left": 1, "Semi": 5}[mode], capi.HY_TYPE_INT32, bits, 17)
    cap = okey.size * 3 + lkey.size + 16
    o_f = of.f if of else None
    if swapped:
        parts = run_fused(hy, l_side, lf.f, o_side, o_f, params, cap)
    else:
        parts = run_fused(hy, o_side, o_f, l_side, lf.f, params, cap)
    check_join(expected, parts, 2, swapped, mode == "Semi")
    for table, filt, chunk in [(scan_l, lf, lchunk)] + ([(left, of, ochunk)] if of else []):
        counts = np.diff(filt.begin.fetch().astype(np.int64))
        want = np.zeros(counts.size, np.int64)
        for k in range(table.chunk_count()):
            pl = table.get_chunk(k).get_column(0).pos_list()
            want[pl[0, 0]] = pl.shape[0]
        assert np.array_equal(counts, want)


def test_scan_join_empty_and_all_none(hy, oracle):
    """Predicates matching nothing (dictionary early-out) and a side without rows."""
    capi = hy.capi
    rng = np.random.default_rng(5)
    okey, ostatus, lkey, _, qty, qty_nulls = orders_lineitem(rng, 5_000, False)
    lk = dt.DeviceColumn(capi, lkey, None, 4_000, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, 4_000, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, 3_000, "Unencoded")
    lf = Filter(capi, lq, "LessThan", -1.0)
    params = capi.JoinParams(0, capi.HY_TYPE_INT32, capi.lib.hy_join_radix_bits(okey.size, 4), 17)
    parts = run_fused(hy, dt.join_side(capi, ok), None, dt.join_side(capi, lk), lf.f, params, okey.size + 16)
    assert sum(p.shape[0] for _, p in parts) == 0
    assert all(o.size == 0 for o in lf.scan_output())


@pytest.mark.parametrize("bits", [12, 16, 20])
@pytest.mark.parametrize("mode", ["Inner", "Left", "Semi"])
@pytest.mark.parametrize("key_enc,filtered", [("Unencoded", True), ("Dictionary", True), ("Unencoded", False)])
@pytest.mark.parametrize("onepass,cap", [(False, None), (True, None), (True, "64"), ("blocked", None)])
def test_multi_digit_plans(hy, oracle, monkeypatch, bits, mode, key_enc, filtered, onepass, cap):
    """Radix plans of two and three digits through the default two-read first pass, the opt-in single-pass first
    radix pass (HY_ONEPASS=1, part1_onepass: gapped per-class bucket regions, look-back per digit) and, with
    HY_ONEPASS_CAP=64, its overflow fallback, and the opt-in pass 0 in Infinity-Cache row blocks (HY_BLOCKED=1,
    part1_count / part1_fill; 7,000-row blocks, so every side has several): scan output and every partition's
    PosLists equal the oracle's at the same radix bits (the reference constructor's radix_bits, join_hash.hpp:28)."""
    if onepass == "blocked":
        monkeypatch.setenv("HY_BLOCKED", "1")
        monkeypatch.setenv("HY_BLOCK_ROWS", "7000")
    elif onepass:
        monkeypatch.setenv("HY_ONEPASS", "1")
    if cap is not None:
        monkeypatch.setenv("HY_ONEPASS_CAP", cap)
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(repr((bits, mode, key_enc, filtered)).encode()))
    okey, ostatus, lkey, lkey_nulls, qty, qty_nulls = orders_lineitem(rng, 30_000, True)
    lchunk, ochunk = 6_000, 5_000
    lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, True), ("l_quantity", hy.DataType.Float, True)],
                                    [lkey, qty], [lkey_nulls, qty_nulls], lchunk)
    orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False), ("o_status", hy.DataType.Int, False)],
                                  [okey, ostatus], [], ochunk)
    probe_t = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24.0, []) if filtered else lineitem
    jm = getattr(hy.JoinMode, mode)
    # orders (the smaller input) builds for Inner; Left / Semi swap so that lineitem's rows are the build side
    expected, used = oracle.join_hash(orders, probe_t, jm, (0, 0), radix_bits=bits)
    assert used == bits
    lk = dt.DeviceColumn(capi, lkey, lkey_nulls, lchunk, key_enc)
    lq = dt.DeviceColumn(capi, qty, qty_nulls, lchunk, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, ochunk, "Unencoded")
    lf = Filter(capi, lq, "LessThan", 24.0) if filtered else None
    swapped = mode in ("Left", "Semi") or orders.row_count() > probe_t.row_count()
    params = capi.JoinParams({"Inner": 0, "Left": 1, "Semi": 5}[mode], capi.HY_TYPE_INT32, bits, 17)
    cap_pairs = okey.size * 3 + lkey.size + 16
    o_side, l_side = dt.join_side(capi, ok), dt.join_side(capi, lk)
    l_f = lf.f if lf else None
    if swapped:
        parts = run_fused(hy, l_side, l_f, o_side, None, params, cap_pairs)
    else:
        parts = run_fused(hy, o_side, None, l_side, l_f, params, cap_pairs)
    if lf is not None:
        check_scan(probe_t, lf)
    check_join(expected, parts, 2, swapped, mode == "Semi")


@pytest.mark.parametrize("variant", ["classic", "onepass", "blocked", "direct", "bloom", "build_filter"])
@pytest.mark.parametrize("mode", ["Inner", "Left"])
def test_scan_row_ids_from_every_pass0(hy, oracle, monkeypatch, variant, mode):
    """hy_join_filter.out_row_ids: the fused scan's PosLists written as RowIDs - by part1_spread itself on the classic
    pass 0, expanded from the offsets after the join on the other pass-0 variants (single-pass, row blocks, direct
    partitioning) - equal the oracle TableScan's output RowID for RowID, and the join output is unchanged."""
    env = {"onepass": {"HY_ONEPASS": "1"}, "blocked": {"HY_BLOCKED": "1", "HY_BLOCK_ROWS": "7000"},
           "direct": {"HY_JOIN_DIRECT": "1"}, "bloom": {"HY_JOIN_BLOOM": "1"}}.get(variant, {})
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(repr(("row_ids", variant, mode)).encode()))
    okey, ostatus, lkey, lkey_nulls, qty, qty_nulls = orders_lineitem(rng, 30_000, True)
    lchunk, ochunk = 6_000, 5_000
    lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, True), ("l_quantity", hy.DataType.Float, True)],
                                    [lkey, qty], [lkey_nulls, qty_nulls], lchunk)
    orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False), ("o_status", hy.DataType.Int, False)],
                                  [okey, ostatus], [], ochunk)
    build_filter = variant == "build_filter"
    scan_l = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24.0, [])
    left = oracle.table_scan(orders, 1, hy.PredicateCondition.GreaterThanEquals, 3, []) if build_filter else orders
    expected, bits = oracle.join_hash(left, scan_l, getattr(hy.JoinMode, mode), (0, 0), radix_bits=16)
    lk = dt.DeviceColumn(capi, lkey, lkey_nulls, lchunk, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, lchunk, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, ochunk, "Unencoded")
    os_ = dt.DeviceColumn(capi, ostatus, None, ochunk, "Dictionary")
    lf = Filter(capi, lq, "LessThan", 24.0, rows=True)
    of = Filter(capi, os_, "GreaterThanEquals", 3, rows=True) if build_filter else None
    swapped = mode == "Left" or left.row_count() > scan_l.row_count()
    params = capi.JoinParams({"Inner": 0, "Left": 1}[mode], capi.HY_TYPE_INT32, bits, 17)
    cap = okey.size * 3 + lkey.size + 16
    o_side, l_side = dt.join_side(capi, ok), dt.join_side(capi, lk)
    o_f = of.f if of else None
    if swapped:
        parts = run_fused(hy, l_side, lf.f, o_side, o_f, params, cap)
    else:
        parts = run_fused(hy, o_side, o_f, l_side, lf.f, params, cap)
    check_scan(scan_l, lf)
    if of is not None:
        check_scan(left, of)
    check_join(expected, parts, 2, swapped, False)


def test_scan_row_ids_need_offsets(hy):
    """out_row_ids without out_offsets is refused (HY_ERR_INVALID_ARGUMENT): other pass-0 variants stage offsets."""
    capi = hy.capi
    rng = np.random.default_rng(3)
    okey, _, lkey, _, qty, qty_nulls = orders_lineitem(rng, 2_000, False)
    lk = dt.DeviceColumn(capi, lkey, None, 1_000, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, 1_000, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, 1_000, "Unencoded")
    lf = Filter(capi, lq, "LessThan", 24.0, offsets=False, rows=True)
    params = capi.JoinParams(0, capi.HY_TYPE_INT32, capi.lib.hy_join_radix_bits(okey.size, 4), 17)
    wsb = ctypes.c_size_t()
    st = capi.lib.hy_scan_join_hash_workspace_size(ctypes.byref(dt.join_side(capi, ok)), None,
                                                   ctypes.byref(dt.join_side(capi, lk)), ctypes.byref(lf.f),
                                                   ctypes.byref(params), ctypes.byref(wsb))
    assert st == 1  # HY_ERR_INVALID_ARGUMENT



@pytest.mark.parametrize("mode", ["Inner", "Semi", "Left", "Anti"])
@pytest.mark.parametrize("bloom", ["0", "1", None])
@pytest.mark.parametrize("span", ["narrow", "wide"])
def test_selective_join_bloom_prefilter(hy, oracle, monkeypatch, mode, bloom, span):
    """A small build side against a large probe side where ~90% of the probe keys have no partner (TPC-H 3's shape):
    the default heuristic (probe >= 16x build) enables the probe-side prefilter for INNER / SEMI, which drops probe
    rows before partitioning; the output PosLists equal the oracle's, with the prefilter forced on, off and by the
    heuristic. `narrow` build keys (negative ones included) span a range the key-range bitmap covers (64 bits per build
    row reserved); `wide` ones span the int32 range, so the prefilter falls back to the Bloom filter."""
    if bloom is not None:
        monkeypatch.setenv("HY_JOIN_BLOOM", bloom)
    else:
        monkeypatch.delenv("HY_JOIN_BLOOM", raising=False)
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(f"bloom/{mode}/{bloom}/{span}".encode()))
    if span == "narrow":
        okey = rng.choice(np.arange(-100_000, 100_000, dtype=np.int32), 4_000, replace=False)
        lkey = rng.integers(-100_000, -60_000, 150_000).astype(np.int32)  # ~2% of them find a partner
        lkey[:50] = [-100_001, 100_000, np.iinfo(np.int32).min, np.iinfo(np.int32).max, 0] * 10  # the range's edges and beyond
    else:
        okey = np.unique(rng.integers(np.iinfo(np.int32).min, np.iinfo(np.int32).max, 4_000, dtype=np.int64))
        okey = rng.permutation(okey).astype(np.int32)
        lkey = rng.integers(np.iinfo(np.int32).min, np.iinfo(np.int32).max, 150_000, dtype=np.int64).astype(np.int32)
        hit = rng.random(150_000) < 0.1
        lkey[hit] = rng.choice(okey, int(hit.sum()))
    okey = np.concatenate([okey, okey[:300]])  # duplicate build keys
    lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, False)], [lkey], [], 20_000)
    orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False)], [okey], [], 3_000)
    jm = getattr(hy.JoinMode, mode)
    expected, bits = oracle.join_hash(orders, lineitem, jm, (0, 0))
    lk = dt.DeviceColumn(capi, lkey, None, 20_000, "Unencoded")
    ok = dt.DeviceColumn(capi, okey, None, 3_000, "Unencoded")
    swapped = mode in ("Left", "Semi", "Anti")
    params = capi.JoinParams({"Inner": 0, "Left": 1, "Semi": 5, "Anti": 6}[mode], capi.HY_TYPE_INT32, bits, 17)
    cap = okey.size * 4 + lkey.size + 16
    if swapped:
        parts = run_fused(hy, dt.join_side(capi, lk), None, dt.join_side(capi, ok), None, params, cap)
    else:
        parts = run_fused(hy, dt.join_side(capi, ok), None, dt.join_side(capi, lk), None, params, cap)
    check_join(expected, parts, 1, swapped, mode in ("Semi", "Anti"))


@pytest.mark.parametrize("mode", ["Inner", "Semi"])
@pytest.mark.parametrize("span", ["narrow", "wide"])
@pytest.mark.parametrize("buckets", ["1", "0"])
def test_prefilter_built_per_region(hy, oracle, monkeypatch, mode, span, buckets):
    """The prefilter's words set per LDS region (filter_bucket_count / scan / scatter / set; HY_FILTER_BUCKETS=0: one
    global atomic per key) with a build side large enough for several regions and several count workgroups: the
    key-range bitmap (`narrow`: 60,000 keys over a 3 M range, 12 regions of 8,192 words) and the Bloom filter (`wide`:
    keys over the int32 range). The output PosLists equal the oracle's."""
    monkeypatch.setenv("HY_JOIN_BLOOM", "1")
    monkeypatch.setenv("HY_FILTER_BUCKETS", buckets)
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(f"regions/{mode}/{span}".encode()))
    if span == "narrow":
        okey = rng.choice(np.arange(-1_000_000, 2_000_000, dtype=np.int32), 60_000, replace=False)
        lkey = rng.integers(-1_100_000, 2_100_000, 400_000).astype(np.int32)
    else:
        okey = np.unique(rng.integers(np.iinfo(np.int32).min, np.iinfo(np.int32).max, 60_000, dtype=np.int64))
        okey = rng.permutation(okey).astype(np.int32)
        lkey = rng.integers(np.iinfo(np.int32).min, np.iinfo(np.int32).max, 400_000, dtype=np.int64).astype(np.int32)
        hit = rng.random(400_000) < 0.05
        lkey[hit] = rng.choice(okey, int(hit.sum()))
    lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, False)], [lkey], [], 50_000)
    orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False)], [okey], [], 20_000)
    jm = getattr(hy.JoinMode, mode)
    expected, bits = oracle.join_hash(orders, lineitem, jm, (0, 0))
    lk = dt.DeviceColumn(capi, lkey, None, 50_000, "Unencoded")
    ok = dt.DeviceColumn(capi, okey, None, 20_000, "Unencoded")
    swapped = mode == "Semi"
    params = capi.JoinParams({"Inner": 0, "Semi": 5}[mode], capi.HY_TYPE_INT32, bits, 17)
    cap = okey.size * 4 + lkey.size + 16
    if swapped:
        parts = run_fused(hy, dt.join_side(capi, lk), None, dt.join_side(capi, ok), None, params, cap)
    else:
        parts = run_fused(hy, dt.join_side(capi, ok), None, dt.join_side(capi, lk), None, params, cap)
    check_join(expected, parts, 1, swapped, mode == "Semi")


@pytest.mark.parametrize("mode", ["Inner", "Left"])
def test_prepared_plan_equals_call(hy, mode):
    """hy_scan_join_plan_execute (descriptors staged on the first execution only) equals hy_scan_join_hash, on its
    first and on later executions, with the scan outputs cleared and the output buffers changed in between."""
    capi, L = hy.capi, hy.capi.lib
    rng = np.random.default_rng(0x504C4E)
    okey, ostatus, lkey, lkey_nulls, qty, qty_nulls = orders_lineitem(rng, 30_000, True)
    lk = dt.DeviceColumn(capi, lkey, lkey_nulls, 8_000, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, 8_000, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, 6_000, "Unencoded")
    lf = Filter(capi, lq, "LessThan", 24.0)
    params = capi.JoinParams({"Inner": 0, "Left": 1}[mode], capi.HY_TYPE_INT32, L.hy_join_radix_bits(okey.size, 4), 17)
    o_side, l_side = dt.join_side(capi, ok), dt.join_side(capi, lk)
    cap = okey.size * 3 + lkey.size + 16
    want = run_fused(hy, o_side, None, l_side, lf.f, params, cap)
    want_scan = lf.scan_output()
    plan = ctypes.c_void_p()
    capi.check(L.hy_scan_join_plan_create(ctypes.byref(o_side), None, ctypes.byref(l_side), ctypes.byref(lf.f),
                                          ctypes.byref(params), ctypes.byref(plan)), "hy_scan_join_plan_create")
    n_parts = 1 << params.radix_bits
    try:
        for run in range(3):
            zeros = np.zeros_like(lf.out.host)  # clear the scan output in place (the plan holds its pointer)
            capi.check(L.hy_memcpy_htod(lf.out.ptr, zeros.ctypes.data, zeros.nbytes, None), "clear")
            ob = capi.DeviceArray(np.full(cap * 2, run + 7, np.uint32))
            op = capi.DeviceArray(np.full(cap * 2, run + 9, np.uint32))
            pbeg, pcnt = capi.DeviceArray(np.zeros(n_parts, np.uint64)), capi.DeviceArray(np.zeros(n_parts, np.uint32))
            res = capi.JoinResult()
            capi.check(L.hy_scan_join_plan_execute(plan, ob.ptr, op.ptr, cap, pbeg.ptr, pcnt.ptr, ctypes.byref(res),
                                                   None), "hy_scan_join_plan_execute")
            b, p = ob.fetch().reshape(-1, 2), op.fetch().reshape(-1, 2)
            got = [(b[x:x + c], p[x:x + c]) for x, c in zip(pbeg.fetch().astype(np.int64), pcnt.fetch().astype(np.int64))]
            assert len(got) == len(want)
            for (gb, gp), (wb, wp) in zip(got, want):
                assert np.array_equal(gb, wb) and np.array_equal(gp, wp), f"execution {run}"
            assert all(np.array_equal(a, c) for a, c in zip(lf.scan_output(), want_scan)), f"execution {run}: scan"
    finally:
        L.hy_scan_join_plan_destroy(plan)


def test_prepared_plan_graph_replay(hy):
    """On a stream of its own the plan's third and later executions replay a captured hipGraph: same output as the
    call; changed output buffers are recaptured; HY_PLAN_GRAPH=0 paths are covered by the test above."""
    capi, L = hy.capi, hy.capi.lib
    rng = np.random.default_rng(0x475250)
    okey, ostatus, lkey, lkey_nulls, qty, qty_nulls = orders_lineitem(rng, 20_000, False)
    lk = dt.DeviceColumn(capi, lkey, None, 5_000, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, 5_000, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, 4_000, "Unencoded")
    lf = Filter(capi, lq, "LessThan", 30.0)
    params = capi.JoinParams(0, capi.HY_TYPE_INT32, L.hy_join_radix_bits(okey.size, 4), 17)
    o_side, l_side = dt.join_side(capi, ok), dt.join_side(capi, lk)
    cap = okey.size * 3 + lkey.size + 16
    want = run_fused(hy, o_side, None, l_side, lf.f, params, cap)
    stream = ctypes.c_void_p()
    capi.check(L.hy_stream_create(ctypes.byref(stream)), "hy_stream_create")
    plan = ctypes.c_void_p()
    capi.check(L.hy_scan_join_plan_create(ctypes.byref(o_side), None, ctypes.byref(l_side), ctypes.byref(lf.f),
                                          ctypes.byref(params), ctypes.byref(plan)), "plan")
    n_parts = 1 << params.radix_bits
    bufs = [tuple(capi.DeviceArray(np.zeros(n, t)) for n, t in ((cap * 2, np.uint32), (cap * 2, np.uint32),
                                                                 (n_parts, np.uint64), (n_parts, np.uint32)))
            for _ in range(2)]
    try:
        for run in range(6):
            ob, op, pbeg, pcnt = bufs[0 if run < 4 else 1]
            res = capi.JoinResult()
            capi.check(L.hy_scan_join_plan_execute(plan, ob.ptr, op.ptr, cap, pbeg.ptr, pcnt.ptr, ctypes.byref(res),
                                                   stream), "execute")
            capi.check(L.hy_stream_synchronize(stream), "sync")
            b, p = ob.fetch().reshape(-1, 2), op.fetch().reshape(-1, 2)
            got = [(b[x:x + c], p[x:x + c]) for x, c in zip(pbeg.fetch().astype(np.int64), pcnt.fetch().astype(np.int64))]
            assert res.total_pairs == sum(len(x) for _, x in want)
            for (gb, gp), (wb, wp) in zip(got, want):
                assert np.array_equal(gb, wb) and np.array_equal(gp, wp), f"execution {run}"
    finally:
        L.hy_scan_join_plan_destroy(plan)
        L.hy_stream_destroy(stream)


def test_prepared_plan_replay_after_ring_wrap(hy, monkeypatch):
    """A captured plan replays from its own workspace, never from the per-thread pinned staging ring (ADVICE r04,
    VERDICT r04 item 2): after the graph is captured, a string TableScan on the same thread stages a 17 MiB constant -
    the ring wraps and is reallocated - and the replays still equal the call. The plan also keeps the knobs it was
    created with: HY_HASH_RECORDS flipped after creation changes neither its layout nor its output."""
    capi, L = hy.capi, hy.capi.lib
    rng = np.random.default_rng(0x57524150)
    okey, ostatus, lkey, lkey_nulls, qty, qty_nulls = orders_lineitem(rng, 20_000, False)
    lk = dt.DeviceColumn(capi, lkey, None, 5_000, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, 5_000, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, 4_000, "Unencoded")
    lf = Filter(capi, lq, "LessThan", 30.0)
    params = capi.JoinParams(0, capi.HY_TYPE_INT32, 16, 17)  # >= 16 bits: 6-byte hash records in the last pass
    o_side, l_side = dt.join_side(capi, ok), dt.join_side(capi, lk)
    cap = okey.size * 3 + lkey.size + 16
    want = run_fused(hy, o_side, None, l_side, lf.f, params, cap)
    stream = ctypes.c_void_p()
    capi.check(L.hy_stream_create(ctypes.byref(stream)), "hy_stream_create")
    plan = ctypes.c_void_p()
    capi.check(L.hy_scan_join_plan_create(ctypes.byref(o_side), None, ctypes.byref(l_side), ctypes.byref(lf.f),
                                          ctypes.byref(params), ctypes.byref(plan)), "plan")
    n_parts = 1 << params.radix_bits
    ob, op = capi.DeviceArray(np.zeros(cap * 2, np.uint32)), capi.DeviceArray(np.zeros(cap * 2, np.uint32))
    pbeg, pcnt = capi.DeviceArray(np.zeros(n_parts, np.uint64)), capi.DeviceArray(np.zeros(n_parts, np.uint32))
    strings = hy.Table([("s", hy.DataType.String, False)], hy.TableType.Data, 64)
    for i in range(100):
        strings.append([f"s{i}"])
    try:
        for run in range(8):
            if run == 4:  # graph captured at execution 2 and replayed since: wrap the ring on this thread
                scan = hy.TableScan(wrap(hy, strings), 0, hy.PredicateCondition.Equals, "x" * (17 << 20))
                scan.execute()
                assert scan.get_output().row_count() == 0
            if run == 6:
                monkeypatch.setenv("HY_HASH_RECORDS", "0")
            capi.check(L.hy_memcpy_htod(ob.ptr, np.zeros(cap * 2, np.uint32).ctypes.data, cap * 8, None), "clear")
            res = capi.JoinResult()
            capi.check(L.hy_scan_join_plan_execute(plan, ob.ptr, op.ptr, cap, pbeg.ptr, pcnt.ptr, ctypes.byref(res),
                                                   stream), "execute")
            capi.check(L.hy_stream_synchronize(stream), "sync")
            b, p = ob.fetch().reshape(-1, 2), op.fetch().reshape(-1, 2)
            got = [(b[x:x + c], p[x:x + c]) for x, c in zip(pbeg.fetch().astype(np.int64), pcnt.fetch().astype(np.int64))]
            assert res.total_pairs == sum(len(x) for _, x in want)
            for (gb, gp), (wb, wp) in zip(got, want):
                assert np.array_equal(gb, wb) and np.array_equal(gp, wp), f"execution {run}"
    finally:
        L.hy_scan_join_plan_destroy(plan)
        L.hy_stream_destroy(stream)


@pytest.mark.parametrize("bits", [16, 18])
@pytest.mark.parametrize("mode", ["Inner", "Left", "Semi", "Anti"])
@pytest.mark.parametrize("variant", ["hash_records", "skewed", "bloom", "key_records"])
def test_hash_records(hy, oracle, monkeypatch, bits, mode, variant):
    """int32 keys with b >= 16 radix bits: the last partition pass keeps the 16 murmur2 bits above the partition
    instead of the key (6-byte SoA records; murmur2 is a bijection on 4-byte keys, so equal remainders inside a
    partition are equal keys). Duplicate build keys, NULL probe keys, unmatched rows; `skewed` caps the LDS tables at
    a few dozen rows so every partition goes through join_partition_skewed, `bloom` forces the probe-side prefilter
    (then keyed by hash and set by the build side's last pass), `key_records` is HY_HASH_RECORDS=0. Output equals the
    oracle's at the same radix bits, partition by partition."""
    if variant == "skewed":
        monkeypatch.setenv("HY_JOIN_LDS_BUDGET", "1024")
    if variant == "bloom":
        monkeypatch.setenv("HY_JOIN_BLOOM", "1")
    if variant == "key_records":
        monkeypatch.setenv("HY_HASH_RECORDS", "0")
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(repr(("hash_records", bits, mode, variant)).encode()))
    okey, ostatus, lkey, lkey_nulls, qty, qty_nulls = orders_lineitem(rng, 25_000, True)
    lchunk, ochunk = 7_000, 4_000
    lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, True), ("l_quantity", hy.DataType.Float, True)],
                                    [lkey, qty], [lkey_nulls, qty_nulls], lchunk)
    orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False), ("o_status", hy.DataType.Int, False)],
                                  [okey, ostatus], [], ochunk)
    probe_t = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 30.0, [])
    jm = getattr(hy.JoinMode, mode)
    expected, used = oracle.join_hash(orders, probe_t, jm, (0, 0), radix_bits=bits)
    assert used == bits
    lk = dt.DeviceColumn(capi, lkey, lkey_nulls, lchunk, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, lchunk, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, ochunk, "Unencoded")
    lf = Filter(capi, lq, "LessThan", 30.0)
    swapped = mode in ("Left", "Semi", "Anti") or orders.row_count() > probe_t.row_count()
    params = capi.JoinParams({"Inner": 0, "Left": 1, "Semi": 5, "Anti": 6}[mode], capi.HY_TYPE_INT32, bits, 17)
    cap_pairs = okey.size * 3 + lkey.size + 16
    o_side, l_side = dt.join_side(capi, ok), dt.join_side(capi, lk)
    if swapped:
        parts = run_fused(hy, l_side, lf.f, o_side, None, params, cap_pairs)
    else:
        parts = run_fused(hy, o_side, None, l_side, lf.f, params, cap_pairs)
    check_scan(probe_t, lf)
    check_join(expected, parts, 2, swapped, mode in ("Semi", "Anti"))


@pytest.mark.parametrize("stash", ["1", "0"])
@pytest.mark.parametrize("avg", [6_100, 6_600])
@pytest.mark.parametrize("mode", ["Inner", "Left", "Right", "Semi", "Anti"])
def test_two_pass_partitions(hy, oracle, monkeypatch, stash, avg, mode):
    """Partitions whose probe records need about two passes of join_partition_multi (the all-multi launch: every
    partition there, as TPC-H SF10's 8,192 partitions of ~7,300 probe rows): with HY_JOIN_STASH=1 a two-pass partition
    keeps its first pass's payloads and match infos in LDS (no reload, no second match), one-pass partitions are
    written from registers, and a partition of a hot key takes the count + reload passes; HY_JOIN_STASH=0 reloads every
    multi-pass partition. Duplicate build keys, unmatched probe keys; every partition's PosLists equal the oracle's."""
    monkeypatch.setenv("HY_JOIN_STASH", stash)
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(repr(("two_pass", avg, mode)).encode()))
    bits, nb = 5, 60_000
    bkeys = rng.permutation(nb).astype(np.int32)
    bkeys = np.concatenate([bkeys, bkeys[rng.integers(0, nb, nb // 20)]])
    n_probe = avg << bits
    pkeys = rng.integers(-2_000, nb, n_probe)
    pkeys[rng.random(n_probe) < 0.02] = 7  # one hot key: its partition needs three passes or more
    pkeys = pkeys.astype(np.int32)
    B = hy.Table.from_arrays([("k", hy.DataType.Int, False)], [bkeys], [], 20_000)
    P = hy.Table.from_arrays([("k", hy.DataType.Int, False)], [pkeys], [], 50_000)
    jm = getattr(hy.JoinMode, mode)
    swapped = mode in ("Left", "Semi", "Anti")  # the reference's swap: the right input builds
    expected, used = (oracle.join_hash(P, B, jm, (0, 0), radix_bits=bits) if swapped
                      else oracle.join_hash(B, P, jm, (0, 0), radix_bits=bits))
    assert used == bits
    bcol = dt.DeviceColumn(capi, bkeys, None, 20_000, "Unencoded")
    pcol = dt.DeviceColumn(capi, pkeys, None, 50_000, "Unencoded")
    params = capi.JoinParams({"Inner": 0, "Left": 1, "Right": 2, "Semi": 5, "Anti": 6}[mode], capi.HY_TYPE_INT32,
                             bits, 17)
    parts = run_fused(hy, dt.join_side(capi, bcol), None, dt.join_side(capi, pcol), None, params,
                      bkeys.size * 4 + n_probe + 16)
    check_join(expected, parts, 1, swapped, mode in ("Semi", "Anti"))
