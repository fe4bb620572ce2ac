"""Direct partitioning of a JoinHash side with a fused TableScan (kernels/join_direct.hip: span match counts,
part1_direct into (span, bucket) regions, part2g_hist / part2g_scatter over (bucket, span group) run lists) against
the oracle's TableScan followed by its JoinHash (reference table_scan.cpp:78-164, join_hash.cpp:203-355 partition
order, write_output_columns :564-613): the scan's per-chunk offsets and every partition's PosLists RowID for RowID,
over radix plans of two digits (9 to 16 bits), span sizes and span-group counts that cut runs mid-tile, the region
overflow fallback (keys concentrated in one bucket) and prepared plans replaying a captured graph."""
import ctypes
import zlib

import numpy as np
import pytest

import device_tables as dt
from test_scan_join_gpu import Filter, check_join, check_scan, orders_lineitem, run_fused

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def direct_on(monkeypatch):
    monkeypatch.setenv("HY_JOIN_DIRECT", "1")  # (opt-in: the classic passes are the default)


def lineitem_orders(hy, rng, n_orders, lchunk, ochunk, skew=0.0):
    okey, ostatus, lkey, lkey_nulls, qty, qty_nulls = orders_lineitem(rng, n_orders, True)
    if skew:  # a share of the probe rows on one build key: its bucket's regions overflow
        hot = rng.random(lkey.size) < skew
        lkey[hot] = okey[0]
    lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, True), ("l_quantity", hy.DataType.Float, True)],
                                    [lkey, qty], [lkey_nulls, qty_nulls], lchunk)
    orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False), ("o_status", hy.DataType.Int, False)],
                                  [okey, ostatus], [], ochunk)
    return okey, lkey, lkey_nulls, qty, qty_nulls, lineitem, orders


@pytest.mark.parametrize("bits", [9, 12, 16])
@pytest.mark.parametrize("span,groups", [("1", "0"), ("3", "7"), ("16", "1"), ("5", "0")])
@pytest.mark.parametrize("key_enc", ["Unencoded", "Dictionary"])
def test_direct_passes_match_oracle(hy, oracle, monkeypatch, bits, span, groups, key_enc):
    monkeypatch.setenv("HY_DIRECT_SPAN", span)
    monkeypatch.setenv("HY_DIRECT_GROUPS", groups)
    monkeypatch.setenv("HY_JOIN_BLOOM", "0")
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(repr(("direct", bits, span, groups, key_enc)).encode()))
    lchunk, ochunk = 13_000, 5_000  # spans end mid-chunk; the last span of a chunk is short
    okey, lkey, lkey_nulls, qty, qty_nulls, lineitem, orders = lineitem_orders(hy, rng, 30_000, lchunk, ochunk)
    probe_t = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24.0, [])
    expected, used = oracle.join_hash(orders, probe_t, hy.JoinMode.Inner, (0, 0), radix_bits=bits)
    assert used == bits
    lk = dt.DeviceColumn(capi, lkey, lkey_nulls, lchunk, key_enc)
    lq = dt.DeviceColumn(capi, qty, qty_nulls, lchunk, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, ochunk, "Unencoded")
    lf = Filter(capi, lq, "LessThan", 24.0)
    assert orders.row_count() < probe_t.row_count()  # orders builds: the filtered lineitem side is the probe side
    params = capi.JoinParams(0, capi.HY_TYPE_INT32, bits, 17)
    parts = run_fused(hy, dt.join_side(capi, ok), None, dt.join_side(capi, lk), lf.f, params,
                      okey.size * 3 + lkey.size + 16)
    check_scan(probe_t, lf)
    check_join(expected, parts, 2, False, False)


@pytest.mark.parametrize("offsets", [True, False])
def test_direct_counts_only_and_semi(hy, oracle, monkeypatch, offsets):
    """The join-output-only form (out_offsets NULL: per-chunk counts still written) and a SEMI join whose probe side
    takes the direct passes."""
    monkeypatch.setenv("HY_JOIN_BLOOM", "0")
    monkeypatch.setenv("HY_DIRECT_SPAN", "2")
    capi = hy.capi
    rng = np.random.default_rng(77 + offsets)
    okey, lkey, lkey_nulls, qty, qty_nulls, lineitem, orders = lineitem_orders(hy, rng, 20_000, 9_000, 4_000)
    probe_t = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 30.0, [])
    lk = dt.DeviceColumn(capi, lkey, lkey_nulls, 9_000, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, 9_000, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, 4_000, "Unencoded")
    for mode, code in (("Inner", 0), ("Semi", 5)):
        # SEMI: the reference swaps (join_hash.cpp:55-76) so that the filtered lineitem rows probe... only when the
        # orders side is the left input; here lineitem is the right input and stays the probe side for Inner
        if mode == "Semi":
            expected, bits = oracle.join_hash(probe_t, orders, hy.JoinMode.Semi, (0, 0), radix_bits=14)
        else:
            expected, bits = oracle.join_hash(orders, probe_t, hy.JoinMode.Inner, (0, 0), radix_bits=14)
        lf = Filter(capi, lq, "LessThan", 30.0, offsets=offsets)
        params = capi.JoinParams(code, capi.HY_TYPE_INT32, bits, 17)
        # Semi: build = the right input (orders), probe = the left input (the filtered lineitem side)
        parts = run_fused(hy, dt.join_side(capi, ok), None, dt.join_side(capi, lk), lf.f, params,
                          okey.size * 3 + lkey.size + 16)
        check_join(expected, parts, 2, mode == "Semi", mode == "Semi")
        counts = np.diff(lf.begin.fetch().astype(np.int64))
        want = np.zeros(counts.size, np.int64)
        for k in range(probe_t.chunk_count()):
            pl = probe_t.get_chunk(k).get_column(0).pos_list()
            want[pl[0, 0]] = pl.shape[0]
        assert np.array_equal(counts, want)
        if offsets:
            check_scan(probe_t, lf)


@pytest.mark.parametrize("skew", [0.6, 0.95])
def test_direct_region_overflow_falls_back(hy, oracle, monkeypatch, skew):
    """Most probe rows on one key: their bucket's (span, bucket) regions overflow (direct_cap is sized for murmur2's
    spread), the device raises the flag, and the join reruns on the classic passes - same output as the oracle."""
    monkeypatch.setenv("HY_JOIN_BLOOM", "0")
    capi = hy.capi
    rng = np.random.default_rng(int(skew * 1000))
    okey, lkey, lkey_nulls, qty, qty_nulls, lineitem, orders = lineitem_orders(hy, rng, 20_000, 60_000, 5_000, skew)
    probe_t = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 40.0, [])
    expected, bits = oracle.join_hash(orders, probe_t, hy.JoinMode.Inner, (0, 0), radix_bits=16)
    lk = dt.DeviceColumn(capi, lkey, lkey_nulls, 60_000, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, 60_000, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, 5_000, "Unencoded")
    lf = Filter(capi, lq, "LessThan", 40.0)
    params = capi.JoinParams(0, capi.HY_TYPE_INT32, bits, 17)
    parts = run_fused(hy, dt.join_side(capi, ok), None, dt.join_side(capi, lk), lf.f, params,
                      okey.size * 3 + lkey.size * 2 + 16)
    check_scan(probe_t, lf)
    check_join(expected, parts, 2, False, False)


@pytest.mark.parametrize("skew", [0.0, 0.9])
def test_direct_prepared_plan_replays(hy, oracle, monkeypatch, skew):
    """A prepared plan on a stream of its own: the eager execution, the capture and the replays of the direct passes
    equal the oracle; with skewed keys the first execution falls back to the classic passes and the plan keeps them
    (its captured graph is then the classic one)."""
    monkeypatch.setenv("HY_JOIN_BLOOM", "0")
    capi, L = hy.capi, hy.capi.lib
    rng = np.random.default_rng(0xD1 + int(skew * 10))
    okey, lkey, lkey_nulls, qty, qty_nulls, lineitem, orders = lineitem_orders(hy, rng, 20_000, 30_000, 4_000, skew)
    probe_t = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 30.0, [])
    expected, bits = oracle.join_hash(orders, probe_t, hy.JoinMode.Inner, (0, 0), radix_bits=16)
    lk = dt.DeviceColumn(capi, lkey, lkey_nulls, 30_000, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, 30_000, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, 4_000, "Unencoded")
    lf = Filter(capi, lq, "LessThan", 30.0)
    params = capi.JoinParams(0, capi.HY_TYPE_INT32, bits, 17)
    o_side, l_side = dt.join_side(capi, ok), dt.join_side(capi, lk)
    cap = okey.size * 3 + lkey.size * 2 + 16
    stream = ctypes.c_void_p()
    capi.check(L.hy_stream_create(ctypes.byref(stream)), "hy_stream_create")
    plan = ctypes.c_void_p()
    capi.check(L.hy_scan_join_plan_create(ctypes.byref(o_side), None, ctypes.byref(l_side), ctypes.byref(lf.f),
                                          ctypes.byref(params), ctypes.byref(plan)), "plan")
    n_parts = 1 << bits
    ob, op = capi.DeviceArray(np.zeros(cap * 2, np.uint32)), capi.DeviceArray(np.zeros(cap * 2, np.uint32))
    pbeg, pcnt = capi.DeviceArray(np.zeros(n_parts, np.uint64)), capi.DeviceArray(np.zeros(n_parts, np.uint32))
    try:
        for run in range(5):
            capi.check(L.hy_memcpy_htod(lf.out.ptr, np.zeros_like(lf.out.host).ctypes.data, lf.out.host.nbytes, None),
                       "clear")
            res = capi.JoinResult()
            capi.check(L.hy_scan_join_plan_execute(plan, ob.ptr, op.ptr, cap, pbeg.ptr, pcnt.ptr, ctypes.byref(res),
                                                   stream), "execute")
            capi.check(L.hy_stream_synchronize(stream), "sync")
            b, p = ob.fetch().reshape(-1, 2), op.fetch().reshape(-1, 2)
            parts = [(b[x:x + c], p[x:x + c]) for x, c in zip(pbeg.fetch().astype(np.int64), pcnt.fetch().astype(np.int64))]
            check_join(expected, parts, 2, False, False)
            check_scan(probe_t, lf)
    finally:
        L.hy_scan_join_plan_destroy(plan)
        L.hy_stream_destroy(stream)


@pytest.mark.parametrize("direct", ["0", "1"])
@pytest.mark.parametrize("mode", ["Inner", "Left", "Semi"])
def test_ballot_rank_fallback(hy, oracle, monkeypatch, direct, mode):
    """HY_RANK_BALLOT=1 forces the ranking a device falls back to when rank_order_check fails (per-bit ballots,
    hyk::rank_item) in every partition pass - classic and direct, both sides: the output still equals the oracle's."""
    monkeypatch.setenv("HY_RANK_BALLOT", "1")
    monkeypatch.setenv("HY_JOIN_DIRECT", direct)
    monkeypatch.setenv("HY_JOIN_BLOOM", "0")
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(repr(("ballot", direct, mode)).encode()))
    okey, lkey, lkey_nulls, qty, qty_nulls, lineitem, orders = lineitem_orders(hy, rng, 20_000, 7_000, 3_000)
    probe_t = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24.0, [])
    jm = getattr(hy.JoinMode, mode)
    expected, bits = oracle.join_hash(orders, probe_t, jm, (0, 0), radix_bits=16)
    lk = dt.DeviceColumn(capi, lkey, lkey_nulls, 7_000, "Unencoded")
    lq = dt.DeviceColumn(capi, qty, qty_nulls, 7_000, "Dictionary")
    ok = dt.DeviceColumn(capi, okey, None, 3_000, "Unencoded")
    lf = Filter(capi, lq, "LessThan", 24.0)
    swapped = mode in ("Left", "Semi")
    params = capi.JoinParams({"Inner": 0, "Left": 1, "Semi": 5}[mode], capi.HY_TYPE_INT32, bits, 17)
    o_side, l_side = dt.join_side(capi, ok), dt.join_side(capi, lk)
    cap = okey.size * 3 + lkey.size + 16
    if swapped:
        parts = run_fused(hy, l_side, lf.f, o_side, None, params, cap)
    else:
        parts = run_fused(hy, o_side, None, l_side, lf.f, params, cap)
    check_scan(probe_t, lf)
    check_join(expected, parts, 2, swapped, mode == "Semi")
