"""agg_dense_lanes (csrc/kernels/aggregate_lanes.hip): the dense Aggregate accumulating per lane, with the Projection's
+ - * expressions evaluated as chains - TPC-H 1's SUM / AVG / COUNT shape (reference projection.cpp:39-87 feeding
aggregate.cpp:133-249). Every case runs hy_aggregate twice - lanes path (default) and HY_AGG_LANES=0 (agg_dense_fused
over every step) - and checks both against numpy: float32 expressions as the reference's functors compute them,
counts exact, float SUM / AVG equal to the exactly rounded sum (math.fsum), int32 sums exact. The data cases drive the
kernel's exits: clean Q1-shaped columns (every step on the lanes path), NULLs, tiny / huge / non-finite / denormal
values, negative and zero values (steps deferred to agg_dense_fused or re-based), more groups than a wave's table,
int32 sums and COUNT(col); data and reference inputs (PosLists into one chunk, and mixing chunks)."""
import ctypes
import math
import zlib

import numpy as np
import pytest

import device_tables as dt

pytestmark = pytest.mark.gpu

N, CHUNK = 60_000, 9_000

# [rf, ls, qty, price, dp = price * (1 - disc), ch = dp * (1 + tax), disc, tax, iq (int32), iexpr = iq * 3 - 7 (int32)]
AGGS = [("SUM", 2), ("SUM", 3), ("SUM", 4), ("SUM", 5), ("AVG", 2), ("AVG", 3), ("AVG", 6), ("COUNT", -1),
        ("SUM", 8), ("AVG", 9), ("COUNT", 7)]
# TPC-H 1's aggregates alone (float sums of columns and chains, COUNT(*)): the shape agg_dense_stream takes
Q1_AGGS = AGGS[:8]


def columns(rng, case):
    rf_dom, ls_dom = (8, 4) if case == "many_groups" else (3, 2)
    rf = rng.integers(0, rf_dom, N).astype(np.int32)
    ls = rng.integers(0, ls_dom, N).astype(np.int32)
    if case == "clustered":  # one group per 5000 rows: the table refills as codes change
        rf = ((np.arange(N) // 5000) % 3).astype(np.int32)
        ls = ((np.arange(N) // 7000) % 2).astype(np.int32)
    qty = rng.integers(1, 51, N).astype(np.float32)
    price = (rng.integers(90_000, 210_001, N) * qty.astype(np.int64) / 100.0).astype(np.float32)
    disc = (rng.integers(0, 11, N) / 100.0).astype(np.float32)
    tax = (rng.integers(0, 9, N) / 100.0).astype(np.float32)
    iq = rng.integers(-1000, 1000, N).astype(np.int32)
    price_n = np.zeros(N, np.uint8)
    disc_n = np.zeros(N, np.uint8)
    if case == "nulls":
        price_n = (rng.random(N) < 0.002).astype(np.uint8)
        disc_n = (rng.random(N) < 0.001).astype(np.uint8)
    elif case == "null_ids":  # NULL value ids in a small-dictionary column only (agg_dense_stream defers their steps)
        disc_n = (rng.random(N) < 0.001).astype(np.uint8)
    elif case == "odd_values":  # steps leave the window / hold non-finite, denormal, negative, zero values
        price[rng.random(N) < 0.0005] = np.float32(-3.5e-30)
        price[rng.random(N) < 0.0005] = np.float32(7.0e25)
        price[rng.random(N) < 0.0002] = np.float32(1.0e-41)  # denormal
        price[rng.random(N) < 0.001] = np.float32(0.0)
        price[rng.random(N) < 0.001] *= np.float32(-1)
        qty[rng.random(N) < 0.0001] = np.float32(np.inf)
    elif case == "wide_range":  # every step spans more binades than one window: re-based or deferred steps
        price = (rng.standard_normal(N) * np.exp2(rng.integers(-40, 40, N))).astype(np.float32)
    elif case == "drift":  # magnitudes drift upwards chunk by chunk: re-bases as the largest exponent grows
        price = (price * np.exp2(np.arange(N) // 3000)).astype(np.float32)
    return rf, ls, qty, price, disc, tax, iq, price_n, disc_n, (rf_dom, ls_dom)


def expected(cols, rows):
    rf, ls, qty, price, disc, tax, iq, price_n, disc_n, _ = cols
    one = np.float32(1)
    with np.errstate(all="ignore"):
        dp = (price * (one - disc)).astype(np.float32)
        ch = (dp * (one + tax)).astype(np.float32)
    ie = (iq.astype(np.int64) * 3 - 7).astype(np.int32)
    dp_null = (price_n | disc_n).astype(bool)
    out = {}
    for r in rows:
        g = (int(rf[r]), int(ls[r]))
        e = out.setdefault(g, {"rows": 0, 2: [], 3: [], 4: [], 5: [], 6: [], 7: 0, 8: [], 9: []})
        e["rows"] += 1
        e[2].append(float(qty[r]))
        e[8].append(int(iq[r]))
        e[9].append(int(ie[r]))
        if not price_n[r]:
            e[3].append(float(price[r]))
        if not dp_null[r]:
            e[4].append(float(dp[r]))
            e[5].append(float(ch[r]))
        if not disc_n[r]:
            e[6].append(float(disc[r]))
        e[7] += 1  # tax has no NULLs
    return out


def fsum_inf(vals):
    if any(math.isnan(v) for v in vals) or (any(v == math.inf for v in vals) and any(v == -math.inf for v in vals)):
        return math.nan
    if any(math.isinf(v) for v in vals):
        return next(v for v in vals if math.isinf(v))
    return math.fsum(vals)


def run(hy, dcols, pos_lists, sizes, doms, part=None, raw=False, filt=None, aggs=AGGS):
    """hy_aggregate over the input (or over input chunks [lo, hi) with part=(lo, hi)); raw: (records, layout,
    params) instead of the decoded results."""
    capi, L = hy.capi, hy.capi.lib
    lo, hi = part if part is not None else (0, len(sizes))
    I32, F32 = capi.HY_TYPE_INT32, capi.HY_TYPE_FLOAT
    N_ = capi.ExprNode
    col = lambda j, t=F32: N_(capi.HY_EXPR_COLUMN, t, 0, j, 0)
    one = N_(capi.HY_EXPR_VALUE, I32, 0, 0, 1)
    dp = [col(3), one, col(6), N_(capi.HY_EXPR_SUB, F32, F32, 0, 0), N_(capi.HY_EXPR_MUL, F32, F32, 0, 0)]
    ch = dp + [one, col(7), N_(capi.HY_EXPR_ADD, F32, F32, 0, 0), N_(capi.HY_EXPR_MUL, F32, F32, 0, 0)]
    ie = [col(8, I32), N_(capi.HY_EXPR_VALUE, I32, 0, 0, 3), N_(capi.HY_EXPR_MUL, I32, I32, 0, 0),
          N_(capi.HY_EXPR_VALUE, I32, 0, 0, 7), N_(capi.HY_EXPR_SUB, I32, I32, 0, 0)]
    progs = [(N_ * len(p))(*p) for p in (dp, ch, ie)]
    sizes = sizes[lo:hi]
    n_chunks = len(sizes)
    ac = (capi.AggColumn * 10)()
    pg = 0 if pos_lists is not None else -1
    specs = {0: (I32, dcols[0], doms[0]), 1: (I32, dcols[1], doms[1]), 2: (F32, dcols[2], 0),
             3: (F32, dcols[3], 0), 6: (F32, dcols[4], 0), 7: (F32, dcols[5], 0), 8: (I32, dcols[6], 0)}
    keep = []
    for j, (vt, c, dom) in specs.items():
        descs = c.descs if pos_lists is not None else c.descs[lo:hi]
        arr = (capi.ColumnChunk * len(descs))(*descs)
        keep.append(arr)
        ac[j].value_type, ac[j].pos_group, ac[j].chunks, ac[j].n_chunks, ac[j].domain = vt, pg, arr, len(descs), dom
    for j, p, t in ((4, progs[0], F32), (5, progs[1], F32), (9, progs[2], I32)):
        ac[j].value_type, ac[j].pos_group, ac[j].program, ac[j].n_nodes = t, -1, p, len(p)
    csz = (ctypes.c_uint32 * n_chunks)(*sizes)
    pls = (ctypes.c_void_p * max(1, n_chunks))(*([p.ptr.value for p in pos_lists[lo:hi]] if pos_lists is not None
                                                  else []))
    inp = capi.AggInput(n_chunks, csz, pls if pos_lists is not None else None, 1 if pos_lists is not None else 0,
                        ac, 10)
    if filt is not None:  # fused TableScan: (ScanChunk array, value type, constant array)
        inp.filter, inp.filter_value_type, inp.filter_constant = filt[0], filt[1], filt[2].ctypes.data
    gb = (ctypes.c_int32 * 2)(0, 1)
    defs = (capi.AggDef * len(aggs))(*[capi.AggDef(getattr(capi, "HY_AGG_" + f), c) for f, c in aggs])
    prm = capi.AggParams(gb, 2, defs, len(aggs), 0)
    lay = capi.AggLayout()
    capi.check(L.hy_aggregate_layout(ctypes.byref(inp), ctypes.byref(prm), ctypes.byref(lay)), "layout")
    assert lay.dense == 1
    wsb = ctypes.c_size_t()
    capi.check(L.hy_aggregate_workspace_size(ctypes.byref(inp), ctypes.byref(prm), ctypes.byref(wsb)), "ws")
    ws = capi.DeviceArray(np.zeros(wsb.value, np.uint8))
    out = capi.DeviceArray(np.zeros(64 * lay.words, np.uint64))
    ng = ctypes.c_uint64()
    capi.check(L.hy_aggregate(ctypes.byref(inp), ctypes.byref(prm), out.ptr, 64, ctypes.byref(ng), ws.ptr, wsb.value,
                              None), "hy_aggregate")
    rec = out.fetch().reshape(-1, lay.words)[:ng.value]
    if raw:
        return rec, lay, prm, (defs, gb)
    return decode(hy, rec, lay, aggs)


def decode(hy, rec, lay, aggs=AGGS):
    capi, L = hy.capi, hy.capi.lib
    res = {}
    for r in rec:
        g = (int(r[0]), int(r[1]))
        vals = {"rows": int(r[2 + 3])}
        for a, (f, c) in enumerate(aggs):
            wd = lay.agg_word[a]
            if c < 0:
                continue
            if f == "COUNT":
                vals[a] = int(r[wd])
            elif lay.agg_limbs[a] == 0:  # int32 input: int64 sum
                vals[a] = (int(r[wd]), int(np.array([r[wd + 1]], np.uint64).view(np.int64)[0]))
            else:
                limbs = (ctypes.c_uint64 * lay.agg_limbs[a])(*[int(x) for x in r[wd + 2:wd + 2 + lay.agg_limbs[a]]])
                sm = ctypes.c_double()
                capi.check(L.hy_agg_float_sum(limbs, lay.agg_limbs[a], lay.agg_emin[a], int(r[wd + 1]),
                                              ctypes.byref(sm)))
                vals[a] = (int(r[wd]), sm.value)
        res[g] = vals
    return res


def same_float(a, b):
    return (math.isnan(a) and math.isnan(b)) or a == b


def check(res, exp, aggs=AGGS):
    assert set(res) == set(exp)
    for g, e in exp.items():
        r = res[g]
        assert r["rows"] == e["rows"], g
        for a, (f, c) in enumerate(aggs):
            if c < 0:
                continue
            if f == "COUNT":
                assert r[a] == (e[c] if c == 7 else len(e[c])), (g, f, c)
                continue
            vals = e[c]
            assert r[a][0] == len(vals), (g, f, c)
            if c in (8, 9):
                assert r[a][1] == sum(vals), (g, f, c)
            else:
                assert same_float(r[a][1], fsum_inf(vals)), (g, f, c, r[a][1], fsum_inf(vals))


def kernels_ran(L):
    n = ctypes.c_uint32()
    L.hy_kernel_stats_collect(ctypes.byref(n))
    names = set()
    for i in range(n.value):
        nm, la, ms = ctypes.c_char_p(), ctypes.c_uint64(), ctypes.c_double()
        un = ctypes.c_uint64()
        L.hy_kernel_stats_get(i, ctypes.byref(nm), ctypes.byref(la), ctypes.byref(ms), ctypes.byref(un))
        names.add(nm.value.decode())
    return names


# data-input kernels under test: (HY_AGG_VEC, stream mode) -> the kernel that must run. Stream mode "j": the plan-compiled
# kernel agg_dense_jit (the default), "1": agg_dense_stream (HY_AGG_JIT=0), "0": neither (HY_AGG_STREAM=0) - the stream
# kernels where their preconditions hold (every dictionary <= 63 entries, so not with the "nulls" case's
# dictionary-encoded prices)
DATA_MODES = [("2", "j"), ("2", "1"), ("2", "0"), ("1", "0"), ("0", "0")]


def set_modes(monkeypatch, vec_mode, stream_mode):
    monkeypatch.setenv("HY_AGG_VEC", vec_mode)
    monkeypatch.setenv("HY_AGG_STREAM", "0" if stream_mode == "0" else "1")
    monkeypatch.setenv("HY_AGG_JIT", "1" if stream_mode == "j" else "0")


STREAM_KERNELS = {"agg_dense_jit", "agg_dense_stream"}


def only_kernel(want, ran):
    """`want` ran, and no other stream kernel did (a plan-compiled kernel that fails falls back to agg_dense_stream)."""
    return want in ran and not ((STREAM_KERNELS - {want}) & ran)


def data_kernel(vec_mode, stream_mode, stream_ok):
    if vec_mode != "2":
        return "agg_dense_lanes"
    if stream_mode == "0" or not stream_ok:
        return "agg_dense_vec"
    return {"j": "agg_dense_jit", "1": "agg_dense_stream"}[stream_mode]


@pytest.mark.parametrize("case", ["clean", "nulls", "null_ids", "odd_values", "wide_range", "drift", "many_groups",
                                  "clustered"])
@pytest.mark.parametrize("input_kind", ["data", "reference", "reference_mixed"])
def test_lanes_path(hy, monkeypatch, case, input_kind):
    capi = hy.capi
    L = capi.lib
    rng = np.random.default_rng(zlib.crc32(f"lanes/{case}/{input_kind}".encode()))
    cols = columns(rng, case)
    rf, ls, qty, price, disc, tax, iq, price_n, disc_n, doms = cols
    dcols = [dt.DeviceColumn(capi, rf, None, CHUNK, "Dictionary"), dt.DeviceColumn(capi, ls, None, CHUNK, "Dictionary"),
             dt.DeviceColumn(capi, qty, None, CHUNK, "Dictionary"),
             dt.DeviceColumn(capi, price, price_n if price_n.any() else None, CHUNK,
                             "Dictionary" if case == "nulls" else "Unencoded"),
             dt.DeviceColumn(capi, disc, disc_n, CHUNK, "Dictionary"), dt.DeviceColumn(capi, tax, None, CHUNK,
                                                                                       "Dictionary"),
             dt.DeviceColumn(capi, iq, None, CHUNK, "Unencoded")]
    n_chunks = dcols[0].n_chunks
    if input_kind == "data":
        rows = list(range(N))
        pos, sizes = None, [dcols[0].chunk_size(c) for c in range(n_chunks)]
    else:
        pos, sizes, rows = [], [], []
        for c in range(n_chunks):
            offs = np.nonzero(rng.random(dcols[0].chunk_size(c)) < 0.7)[0].astype(np.uint32)
            if input_kind == "reference_mixed":  # this chunk's PosList also references the next chunk
                nxt = (c + 1) % n_chunks
                more = np.nonzero(rng.random(dcols[0].chunk_size(nxt)) < 0.05)[0].astype(np.uint32)
                ids = np.concatenate([np.full(offs.size, c, np.uint32), np.full(more.size, nxt, np.uint32)])
                offs = np.concatenate([offs, more])
                order = np.argsort(rng.random(ids.size) + np.where(ids == c, 0.0, 0.3), kind="stable")
                ids, offs = ids[order], offs[order]
            else:
                ids = np.full(offs.size, c, np.uint32)
            pl = np.stack([ids, offs], axis=1).astype(np.uint32)
            pos.append(capi.DeviceArray(pl.reshape(-1) if pl.size else np.zeros(2, np.uint32)))
            sizes.append(pl.shape[0])
            rows += [int(i) * CHUNK + int(o) for i, o in zip(ids, offs)]
    exp = expected(cols, rows)
    # data input: agg_dense_stream (default), agg_dense_vec (HY_AGG_STREAM=0), agg_dense_lanes' contiguous instance
    # (HY_AGG_VEC=1) and its strided one (0)
    headers = {}
    for vec_mode, stream_mode in (DATA_MODES if input_kind == "data" else [("2", "j")]):
        set_modes(monkeypatch, vec_mode, stream_mode)
        L.hy_kernel_stats_enable(1)
        L.hy_kernel_stats_reset()
        res_lanes = run(hy, dcols, pos, sizes, doms)
        ran = kernels_ran(L)
        L.hy_kernel_stats_enable(0)
        # (the int32 expression chain of AGGS is not agg_dense_stream's: that set never streams)
        want = data_kernel(vec_mode, stream_mode, False) if input_kind == "data" else "agg_dense_lanes"
        assert only_kernel(want, ran), (vec_mode, stream_mode, ran)
        check(res_lanes, exp)
        headers[vec_mode + stream_mode] = {(int(r[0]), int(r[1])): tuple(int(x) for x in r[2:6])
                                           for r in run(hy, dcols, pos, sizes, doms, raw=True)[0]}
    if input_kind == "data":  # TPC-H 1's aggregate set: agg_dense_stream where it applies, against agg_dense_vec
        for vec_mode, stream_mode in DATA_MODES[:3]:
            set_modes(monkeypatch, vec_mode, stream_mode)
            L.hy_kernel_stats_enable(1)
            L.hy_kernel_stats_reset()
            res_q1 = run(hy, dcols, pos, sizes, doms, aggs=Q1_AGGS)
            ran = kernels_ran(L)
            L.hy_kernel_stats_enable(0)
            assert only_kernel(data_kernel(vec_mode, stream_mode, case != "nulls"), ran), (stream_mode, ran)
            check(res_q1, exp, Q1_AGGS)
            headers["q1/" + vec_mode + stream_mode] = {(int(r[0]), int(r[1])): tuple(int(x) for x in r[2:6])
                                                       for r in run(hy, dcols, pos, sizes, doms, raw=True,
                                                                    aggs=Q1_AGGS)[0]}
    monkeypatch.setenv("HY_AGG_LANES", "0")
    # NULL mask, first row, last row, rows of every group (the Aggregate's output order follows the first rows)
    fused_headers = {(int(r[0]), int(r[1])): tuple(int(x) for x in r[2:6])
                     for r in run(hy, dcols, pos, sizes, doms, raw=True)[0]}
    for mode, hd in headers.items():
        assert hd == fused_headers, mode
    res_fused = run(hy, dcols, pos, sizes, doms)
    check(res_fused, exp)
    assert res_lanes == res_fused or all(
        all(same_float(x[1], y[1]) if isinstance(x, tuple) else x == y for x, y in zip(res_lanes[g].values(),
                                                                                       res_fused[g].values()))
        for g in res_lanes)


@pytest.mark.parametrize("case", ["clean", "odd_values", "wide_range", "many_groups"])
@pytest.mark.parametrize("n_parts", [2, 3, 7])
def test_merge_of_partial_aggregates(hy, case, n_parts):
    """The multi-GPU Aggregate's merge (hy_aggregate_merge): the input's chunks split into contiguous ranges (one per
    rank), each aggregated alone, the partial records merged with the ranges' first global rows - equal to ONE
    aggregate over all chunks: same groups, first / last row words, counts, int sums, and float sums decoding to the
    same exactly rounded double (exact limb merge)."""
    capi, L = hy.capi, hy.capi.lib
    rng = np.random.default_rng(zlib.crc32(f"merge/{case}/{n_parts}".encode()))
    cols = columns(rng, case)
    rf, ls, qty, price, disc, tax, iq, price_n, disc_n, doms = cols
    dcols = [dt.DeviceColumn(capi, rf, None, CHUNK, "Dictionary"), dt.DeviceColumn(capi, ls, None, CHUNK, "Dictionary"),
             dt.DeviceColumn(capi, qty, None, CHUNK, "Dictionary"),
             dt.DeviceColumn(capi, price, price_n if price_n.any() else None, CHUNK, "Unencoded"),
             dt.DeviceColumn(capi, disc, disc_n if disc_n.any() else None, CHUNK, "Dictionary"),
             dt.DeviceColumn(capi, tax, None, CHUNK, "Dictionary"), dt.DeviceColumn(capi, iq, None, CHUNK, "Unencoded")]
    sizes = [d.size for d in dcols[0].descs]
    whole, lay, prm, _keep = run(hy, dcols, None, sizes, doms, raw=True)
    bounds = np.linspace(0, len(sizes), n_parts + 1).astype(int)
    parts, keep = [], []
    for p in range(n_parts):
        rec, _, _, k = run(hy, dcols, None, sizes, doms, part=(bounds[p], bounds[p + 1]), raw=True)
        parts.append(np.ascontiguousarray(rec, dtype=np.uint64))
        keep.append(k)
    ptrs = (ctypes.POINTER(ctypes.c_uint64) * n_parts)(*[p.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
                                                         for p in parts])
    ngs = (ctypes.c_uint64 * n_parts)(*[p.shape[0] for p in parts])
    bases = (ctypes.c_uint64 * n_parts)(*[int(sum(sizes[:bounds[p]])) for p in range(n_parts)])
    out = np.zeros((64, lay.words), np.uint64)
    n_out = ctypes.c_uint64()
    capi.check(L.hy_aggregate_merge(ctypes.byref(prm), ctypes.byref(lay), ptrs, ngs, bases, n_parts,
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 64, ctypes.byref(n_out)),
               "hy_aggregate_merge")
    merged = out[:n_out.value]
    assert n_out.value == whole.shape[0]
    by_key = lambda recs: {(int(r[0]), int(r[1])): r for r in recs}
    mw, ww = by_key(merged), by_key(whole)
    assert set(mw) == set(ww)
    for g in ww:  # NULL mask, first row, last row, rows
        assert np.array_equal(mw[g][2:6], ww[g][2:6]), g
    dm, dw = decode(hy, merged, lay), decode(hy, whole, lay)
    for g, vals in dw.items():
        for k, v in vals.items():
            a = dm[g][k]
            if isinstance(v, tuple) and isinstance(v[1], float):
                assert a[0] == v[0] and same_float(a[1], v[1]), (g, k, a, v)
            else:
                assert a == v, (g, k, a, v)


@pytest.mark.parametrize("pred_enc,cond,value", [("Dictionary", "LessThanEquals", 300), ("Unencoded", "LessThan", 250),
                                                 ("Dictionary", "GreaterThan", 1000), ("Dictionary", "LessThan", 0)])
@pytest.mark.parametrize("case", ["clean", "nulls", "odd_values"])
def test_fused_scan_filter(hy, monkeypatch, case, pred_enc, cond, value):
    """hy_aggregate with a fused TableScan (hy_agg_input.filter) over a data input: every aggregate equals the
    aggregate of exactly the matching rows (numpy over the predicate's rows) - TPC-H 1's Scan -> Aggregate in one
    pass, the lanes path and the steps it defers to agg_dense_fused (NULLs, odd values) alike; predicates with all,
    some and no matches, dictionary (u16 vids: value ids compared after the host's dictionary rewrite) and value."""
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(f"filter/{case}/{pred_enc}/{cond}/{value}".encode()))
    cols = columns(rng, case)
    rf, ls, qty, price, disc, tax, iq, price_n, disc_n, doms = cols
    ship = rng.integers(0, 1000, N).astype(np.int32)  # > 256 distinct values: 2-byte value ids
    dcols = [dt.DeviceColumn(capi, rf, None, CHUNK, "Dictionary"), dt.DeviceColumn(capi, ls, None, CHUNK, "Dictionary"),
             dt.DeviceColumn(capi, qty, None, CHUNK, "Dictionary"),
             dt.DeviceColumn(capi, price, price_n if price_n.any() else None, CHUNK,
                             "Dictionary" if case == "nulls" else "Unencoded"),
             dt.DeviceColumn(capi, disc, disc_n, CHUNK, "Dictionary"),
             dt.DeviceColumn(capi, tax, None, CHUNK, "Dictionary"), dt.DeviceColumn(capi, iq, None, CHUNK, "Unencoded")]
    pred = dt.DeviceColumn(capi, ship, None, CHUNK, pred_enc)
    chunks = pred.scan_chunks(cond, value)
    sizes = [d.size for d in dcols[0].descs]
    op = {"LessThanEquals": np.less_equal, "LessThan": np.less, "GreaterThan": np.greater}[cond]
    rows = list(np.nonzero(op(ship, value))[0])
    # stream (TPC-H 1's aggregate set), vec, lanes (strided)
    for vec_mode, stream_mode, aggs in (("2", "j", Q1_AGGS), ("2", "1", Q1_AGGS), ("2", "0", AGGS), ("0", "0", AGGS)):
        set_modes(monkeypatch, vec_mode, stream_mode)
        capi.lib.hy_kernel_stats_enable(1)
        capi.lib.hy_kernel_stats_reset()
        res = run(hy, dcols, None, sizes, doms, filt=(chunks, capi.HY_TYPE_INT32, pred.constant(value)), aggs=aggs)
        ran = kernels_ran(capi.lib)
        capi.lib.hy_kernel_stats_enable(0)
        # agg_dense_stream takes dictionary id-range filters only
        assert only_kernel(data_kernel(vec_mode, stream_mode, case != "nulls" and pred_enc == "Dictionary"), ran), ran
        check(res, expected(cols, rows), aggs)


@pytest.mark.parametrize("case", ["clean", "nulls", "null_ids", "drift"])
@pytest.mark.parametrize("cond,value", [("LessThanEquals", 300), ("GreaterThan", 700)])
@pytest.mark.parametrize("stream_mode", ["j", "1", "0"])
def test_fused_scan_filter_against_oracle(hy, oracle, monkeypatch, case, cond, value, stream_mode):
    """agg_dense_jit / agg_dense_stream / agg_dense_vec with the TableScan fused (TPC-H 1's default plan) against the ORACLE's plan on
    the same table:
    oracle TableScan (single_column_table_scan_impl.cpp) -> Projection of the two float expressions
    (projection.cpp:39-87) -> Aggregate (aggregate.cpp:203-249, sequential double sums). Group keys, counts and int
    sums equal; every float SUM / AVG is the exactly rounded sum (== math.fsum of the projected values) and within
    1 ULP of the oracle's sequential sum, the north star's bar."""
    capi, L = hy.capi, hy.capi.lib
    rng = np.random.default_rng(zlib.crc32(f"vec-oracle/{case}/{cond}/{value}".encode()))
    cols = columns(rng, case)
    rf, ls, qty, price, disc, tax, iq, price_n, disc_n, doms = cols
    ship = rng.integers(0, 1000, N).astype(np.int32)
    dcols = [dt.DeviceColumn(capi, rf, None, CHUNK, "Dictionary"), dt.DeviceColumn(capi, ls, None, CHUNK, "Dictionary"),
             dt.DeviceColumn(capi, qty, None, CHUNK, "Dictionary"),
             dt.DeviceColumn(capi, price, price_n if price_n.any() else None, CHUNK,
                             "Dictionary" if case == "nulls" else "Unencoded"),
             dt.DeviceColumn(capi, disc, disc_n if disc_n.any() else None, CHUNK, "Dictionary"),
             dt.DeviceColumn(capi, tax, None, CHUNK, "Dictionary"), dt.DeviceColumn(capi, iq, None, CHUNK, "Unencoded")]
    pred = dt.DeviceColumn(capi, ship, None, CHUNK, "Dictionary")
    sizes = [d.size for d in dcols[0].descs]
    set_modes(monkeypatch, "2", stream_mode)
    L.hy_kernel_stats_enable(1)
    L.hy_kernel_stats_reset()
    aggs = Q1_AGGS if stream_mode != "0" else AGGS  # (agg_dense_stream: TPC-H 1's set, no int32 chain)
    res = run(hy, dcols, None, sizes, doms,
              filt=(pred.scan_chunks(cond, value), capi.HY_TYPE_INT32, pred.constant(value)), aggs=aggs)
    ran = kernels_ran(L)
    L.hy_kernel_stats_enable(0)
    assert only_kernel(data_kernel("2", stream_mode, case != "nulls"), ran), ran

    # the oracle's plan over a table of the same columns
    T = hy.DataType
    table = hy.Table.from_arrays(
        [("rf", T.Int, False), ("ls", T.Int, False), ("qty", T.Float, False), ("price", T.Float, True),
         ("disc", T.Float, True), ("tax", T.Float, False), ("iq", T.Int, False), ("ship", T.Int, False)],
        [rf, ls, qty, price, disc, tax, iq, ship], [None, None, None, price_n, disc_n, None, None, None], CHUNK)
    hy.encode_columns(table, [7], hy.EncodingType.Dictionary)
    scan = oracle.table_scan(table, 7, getattr(hy.PredicateCondition, cond), value, [])
    c = lambda i: hy.PQPColumnExpression.from_table(scan, i)
    A = hy.ArithmeticOperator
    one = hy.ValueExpression(1)
    dp = hy.ArithmeticExpression(A.Multiplication, c(3), hy.ArithmeticExpression(A.Subtraction, one, c(4)))
    ch = hy.ArithmeticExpression(A.Multiplication, dp, hy.ArithmeticExpression(A.Addition, one, c(5)))
    ie = hy.ArithmeticExpression(A.Subtraction, hy.ArithmeticExpression(A.Multiplication, c(6), hy.ValueExpression(3)),
                                 hy.ValueExpression(7))
    # projected columns in the C-ABI test's numbering: 0 rf, 1 ls, 2 qty, 3 price, 4 dp, 5 ch, 6 disc, 7 tax, 8 iq, 9 ie
    proj = oracle.projection(scan, [c(0), c(1), c(2), c(3), dp, ch, c(4), c(5), c(6), ie])
    F = {"SUM": "Sum", "AVG": "Avg", "COUNT": "Count"}
    defs = [hy.AggregateColumnDefinition(None if col < 0 else col, getattr(hy.AggregateFunction, F[f]))
            for f, col in aggs]
    agg = oracle.aggregate(proj, defs, [0, 1])
    want = {(r[0], r[1]): r[2:] for r in agg.rows()}
    proj_rows = proj.rows()
    assert set(res) == set(want)
    for g, vals in res.items():
        members = [r for r in proj_rows if (r[0], r[1]) == g]
        for a, (f, col) in enumerate(aggs):
            w = want[g][a]
            if f == "COUNT":
                got = vals["rows"] if col < 0 else vals[a]
                assert got == w, (g, f, col)
                continue
            n, s = vals[a]
            if col in (8, 9):  # int32 inputs: int64 sums, exact
                assert (s if f == "SUM" else s / n) == w, (g, f, col)
                continue
            exact = math.fsum(r[col] for r in members if r[col] is not None)
            got = s if f == "SUM" else s / n
            assert s == exact, (g, f, col)  # the exactly rounded sum
            assert abs(int(np.float64(got).view(np.int64)) - int(np.float64(w).view(np.int64))) <= 1, (g, f, col, got, w)
