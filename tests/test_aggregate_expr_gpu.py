"""Expression columns of hy_aggregate (the Projection fused into the Aggregate, TPC-H 1's
SUM(l_extendedprice * (1 - l_discount)) shape; reference projection.cpp:39-87 feeding aggregate.cpp:133-249): every
path - agg_dense_fused (expressions evaluated in the kernel), the materialised fallback (HY_AGG_FUSED=0: projection
kernel, then agg_dense_span / agg_dense_rows) and the hash path - on data and reference inputs (PosLists into one
chunk, and PosLists mixing chunks), with NULLs, against numpy: expressions in float32 exactly as the reference's
float functors compute them (NULL if an operand is NULL), group counts exact, float SUM/AVG equal to the exactly
rounded sum (math.fsum), MIN/MAX exact."""
import ctypes
import math
import zlib

import numpy as np
import pytest

import device_tables as dt

pytestmark = pytest.mark.gpu

N, CHUNK = 50_000, 7_000


def data(rng):
    rf = rng.integers(0, 3, N).astype(np.int32)
    ls = rng.integers(0, 2, N).astype(np.int32)
    qty = rng.integers(1, 51, N).astype(np.float32)
    price = (rng.integers(90_000, 210_001, N) * qty.astype(np.int64) / 100.0).astype(np.float32)
    disc = (rng.integers(0, 11, N) / 100.0).astype(np.float32)
    tax = (rng.integers(0, 9, N) / 100.0).astype(np.float32)
    price_n = (rng.random(N) < 0.03).astype(np.uint8)
    disc_n = (rng.random(N) < 0.02).astype(np.uint8)
    price[rng.random(N) < 0.001] = np.float32(-3.5e-30)  # a tiny value outside a step's exponent window
    return rf, ls, qty, price, disc, tax, price_n, disc_n


def expected(rf, ls, qty, price, disc, tax, price_n, disc_n, rows):
    one = np.float32(1)
    dp = (price * (one - disc)).astype(np.float32)
    ch = (dp * (one + tax)).astype(np.float32)
    dp_null = (price_n | disc_n).astype(bool)
    out = {}
    for r in rows:
        g = (int(rf[r]), int(ls[r]))
        e = out.setdefault(g, {"rows": 0, "qty": [], "price": [], "dp": [], "ch": []})
        e["rows"] += 1
        e["qty"].append(float(qty[r]))
        if not price_n[r]:
            e["price"].append(float(price[r]))
        if not dp_null[r]:
            e["dp"].append(float(dp[r]))
            e["ch"].append(float(ch[r]))
    return out


AGGS = [("SUM", 2), ("SUM", 3), ("SUM", 4), ("SUM", 5), ("AVG", 4), ("MIN", 5), ("MAX", 4), ("COUNT", 4),
        ("COUNT", -1)]


def run(hy, cols, pos_lists, sizes, dense):
    """hy_aggregate over columns [rf, ls, qty, price, dp(expr), ch(expr), disc, tax]; returns decoded groups."""
    capi, L = hy.capi, hy.capi.lib
    I32, F32 = capi.HY_TYPE_INT32, capi.HY_TYPE_FLOAT
    N_ = capi.ExprNode
    col = lambda j: N_(capi.HY_EXPR_COLUMN, F32, 0, j, 0)
    one = N_(capi.HY_EXPR_VALUE, I32, 0, 0, 1)
    dp = [col(3), one, col(6), N_(capi.HY_EXPR_SUB, F32, F32, 0, 0), N_(capi.HY_EXPR_MUL, F32, F32, 0, 0)]
    ch = dp + [one, col(7), N_(capi.HY_EXPR_ADD, F32, F32, 0, 0), N_(capi.HY_EXPR_MUL, F32, F32, 0, 0)]
    progs = [(N_ * len(p))(*p) for p in (dp, ch)]
    n_chunks = len(sizes)
    ac = (capi.AggColumn * 8)()
    pg = 0 if pos_lists is not None else -1
    specs = {0: (I32, cols[0], 3 if dense else 0), 1: (I32, cols[1], 2 if dense else 0), 2: (F32, cols[2], 0),
             3: (F32, cols[3], 0), 6: (F32, cols[4], 0), 7: (F32, cols[5], 0)}
    keep = []
    for j, (vt, c, dom) in specs.items():
        arr = (capi.ColumnChunk * len(c.descs))(*c.descs)
        keep.append(arr)
        ac[j].value_type, ac[j].pos_group, ac[j].chunks, ac[j].n_chunks, ac[j].domain = vt, pg, arr, len(c.descs), dom
    for j, p in ((4, progs[0]), (5, progs[1])):
        ac[j].value_type, ac[j].pos_group, ac[j].program, ac[j].n_nodes = F32, -1, p, len(p)
    csz = (ctypes.c_uint32 * n_chunks)(*sizes)
    pls = (ctypes.c_void_p * max(1, n_chunks))(*([p.ptr.value for p in pos_lists] if pos_lists is not None else []))
    inp = capi.AggInput(n_chunks, csz, pls if pos_lists is not None else None, 1 if pos_lists is not None else 0,
                        ac, 8)
    gb = (ctypes.c_int32 * 2)(0, 1)
    defs = (capi.AggDef * len(AGGS))(*[capi.AggDef(getattr(capi, "HY_AGG_" + f), c) for f, c in AGGS])
    prm = capi.AggParams(gb, 2, defs, len(AGGS), 0)
    lay = capi.AggLayout()
    capi.check(L.hy_aggregate_layout(ctypes.byref(inp), ctypes.byref(prm), ctypes.byref(lay)), "layout")
    assert bool(lay.dense) == dense
    wsb = ctypes.c_size_t()
    capi.check(L.hy_aggregate_workspace_size(ctypes.byref(inp), ctypes.byref(prm), ctypes.byref(wsb)), "ws")
    ws = capi.DeviceArray(np.zeros(wsb.value, np.uint8))
    out = capi.DeviceArray(np.zeros(64 * lay.words, np.uint64))
    ng = ctypes.c_uint64()
    capi.check(L.hy_aggregate(ctypes.byref(inp), ctypes.byref(prm), out.ptr, 64, ctypes.byref(ng), ws.ptr, wsb.value,
                              None), "hy_aggregate")
    rec = out.fetch().reshape(-1, lay.words)[:ng.value]
    res = {}
    for r in rec:
        g = (int(r[0]), int(r[1]))
        vals = {"rows": int(r[2 + 3])}
        for a, (f, c) in enumerate(AGGS):
            wd = lay.agg_word[a]
            if c < 0:
                continue
            if f == "COUNT":
                vals[a] = int(r[wd])
            elif f in ("MIN", "MAX"):
                b = L.hy_agg_decode_ordered(int(r[wd + 1]), capi.HY_TYPE_FLOAT)
                vals[a] = (int(r[wd]), float(np.array([b], np.uint32).view(np.float32)[0]))
            else:
                limbs = (ctypes.c_uint64 * lay.agg_limbs[a])(*[int(x) for x in r[wd + 2:wd + 2 + lay.agg_limbs[a]]])
                sm = ctypes.c_double()
                capi.check(L.hy_agg_float_sum(limbs, lay.agg_limbs[a], lay.agg_emin[a], int(r[wd + 1]),
                                              ctypes.byref(sm)))
                vals[a] = (int(r[wd]), sm.value)
        res[g] = vals
    return res


def check(res, exp):
    assert set(res) == set(exp)
    names = {2: "qty", 3: "price", 4: "dp", 5: "ch"}
    for g, e in exp.items():
        r = res[g]
        assert r["rows"] == e["rows"]
        for a, (f, c) in enumerate(AGGS):
            if c < 0:
                continue
            vals = e[names[c]]
            if f == "COUNT":
                assert r[a] == len(vals)
            elif f == "SUM":
                assert r[a] == (len(vals), math.fsum(vals)), (g, f, c)
            elif f == "AVG":
                assert r[a][0] == len(vals) and r[a][1] == math.fsum(vals), (g, f, c)
            else:
                assert r[a] == (len(vals), (min if f == "MIN" else max)(vals)), (g, f, c)


@pytest.mark.parametrize("path", ["fused", "materialized", "hash"])
@pytest.mark.parametrize("input_kind", ["data", "reference", "reference_mixed"])
def test_expression_columns(hy, monkeypatch, path, input_kind):
    capi = hy.capi
    rng = np.random.default_rng(zlib.crc32(f"{path}/{input_kind}".encode()))
    rf, ls, qty, price, disc, tax, price_n, disc_n = data(rng)
    cols = [dt.DeviceColumn(capi, rf, None, CHUNK, "Dictionary"), dt.DeviceColumn(capi, ls, None, CHUNK, "Dictionary"),
            dt.DeviceColumn(capi, qty, None, CHUNK, "Dictionary"), dt.DeviceColumn(capi, price, price_n, CHUNK,
                                                                                   "Unencoded"),
            dt.DeviceColumn(capi, disc, disc_n, CHUNK, "Dictionary"), dt.DeviceColumn(capi, tax, None, CHUNK,
                                                                                      "Dictionary")]
    n_chunks = cols[0].n_chunks
    if path == "materialized":
        monkeypatch.setenv("HY_AGG_FUSED", "0")
    if input_kind == "data":
        rows = list(range(N))
        pos, sizes = None, [cols[0].chunk_size(c) for c in range(n_chunks)]
    else:
        pos, sizes, rows = [], [], []
        for c in range(n_chunks):
            offs = np.nonzero(rng.random(cols[0].chunk_size(c)) < 0.6)[0].astype(np.uint32)
            if input_kind == "reference_mixed":  # this chunk's PosList also references the next chunk
                nxt = (c + 1) % n_chunks
                more = np.nonzero(rng.random(cols[0].chunk_size(nxt)) < 0.1)[0].astype(np.uint32)
                ids = np.concatenate([np.full(offs.size, c, np.uint32), np.full(more.size, nxt, np.uint32)])
                offs = np.concatenate([offs, more])
                order = rng.permutation(ids.size)
                ids, offs = ids[order], offs[order]
            else:
                ids = np.full(offs.size, c, np.uint32)
            pl = np.stack([ids, offs], axis=1).astype(np.uint32)
            pos.append(capi.DeviceArray(pl.reshape(-1) if pl.size else np.zeros(2, np.uint32)))
            sizes.append(pl.shape[0])
            rows += [int(i) * CHUNK + int(o) for i, o in zip(ids, offs)]
    res = run(hy, cols, pos, sizes, dense=(path != "hash"))
    check(res, expected(rf, ls, qty, price, disc, tax, price_n, disc_n, rows))
