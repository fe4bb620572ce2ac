"""The multi-GPU Aggregate plans of SURVEY.md 8(e), restated on the CPU and run over gloo with 2 and 3 ranks, against
the oracle on the whole table:

* TPC-H 3 (BASELINE.json configs[4]) as bench_q3_dist.py runs it: each rank takes contiguous chunk ranges of customer,
  orders and lineitem (bench_q3_dist.shard_q3), all-gathers its customer matches (broadcast side of join 1), joins them
  with its orders shard, picks join 2's radix bits from the all-reduced global join-1 size (join_hash.cpp:640-668),
  forms the exchange records {key, row} of both sides grouped by first-digit bucket (murmur2 seed 17, bucket ownership
  as hy_join_exchange_bucket_bits / dist.owned_buckets) with the projection's columns carried in record order, routes
  them with dist.exchange_columns (all_gather + all_to_all_single, the bench's own plumbing), and aggregates GROUP BY
  l_orderkey, o_orderdate, o_shippriority over the partitions it owns. The ranks' groups must be disjoint and their
  union must equal the oracle's TPC-H 3 chain on the whole tables, every SUM exactly.
* TPC-H 1 (BASELINE.json configs[3] on N GPUs): each rank's partial group records in hy_aggregate's record layout
  (hy_aggregate_layout; float sums as exact fixed-point limbs) are all-gathered and merged by the library's own
  hy_aggregate_merge (host code of the C-ABI); the merged groups must equal the oracle's TPC-H 1 chain on the whole
  table: counts exactly, every SUM / AVG equal to the exactly rounded sum of the float32 inputs and within 1e-12 of
  the oracle's sequential double sums.

The device side of the same plans is covered by tests/test_dist_q3_gpu.py and test_aggregate_lanes_gpu.py."""
import ctypes
import importlib
import math
import os
import socket

import numpy as np
import pytest

from helpers import load_oracle, load_pkg, murmur2_int32_np

Q3_SF, Q1_SF, CHUNK = 0.01, 0.01, 2_000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


# ----------------------------------------------------------------------------------------------------------------
# TPC-H 3
# ----------------------------------------------------------------------------------------------------------------
def _q3_worker(rank, world, port, out_dir):
    import torch

    dist = _init(rank, world, port)
    try:
        hy = load_pkg()
        L = hy.capi.lib
        synth = importlib.import_module("hyrise-1_amd.synth")
        hd = importlib.import_module("hyrise-1_amd.dist")
        q3d = importlib.import_module("bench_q3_dist")
        D = synth.DATE_1995_03_15
        cols = synth.q3_columns(Q3_SF, "cpu")
        cols.pop("l_order_index")
        sh = {k: v.numpy() for k, v in q3d.shard_q3(cols, CHUNK, rank, world).items()}
        # A: customer scan on the shard; all-gather of the matches' keys (rank order = global scan order)
        ck = torch.from_numpy(np.ascontiguousarray(sh["c_custkey"][sh["c_mktsegment"] == 1]))
        ns = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(ns, torch.tensor([ck.numel()], dtype=torch.int64))
        m = max(int(n) for n in ns)
        buf = torch.zeros(max(1, m), dtype=torch.int32)
        buf[: ck.numel()] = ck
        parts = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf)
        gathered = np.concatenate([p[: int(n)].numpy() for p, n in zip(parts, ns)])
        # B: join 1, local (the orders scan o_orderdate < D fused; customer matches build)
        j1 = (sh["o_orderdate"] < D) & np.isin(sh["o_custkey"], gathered)
        total = torch.tensor([int(j1.sum())], dtype=torch.int64)
        dist.all_reduce(total)
        bits = int(L.hy_join_radix_bits(int(total.item()), 4))
        w0 = int(L.hy_join_exchange_bucket_bits(bits, world))
        n_buckets = 1 << w0

        def grouped(keys, carried):  # exchange records grouped by first-digit bucket (stable), carried columns alike
            bucket = (murmur2_int32_np(keys).astype(np.int64) & ((1 << bits) - 1)) >> (bits - w0)
            order = np.argsort(bucket, kind="stable")
            cols_ = [torch.from_numpy(np.ascontiguousarray(a[order])) for a in [keys] + carried]
            return cols_, np.bincount(bucket, minlength=n_buckets)

        bcols, bcnt = grouped(sh["o_orderkey"][j1], [sh["o_orderdate"][j1], sh["o_shippriority"][j1]])
        lm = sh["l_shipdate"] > D  # the lineitem scan fused into the probe side's exchange partition
        rev = (sh["l_extendedprice"][lm] * (np.float32(1) - sh["l_discount"][lm])).astype(np.float32)
        pcols, pcnt = grouped(sh["l_orderkey"][lm], [rev])
        (bk, bd, bp), _ = hd.exchange_columns(dist, bcols, bcnt, rank, world)
        (pk, pr), _ = hd.exchange_columns(dist, pcols, pcnt, rank, world)
        # D: join 2 over the owned partitions (every received key's partition is owned here) + local GROUP BY
        lo, hi = hd.owned_buckets(n_buckets, rank, world)
        for k in (bk.numpy(), pk.numpy()):
            b = (murmur2_int32_np(k).astype(np.int64) & ((1 << bits) - 1)) >> (bits - w0)
            assert ((b >= lo) & (b < hi)).all()
        build = {}
        for k, d, p in zip(bk.tolist(), bd.tolist(), bp.tolist()):
            build.setdefault(k, []).append((d, p))
        groups = {}
        for k, r in zip(pk.tolist(), pr.tolist()):
            for d, p in build.get(k, []):
                groups.setdefault((k, d, p), []).append(r)
        out = {g: math.fsum(v) for g, v in groups.items()}
        np.save(os.path.join(out_dir, f"q3_r{rank}.npy"),
                np.array([[g[0], g[1], g[2], s] for g, s in out.items()], dtype=np.float64).reshape(-1, 4))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_q3_plan_equals_oracle(tmp_path, world):
    import torch.multiprocessing as mp

    from q3_oracle import oracle_q3

    hy = load_pkg()
    synth = importlib.import_module("hyrise-1_amd.synth")
    mp.spawn(_q3_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = {}
    for r in range(world):
        for row in np.load(tmp_path / f"q3_r{r}.npy"):
            key = (int(row[0]), int(row[1]), int(row[2]))
            assert key not in got, f"group {key} on two ranks"
            got[key] = float(row[3])
    cols = {k: v.numpy() for k, v in synth.q3_columns(Q3_SF, "cpu").items()}
    want, _, _ = oracle_q3(hy, cols, CHUNK)
    assert len(want) > 100 and set(got) == set(want)
    assert all(got[k] == want[k] for k in want)


# ----------------------------------------------------------------------------------------------------------------
# TPC-H 1
# ----------------------------------------------------------------------------------------------------------------
Q1_AGGS = [("SUM", 2), ("SUM", 3), ("SUM", 4), ("SUM", 5), ("AVG", 2), ("AVG", 3), ("AVG", 6), ("COUNT", -1)]


def _q1_layout(capi):
    """hy_aggregate_layout of bench_tpch's TPC-H 1 input: returnflag / linestatus codes (dense domains 3 / 2) and six
    float columns (quantity, price, disc_price, charge, discount, tax)."""
    I32, F32 = capi.HY_TYPE_INT32, capi.HY_TYPE_FLOAT
    chunks = [(capi.ColumnChunk * 1)() for _ in range(8)]
    cols = (capi.AggColumn * 8)()
    for j in range(8):
        chunks[j][0].size = 1
        chunks[j][0].kind = capi.HY_COL_VALUE
        cols[j].value_type, cols[j].pos_group, cols[j].chunks, cols[j].n_chunks = (I32 if j < 2 else F32), -1, \
            chunks[j], 1
    cols[0].domain, cols[1].domain = 3, 2
    sizes = (ctypes.c_uint32 * 1)(1)
    ain = capi.AggInput(1, sizes, None, 0, cols, 8)
    fn = {"SUM": capi.HY_AGG_SUM, "AVG": capi.HY_AGG_AVG, "COUNT": capi.HY_AGG_COUNT}
    defs = (capi.AggDef * len(Q1_AGGS))(*[capi.AggDef(fn[f], c) for f, c in Q1_AGGS])
    gb = (ctypes.c_int32 * 2)(0, 1)
    prm = capi.AggParams(gb, 2, defs, len(Q1_AGGS), 0)
    lay = capi.AggLayout()
    capi.check(capi.lib.hy_aggregate_layout(ctypes.byref(ain), ctypes.byref(prm), ctypes.byref(lay)), "layout")
    prm._keep = (gb, defs)
    return lay, prm


def _exact_limbs(values, emin, n_limbs):
    """The exact sum of float32 values as n_limbs signed base-2^32 digits of weight 2^(32 i + emin) (the record's
    fixed-point float sum)."""
    m, e = np.frexp(values.astype(np.float64))
    mant = np.round(m * (1 << 24)).astype(np.int64)  # float32: 24-bit significands, exact
    x = 0
    for ex in np.unique(e):
        s = int(mant[e == ex].sum())
        shift = int(ex) - 24 - emin
        x += s << shift if shift >= 0 else s >> -shift
    limbs = []
    for i in range(n_limbs - 1):
        limbs.append((x >> (32 * i)) & 0xFFFFFFFF)
    limbs.append((x >> (32 * (n_limbs - 1))) & 0xFFFFFFFFFFFFFFFF)  # signed top limb, two's complement
    return limbs


def _q1_inputs(synth, sf):
    c = {k: v.numpy() for k, v in synth.q1_columns(sf, "cpu").items()}
    price, disc, tax = c["l_extendedprice"], c["l_discount"], c["l_tax"]
    dp = (price * (np.float32(1) - disc)).astype(np.float32)
    ch = (dp * (np.float32(1) + tax)).astype(np.float32)
    return c, [c["l_quantity"], price, dp, ch, disc, tax]


def _q1_worker(rank, world, port, out_dir):
    import torch

    dist = _init(rank, world, port)
    try:
        hy = load_pkg()
        capi = hy.capi
        synth = importlib.import_module("hyrise-1_amd.synth")
        lay, prm = _q1_layout(capi)
        c, vals = _q1_inputs(synth, Q1_SF)
        n = c["l_shipdate"].size
        n_chunks = (n + CHUNK - 1) // CHUNK
        lo, hi = min(n, rank * n_chunks // world * CHUNK), min(n, (rank + 1) * n_chunks // world * CHUNK)
        keep = c["l_shipdate"][lo:hi] <= synth.DATE_1998_09_02  # the shard's TableScan
        rf, ls = c["l_returnflag"][lo:hi][keep], c["l_linestatus"][lo:hi][keep]
        vals = [v[lo:hi][keep] for v in vals]
        W = lay.words
        recs = np.zeros((64, W), np.uint64)
        g = 0
        for f in range(3):
            for s in range(2):
                idx = np.nonzero((rf == f) & (ls == s))[0]
                if idx.size == 0:
                    continue
                r = recs[g]
                r[0], r[1], r[2], r[3], r[4], r[5] = f, s, 0, idx[0], idx[-1], idx.size
                for a, (fn, col) in enumerate(Q1_AGGS):
                    if col < 0:
                        continue
                    w = lay.agg_word[a]
                    r[w], r[w + 1] = idx.size, 0
                    r[w + 2:w + 2 + lay.agg_limbs[a]] = _exact_limbs(vals[col - 2][idx], lay.agg_emin[a],
                                                                     lay.agg_limbs[a])
                g += 1
        buf = torch.from_numpy(np.concatenate([[g], recs.view(np.int64).ravel()]).astype(np.int64))
        parts = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf)
        bases = [0]
        cnt = torch.tensor([int(keep.sum())], dtype=torch.int64)
        counts = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(counts, cnt)
        for x in counts[:-1]:
            bases.append(bases[-1] + int(x))
        if rank == 0:
            host = [np.ascontiguousarray(p.numpy().view(np.uint64)) for p in parts]
            ptrs = (ctypes.POINTER(ctypes.c_uint64) * world)(
                *[h[1:].ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)) for h in host])
            ngs = (ctypes.c_uint64 * world)(*[int(h[0]) for h in host])
            bs = (ctypes.c_uint64 * world)(*bases)
            merged = np.zeros((64, W), np.uint64)
            n_out = ctypes.c_uint64()
            capi.check(capi.lib.hy_aggregate_merge(ctypes.byref(prm), ctypes.byref(lay), ptrs, ngs, bs, world,
                                                   merged.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 64,
                                                   ctypes.byref(n_out)), "hy_aggregate_merge")
            np.save(os.path.join(out_dir, "q1_merged.npy"), merged[: n_out.value])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_q1_merge_equals_oracle(tmp_path, world):
    import torch.multiprocessing as mp

    hy = load_pkg()
    capi, oracle = hy.capi, load_oracle()
    synth = importlib.import_module("hyrise-1_amd.synth")
    mp.spawn(_q1_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    merged = np.load(tmp_path / "q1_merged.npy")
    lay, _ = _q1_layout(capi)
    c, vals = _q1_inputs(synth, Q1_SF)
    keep = c["l_shipdate"] <= synth.DATE_1998_09_02
    # the oracle's TPC-H 1 chain on the whole table (bench_tpch.cpu_baseline_q1's plan)
    I, F = hy.DataType.Int, hy.DataType.Float
    names = ["l_returnflag", "l_linestatus", "l_quantity", "l_extendedprice", "l_discount", "l_tax", "l_shipdate"]
    t = hy.Table.from_arrays([(nm, ty, False) for nm, ty in zip(names, [I, I, F, F, F, F, I])],
                             [c[nm] for nm in names], [], CHUNK)
    hy.encode_all_chunks(t, hy.EncodingType.Dictionary)
    P, A, O, V = (hy.PQPColumnExpression.from_table, hy.ArithmeticExpression, hy.ArithmeticOperator,
                  hy.ValueExpression)
    s = oracle.table_scan(t, 6, hy.PredicateCondition.LessThanEquals, synth.DATE_1998_09_02, [])
    dp = A(O.Multiplication, P(s, 3), A(O.Subtraction, V(1), P(s, 4)))
    p = oracle.projection(s, [P(s, 0), P(s, 1), P(s, 2), P(s, 3), dp,
                              A(O.Multiplication, dp, A(O.Addition, V(1), P(s, 5))), P(s, 4)])
    aggs = [hy.AggregateColumnDefinition(None if col < 0 else col, getattr(hy.AggregateFunction, f.capitalize()))
            for f, col in Q1_AGGS]
    want = {(int(r[0]), int(r[1])): r[2:] for r in oracle.aggregate(p, aggs, [0, 1]).rows()}
    assert len(merged) == len(want) >= 3

    def fsum(r, a):
        w = lay.agg_word[a]
        limbs = (ctypes.c_uint64 * lay.agg_limbs[a])(*[int(x) for x in r[w + 2:w + 2 + lay.agg_limbs[a]]])
        out = ctypes.c_double(0)
        capi.check(capi.lib.hy_agg_float_sum(limbs, lay.agg_limbs[a], lay.agg_emin[a], int(r[w + 1]),
                                             ctypes.byref(out)))
        return out.value

    for r in merged:
        key = (int(r[0]), int(r[1]))
        sel = keep & (c["l_returnflag"] == key[0]) & (c["l_linestatus"] == key[1])
        rows = int(r[5])
        assert rows == int(sel.sum()) == want[key][7]
        for a, (fn, col) in enumerate(Q1_AGGS[:7]):
            exact = math.fsum(vals[col - 2][sel].astype(np.float64))
            got = fsum(r, a) if fn == "SUM" else fsum(r, a) / rows
            ref = exact if fn == "SUM" else exact / rows
            assert got == ref, (key, fn, col)
            assert abs(got - want[key][a]) <= 1e-12 * abs(ref), (key, fn, col, got, want[key][a])
