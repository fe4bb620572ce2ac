"""Seeded, counter-based synthetic TPC-H-shaped columns.

Every value is a pure function of (seed, global row index), so any shard regenerates its rows independently and the
torch (device) and numpy (host) generators produce identical data:

* orders:   o_orderkey = dbgen sparse key ((i >> 3) << 5) + (i & 7) for i = 1..1.5M*SF (third_party/tpch-dbgen build.c)
* lineitem: 1..7 lines per order (dss.h), l_orderkey = parent key (sorted like dbgen),
            l_quantity = 1..50 uniform (stored as float in the reference schema, tpch_db_generator.cpp:20-27)
"""
import numpy as np

SEED = 0x48595249
ORDERS_PER_SF = 1_500_000
M64 = (1 << 64) - 1


def _splitmix64_np(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(M64)
    z = x
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _splitmix64_torch(x):
    import torch

    def lsr(v, k):  # logical shift right on int64
        return (v >> k) & ((1 << (64 - k)) - 1)

    x = x + torch.tensor(0x9E3779B97F4A7C15 - (1 << 64), dtype=torch.int64, device=x.device)
    z = x
    z = (z ^ lsr(z, 30)) * torch.tensor(0xBF58476D1CE4E5B9 - (1 << 64), dtype=torch.int64, device=x.device)
    z = (z ^ lsr(z, 27)) * torch.tensor(0x94D049BB133111EB - (1 << 64), dtype=torch.int64, device=x.device)
    return z ^ lsr(z, 31)


def n_orders(sf):
    return int(round(ORDERS_PER_SF * sf))


def orders_numpy(sf, first_order=0, seed=SEED):
    i = np.arange(first_order + 1, first_order + n_orders(sf) + 1, dtype=np.int64)
    okey = ((i >> 3) << 5) + (i & 7)
    lines = (_splitmix64_np(i.astype(np.uint64) ^ np.uint64(seed)) % np.uint64(7)).astype(np.int64) + 1
    return okey.astype(np.int32), lines


def lineitem_numpy(okey, lines, first_row=0, seed=SEED):
    lkey = np.repeat(okey, lines)
    r = np.arange(first_row, first_row + lkey.size, dtype=np.uint64)
    qty = (_splitmix64_np(r ^ np.uint64(seed ^ 0x5155)) % np.uint64(50)).astype(np.int32) + 1
    return lkey, qty


def orders_torch(sf, device, first_order=0, seed=SEED):
    import torch

    i = torch.arange(first_order + 1, first_order + n_orders(sf) + 1, dtype=torch.int64, device=device)
    okey = ((i >> 3) << 5) + (i & 7)
    h = _splitmix64_torch(i ^ seed)
    lines = torch.remainder(h, 7) + 1  # remainder of a possibly negative int64 -> use unsigned semantics below
    # unsigned modulo: (h mod 2^64) % 7 == ((h % 7) + (2^64 % 7) * [h < 0]) % 7
    lines = torch.remainder(torch.remainder(h, 7) + torch.where(h < 0, (1 << 64) % 7, 0), 7) + 1
    return okey.to(torch.int32), lines


def lineitem_torch(okey, lines, first_row=0, seed=SEED):
    import torch

    lkey = torch.repeat_interleave(okey, lines)
    r = torch.arange(first_row, first_row + lkey.numel(), dtype=torch.int64, device=okey.device)
    h = _splitmix64_torch(r ^ (seed ^ 0x5155))
    qty = torch.remainder(torch.remainder(h, 50) + torch.where(h < 0, (1 << 64) % 50, 0), 50) + 1
    return lkey, qty.to(torch.int32)


def _umod_torch(h, m):
    """(h mod 2^64) % m for int64 tensors holding uint64 bit patterns."""
    import torch

    return torch.remainder(torch.remainder(h, m) + torch.where(h < 0, (1 << 64) % m, 0), m)


# days since 1970-01-01 (dbgen's date range, dss.h STARTDATE / CURRENTDATE / ENDDATE - 151)
DATE_1992_01_01, DATE_1995_06_17, DATE_1998_08_02, DATE_1998_09_02 = 8035, 9298, 10440, 10471


def lineitem_q1_torch(sf, device, seed=SEED):
    """The lineitem columns TPC-H 1 reads, TPC-H-shaped (dbgen dss.h / build.c value ranges), as torch tensors:
    l_shipdate int32 days (o_orderdate + 1..121, o_orderdate uniform 1992-01-01..1998-08-02), l_returnflag code
    (A=0, N=1, R=2: R/A when the receipt date l_shipdate + 1..30 is <= 1995-06-17, else N), l_linestatus code (F=0,
    O=1: O when l_shipdate > 1995-06-17), l_quantity 1..50, l_extendedprice int64 cents = quantity x retail price
    (900.00..2100.00), l_discount 0..10 (hundredths). Works on any torch device (the CPU baseline uses the same
    generator on a smaller scale factor)."""
    import torch

    okey, lines = orders_torch(sf, device, seed=seed)
    i = torch.arange(1, okey.numel() + 1, dtype=torch.int64, device=device)
    odate = DATE_1992_01_01 + _umod_torch(_splitmix64_torch(i ^ (seed ^ 0x0D47)), DATE_1998_08_02 - DATE_1992_01_01 + 1)
    odate = torch.repeat_interleave(odate, lines)
    del okey, i
    _, qty = lineitem_torch(torch.zeros(lines.numel(), dtype=torch.int32, device=device), lines)
    del lines
    n = qty.numel()
    r = torch.arange(n, dtype=torch.int64, device=device)
    h = _splitmix64_torch(r ^ (seed ^ 0x5344))
    ship = odate + 1 + _umod_torch(h, 121)
    del odate
    receipt = ship + 1 + torch.remainder(h >> 8, 30)  # h >> 8 may be negative: arithmetic shift, remainder >= 0
    rflag = torch.where(receipt <= DATE_1995_06_17, torch.where((h >> 20) & 1 == 1, 2, 0), 1).to(torch.int32)
    del receipt
    lstatus = (ship > DATE_1995_06_17).to(torch.int32)
    h = _splitmix64_torch(r ^ (seed ^ 0x5052))
    retail = 90_000 + _umod_torch(h, 120_001)
    price = qty.to(torch.int64) * retail
    disc = torch.remainder(h >> 24, 11).to(torch.int32)
    return {"l_shipdate": ship.to(torch.int32), "l_returnflag": rflag, "l_linestatus": lstatus, "l_quantity": qty,
            "l_extendedprice": price, "l_discount": disc}


def dictionary_encode_small_domain(values_np_or_torch, chunk, domain):
    """Per-chunk dictionary encoding of values in [1, domain] (FixedSizeByteAligned u8 when domain < 255):
    returns (vids u8, present[chunks, domain] bool). vid = rank of the value among the chunk's distinct values,
    exactly what DictionaryEncoder produces (dictionary_encoder.hpp:57-130)."""
    try:
        import torch

        is_torch = isinstance(values_np_or_torch, torch.Tensor)
    except ImportError:  # pragma: no cover
        is_torch = False
    v = values_np_or_torch
    n = v.numel() if is_torch else v.size
    n_chunks = (n + chunk - 1) // chunk
    if is_torch:
        import torch

        cid = torch.arange(n, device=v.device, dtype=torch.int64) // chunk
        present = torch.zeros(n_chunks, domain + 1, dtype=torch.int32, device=v.device)
        present.index_put_((cid, v.to(torch.int64)), torch.ones_like(cid, dtype=torch.int32), accumulate=False)
        present[:, 0] = 0
        rank = torch.cumsum(present, dim=1) - 1
        vids = rank[cid, v.to(torch.int64)].to(torch.uint8)
        return vids, present[:, 1:].bool()
    cid = np.arange(n, dtype=np.int64) // chunk
    present = np.zeros((n_chunks, domain + 1), dtype=np.int32)
    present[cid, v] = 1
    present[:, 0] = 0
    rank = np.cumsum(present, axis=1) - 1
    return rank[cid, v].astype(np.uint8), present[:, 1:].astype(bool)


CUSTOMERS_PER_SF = 150_000
# c_mktsegment codes in dictionary order (dbgen c_mseg_set: AUTOMOBILE, BUILDING, FURNITURE, HOUSEHOLD, MACHINERY)
MKTSEGMENTS = ["AUTOMOBILE", "BUILDING", "FURNITURE", "HOUSEHOLD", "MACHINERY"]
DATE_1995_03_15 = 9204  # TPC-H 3's date (days since 1970-01-01)


def n_customers(sf):
    return int(round(CUSTOMERS_PER_SF * sf))


def q3_columns(sf, device, seed=SEED):
    """The columns TPC-H 3 reads (tpch_queries.cpp:101-106), TPC-H-shaped (dbgen build.c / dss.h ranges), as torch
    tensors on `device`:
      customer: c_custkey 1..150k*SF, c_mktsegment code 0..4 (uniform, MKTSEGMENTS order)
      orders:   o_orderkey (dbgen sparse keys), o_custkey uniform over the custkeys that are not multiples of 3 (dbgen
                leaves every third customer without orders), o_orderdate int32 days uniform 1992-01-01..1998-08-02,
                o_shippriority 0 (dbgen writes 0)
      lineitem: 1..7 lines per order, l_orderkey = parent key, l_shipdate = o_orderdate + 1..121,
                l_extendedprice = l_quantity x retail price (900.00..2100.00) and l_discount 0.00..0.10 as float32
                (the reference schema's float columns, tpch_db_generator.cpp:20-27)
    plus `l_order_index` (row index of the parent order, for the expected-result check)."""
    import torch

    n_cust = n_customers(sf)
    ci = torch.arange(1, n_cust + 1, dtype=torch.int64, device=device)
    seg = _umod_torch(_splitmix64_torch(ci ^ (seed ^ 0x4353)), 5).to(torch.int32)
    okey, lines = orders_torch(sf, device, seed=seed)
    n_ord = okey.numel()
    i = torch.arange(1, n_ord + 1, dtype=torch.int64, device=device)
    odate = DATE_1992_01_01 + _umod_torch(_splitmix64_torch(i ^ (seed ^ 0x0D47)), DATE_1998_08_02 - DATE_1992_01_01 + 1)
    k = _umod_torch(_splitmix64_torch(i ^ (seed ^ 0x4F43)), max(1, (n_cust // 3) * 2))
    ocust = (k // 2) * 3 + (k % 2) + 1
    del i, k
    lkey, qty = lineitem_torch(okey, lines, seed=seed)
    oidx = torch.repeat_interleave(torch.arange(n_ord, dtype=torch.int64, device=device), lines)
    n = lkey.numel()
    r = torch.arange(n, dtype=torch.int64, device=device)
    h = _splitmix64_torch(r ^ (seed ^ 0x5344))
    ship = odate[oidx] + 1 + _umod_torch(h, 121)
    h = _splitmix64_torch(r ^ (seed ^ 0x5052))
    del r
    retail = 90_000 + _umod_torch(h, 120_001)
    price = ((qty.to(torch.int64) * retail).to(torch.float64) / 100.0).to(torch.float32)
    disc = (torch.remainder(h >> 24, 11).to(torch.float64) / 100.0).to(torch.float32)
    del h, retail, qty
    return {"c_custkey": ci.to(torch.int32), "c_mktsegment": seg,
            "o_orderkey": okey, "o_custkey": ocust.to(torch.int32), "o_orderdate": odate.to(torch.int32),
            "o_shippriority": torch.zeros(n_ord, dtype=torch.int32, device=device),
            "l_orderkey": lkey, "l_shipdate": ship.to(torch.int32), "l_extendedprice": price, "l_discount": disc,
            "l_order_index": oidx}


def dictionary_encode_chunks(values, chunk, lo, domain):
    """Per-chunk dictionary encoding of integer values in [lo, lo + domain) (DictionaryEncoder: sorted distinct
    values, vid = rank; dictionary_encoder.hpp:57-130) on the values' torch device. Returns (vids int32, present
    [chunks, domain] bool): dictionary of chunk c = lo + nonzero(present[c]), vid width from its size."""
    import torch

    n = values.numel()
    n_chunks = (n + chunk - 1) // chunk
    cid = torch.arange(n, device=values.device, dtype=torch.int64) // chunk
    v = (values.to(torch.int64) - lo)
    present = torch.zeros(n_chunks, domain, dtype=torch.int32, device=values.device)
    present.index_put_((cid, v), torch.ones_like(cid, dtype=torch.int32), accumulate=False)
    rank = torch.cumsum(present, dim=1) - 1
    vids = rank[cid, v].to(torch.int32)
    return vids, present.bool()


def q1_columns(sf, device, seed=SEED):
    """The lineitem columns TPC-H 1 reads with the reference schema's types (tpch_db_generator.cpp:20-27):
    l_quantity, l_extendedprice, l_discount, l_tax as float32 (quantity 1..50, price = quantity x retail
    900.00..2100.00, discount 0.00..0.10, tax 0.00..0.08), l_returnflag / l_linestatus codes (A=0, N=1, R=2 / F=0,
    O=1) and l_shipdate int32 days, from the same generator as lineitem_q1_torch (same rows, same flags and dates)."""
    import torch

    c = lineitem_q1_torch(sf, device, seed=seed)
    n = c["l_shipdate"].numel()
    r = torch.arange(n, dtype=torch.int64, device=device)
    h = _splitmix64_torch(r ^ (seed ^ 0x5052))
    retail = 90_000 + _umod_torch(h, 120_001)
    price = ((c["l_quantity"].to(torch.int64) * retail).to(torch.float64) / 100.0).to(torch.float32)
    disc = (c["l_discount"].to(torch.float64) / 100.0).to(torch.float32)
    h = _splitmix64_torch(r ^ (seed ^ 0x5441))
    tax = (_umod_torch(h, 9).to(torch.float64) / 100.0).to(torch.float32)
    return {"l_returnflag": c["l_returnflag"], "l_linestatus": c["l_linestatus"],
            "l_quantity": c["l_quantity"].to(torch.float32), "l_extendedprice": price, "l_discount": disc,
            "l_tax": tax, "l_shipdate": c["l_shipdate"]}


def shard_torch(sf, chunk, rank, world, device, seed=SEED):
    """Rank `rank`'s chunk-aligned shard of the SF `sf` orders / lineitem tables (contiguous global chunk ranges, rank
    r holding chunks [r * C / N, (r + 1) * C / N) of each table), generated from global row indexes so that the
    union of the shards is exactly orders_torch / lineitem_torch of the whole table for any N. Returns a dict with
    o_orderkey, l_orderkey, l_quantity (this shard), o_row_base / l_row_base (global index of the shard's first
    row), o_chunk_lo / l_chunk_lo (its first global chunk id) and o_layout / l_layout (every global chunk's size)."""
    import torch

    n_ord = n_orders(sf)
    i = torch.arange(1, n_ord + 1, dtype=torch.int64, device=device)
    lines = _umod_torch(_splitmix64_torch(i ^ seed), 7) + 1
    del i
    ends = torch.cumsum(lines, 0)  # global lineitem row after each order's last line
    del lines
    n_li = int(ends[-1]) if n_ord else 0

    def chunks(n):
        return (n + chunk - 1) // chunk

    def layout(n):
        return [min(chunk, n - c * chunk) for c in range(chunks(n))]

    out = {"o_layout": layout(n_ord), "l_layout": layout(n_li)}
    for t, n in (("o", n_ord), ("l", n_li)):
        c_lo, c_hi = rank * chunks(n) // world, (rank + 1) * chunks(n) // world
        out[t + "_chunk_lo"], out[t + "_chunk_hi"] = c_lo, c_hi
        out[t + "_row_base"], out[t + "_row_end"] = c_lo * chunk, min(c_hi * chunk, n)
    o = torch.arange(out["o_row_base"] + 1, out["o_row_end"] + 1, dtype=torch.int64, device=device)
    out["o_orderkey"] = (((o >> 3) << 5) + (o & 7)).to(torch.int32)
    del o
    r = torch.arange(out["l_row_base"], out["l_row_end"], dtype=torch.int64, device=device)
    oi = torch.searchsorted(ends, r, right=True) + 1  # 1-based order index of each line
    del ends
    out["l_orderkey"] = (((oi >> 3) << 5) + (oi & 7)).to(torch.int32)
    del oi
    out["l_quantity"] = (_umod_torch(_splitmix64_torch(r ^ (seed ^ 0x5155)), 50) + 1).to(torch.int32)
    return out
