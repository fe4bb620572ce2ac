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
