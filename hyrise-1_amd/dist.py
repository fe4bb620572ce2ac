"""Distributed JoinHash across the GPUs of one node: one process per GPU, chunks sharded by
contiguous chunk ranges, one exchange step.

    step 1  every rank, each side: hy_scan_join_exchange_partition -> 8-byte exchange records {int32 key, global row
            index} (data-table sides, optionally with the side's TableScan fused in) or hy_join_exchange_partition ->
            16-byte records {key, global RowID} (reference sides), grouped by first-digit bucket of the GLOBAL radix
            partition, plus per-bucket counts
    counts  all_gather of the per-bucket counts (B <= 256 integers per rank and side)
    records all_to_all_single over RCCL/xGMI: rank r receives, sender by sender, every record of the buckets it owns
    step 2  every rank: hy_join_exchange_join_rows / hy_join_exchange_join -> remaining radix passes + LDS
            build/probe of its partitions

The ranks' outputs, concatenated in rank order, are the single-node JoinHash output: one output chunk per radix
partition in ascending order, probe rows in (chunk, offset) order, build matches in build order (join_hash.cpp).

The collective plumbing (split sizes, count matrices) is plain Python over torch.distributed so it runs on RCCL for
the GPU path and on gloo for the CPU tests; the records themselves are opaque int64 pairs.
"""
import ctypes

import numpy as np

RECORD_BYTES = 16


def bucket_bits(capi, radix_bits, world):
    return int(capi.lib.hy_join_exchange_bucket_bits(radix_bits, world))


def owned_buckets(n_buckets, rank, world):
    """Rank r owns first-digit buckets [r * B // N, (r + 1) * B // N) (include/hyrise_amd.h)."""
    return rank * n_buckets // world, (rank + 1) * n_buckets // world


def murmur2_int32_torch(keys, seed=17):
    """MurmurHash2 of 4-byte keys on torch tensors (murmur_hash.cpp:21-75 for len = 4; the numpy twin is pinned by
    tests/test_murmur_golden.py). 32-bit arithmetic in int64 lanes."""
    import torch

    M, m = 0xFFFFFFFF, 0x5BD1E995
    k = keys.to(torch.int64) & M
    k = (k * m) & M
    k = k ^ (k >> 24)
    k = (k * m) & M
    h = torch.full_like(k, ((seed ^ 4) * m) & M)
    h = h ^ k
    h = h ^ (h >> 13)
    h = (h * m) & M
    return h ^ (h >> 15)


def partition_sums(partitions, probe_rows, build_rows, n_parts):
    """Per partition: (pairs, sum of probe rows, sum of build rows) as int64 tensors of n_parts entries."""
    import torch

    dev = partitions.device
    out = [torch.zeros(n_parts, dtype=torch.int64, device=dev) for _ in range(3)]
    out[0].index_add_(0, partitions, torch.ones_like(partitions))
    out[1].index_add_(0, partitions, probe_rows)
    out[2].index_add_(0, partitions, build_rows)
    return out


def headline_expected(dist, lkey, match, l_row_base, radix_bits, seed=17):
    """The single-GPU layout of the headline join over the whole (sharded) database: per global partition the pairs,
    the sum of their probe rows and of their build rows, from this rank's shard (its scan matches: l_orderkey of
    every matching lineitem row meets exactly one order, whose row follows from the dbgen sparse key
    ((i >> 3) << 5) + (i & 7), i = row + 1) summed over the ranks. Only the join's definition enters: murmur2 seed 17
    partitions (join_hash.cpp:253) and the reference's output order is checked separately (probe rows ascending)."""
    import torch

    idx = torch.nonzero(match, as_tuple=True)[0]
    keys = lkey[idx].to(torch.int64)
    parts = murmur2_int32_torch(keys, seed) & ((1 << radix_bits) - 1)
    orow = (((keys >> 5) << 3) + (keys & 7)) - 1
    sums = partition_sums(parts, idx.to(torch.int64) + l_row_base, orow, 1 << radix_bits)
    for t in sums:
        dist.all_reduce(t)
    return sums


def check_partition_output(expected, out_b, out_p, part_begin, part_count, first_part, chunk):
    """This rank's join output (its owned partitions [first_part, first_part + n)) against headline_expected: pairs,
    probe / build row sums per partition, and probe rows strictly ascending inside every partition (the reference's
    probe order). RowIDs name global chunks of `chunk` rows. Returns a dict of the checks (all True = ok)."""
    import torch

    n = part_count.numel()
    counts = part_count.to(torch.int64)
    total = int(counts.sum())
    dev = counts.device
    pid = torch.repeat_interleave(torch.arange(n, device=dev), counts)
    excl = torch.cumsum(counts, 0) - counts
    pos = torch.repeat_interleave(part_begin.to(torch.int64), counts) + (
        torch.arange(total, device=dev) - torch.repeat_interleave(excl, counts))
    p = out_p.view(torch.int32).view(-1, 2)[pos].to(torch.int64)
    b = out_b.view(torch.int32).view(-1, 2)[pos].to(torch.int64)
    prow, brow = p[:, 0] * chunk + p[:, 1], b[:, 0] * chunk + b[:, 1]
    got = partition_sums(pid, prow, brow, n)
    want = [t[first_part:first_part + n] for t in expected]
    same_part = pid[1:] == pid[:-1]
    return {
        "pair_counts": bool(torch.equal(got[0], want[0])),
        "probe_row_sums": bool(torch.equal(got[1], want[1])),
        "build_row_sums": bool(torch.equal(got[2], want[2])),
        "probe_ascending_within_partitions": bool(((prow[1:] > prow[:-1]) | ~same_part).all()),
    }


def exchange_plan(all_counts, rank, world):
    """all_counts[s][b] = rows of bucket b on sender s (every rank's counts, from all_gather).
    Returns (send_rows[d], recv_rows[s], recv_matrix[s][j]) for this rank: rows sent to each destination rank, rows
    received from each sender, and per sender the counts of this rank's local buckets j."""
    all_counts = np.asarray(all_counts, dtype=np.int64)
    n_buckets = all_counts.shape[1]
    send = []
    for d in range(world):
        lo, hi = owned_buckets(n_buckets, d, world)
        send.append(int(all_counts[rank, lo:hi].sum()))
    lo, hi = owned_buckets(n_buckets, rank, world)
    recv_matrix = all_counts[:, lo:hi].copy()
    recv = [int(x) for x in recv_matrix.sum(axis=1)]
    return send, recv, recv_matrix


def exchange_records(dist, records, bucket_counts, rank, world, device=None, record_bytes=RECORD_BYTES):
    """Routes this rank's exchange records (int64 tensor of record_bytes / 8 words per record, grouped by bucket) to
    their owners. Returns (received records, recv_matrix[s][j])."""
    import torch

    counts = torch.as_tensor(np.asarray(bucket_counts, dtype=np.int64), device=device)
    gathered = [torch.empty_like(counts) for _ in range(world)]
    dist.all_gather(gathered, counts)
    all_counts = np.stack([g.cpu().numpy() for g in gathered])
    send, recv, recv_matrix = exchange_plan(all_counts, rank, world)
    words = record_bytes // 8
    out = torch.empty(sum(recv) * words, dtype=torch.int64, device=records.device)
    dist.all_to_all_single(out, records[: sum(send) * words], [r * words for r in recv], [s * words for s in send])
    return out, recv_matrix


def exchange_columns(dist, columns, bucket_counts, rank, world, per_row=None):
    """Routes this rank's exchange records AND the columns carried with them (include/hyrise_amd.h, "Columns carried
    with the exchange"): every tensor in `columns` has one row per record, in record order (rows grouped by bucket as
    step 1 wrote them; per_row[j] elements per row, default 1, e.g. 2 int64 words of 16-byte records). One all_gather
    of the counts, one all_to_all_single per column with the same row splits. Returns (received columns,
    recv_matrix)."""
    import torch

    dev = columns[0].device
    counts = torch.as_tensor(np.asarray(bucket_counts, dtype=np.int64), device=dev)
    gathered = [torch.empty_like(counts) for _ in range(world)]
    dist.all_gather(gathered, counts)
    send, recv, recv_matrix = exchange_plan(np.stack([g.cpu().numpy() for g in gathered]), rank, world)
    n_send = sum(send)
    out = []
    for j, t in enumerate(columns):
        per = per_row[j] if per_row else 1
        r = torch.empty(sum(recv) * per, dtype=t.dtype, device=dev)
        dist.all_to_all_single(r, t[: n_send * per].contiguous(), [x * per for x in recv], [x * per for x in send])
        out.append(r)
    return out, recv_matrix


def exchange_columns_in_process(all_columns, all_counts, per_row=None):
    """The same routing for N ranks simulated in one process (tests on one GPU): all_columns[r] = rank r's columns,
    all_counts[r] = its bucket counts. Returns per rank (received columns, recv_matrix)."""
    import torch

    world = len(all_columns)
    all_counts = np.stack([np.asarray(c, dtype=np.int64) for c in all_counts])
    n_buckets = all_counts.shape[1]
    out = []
    for d in range(world):
        lo, hi = owned_buckets(n_buckets, d, world)
        _, _, recv_matrix = exchange_plan(all_counts, d, world)
        cols = []
        for j in range(len(all_columns[0])):
            parts = []
            for s in range(world):
                t = all_columns[s][j]
                per = per_row[j] if per_row else 1
                b0, b1 = int(all_counts[s, :lo].sum()), int(all_counts[s, :hi].sum())
                parts.append(t[b0 * per:b1 * per])
            cols.append(torch.cat(parts) if parts else all_columns[0][j][:0])
        out.append((cols, recv_matrix))
    return out


class RcclExchange:
    """The exchange step through the C-ABI's own RCCL communicator (hy_comm_init, hy_join_exchange_counts,
    hy_join_exchange_records): what a C++ Hyrise process linking libhyrise_amd.so calls. torch.distributed only hands
    rank 0's 128-byte communicator id to the other ranks. Opt-in from Python (bench.py --transport capi): a torch
    process also loads torch's bundled RCCL and HIP runtime under the same sonames, and which one libhyrise_amd.so's
    RCCL calls resolve to depends on load order; the native check (tests/native/exchange_check.cpp) runs without
    torch."""

    def __init__(self, capi, dist, rank, world, device):
        import torch

        self.capi, self.lib, self.rank, self.world = capi, capi.lib, rank, world
        cid = (ctypes.c_char * capi.HY_COMM_ID_BYTES)()
        if rank == 0:
            capi.check(self.lib.hy_comm_get_unique_id(cid), "hy_comm_get_unique_id")
        t = torch.tensor(list(bytes(cid)), dtype=torch.uint8, device=device)
        dist.broadcast(t, 0)
        cid = (ctypes.c_char * capi.HY_COMM_ID_BYTES)(*t.cpu().tolist())
        self.comm = ctypes.c_void_p()
        capi.check(self.lib.hy_comm_init(ctypes.byref(self.comm), world, cid, rank), "hy_comm_init")

    def close(self):
        if self.comm:
            self.capi.check(self.lib.hy_comm_destroy(self.comm), "hy_comm_destroy")
            self.comm = ctypes.c_void_p()

    def exchange(self, records, bucket_counts, record_bytes, stream, out=None):
        """Same contract as exchange_records: returns (received records as int64 words, recv_matrix[s][j])."""
        import torch

        capi, lib = self.capi, self.lib
        nb = len(bucket_counts)
        counts = (ctypes.c_uint64 * nb)(*[int(x) for x in bucket_counts])
        all_counts = (ctypes.c_uint64 * (nb * self.world))()
        capi.check(lib.hy_join_exchange_counts(self.comm, counts, nb, all_counts, stream), "hy_join_exchange_counts")
        _, recv, recv_matrix = exchange_plan(np.frombuffer(all_counts, dtype=np.uint64).reshape(self.world, nb),
                                             self.rank, self.world)
        words = record_bytes // 8
        if out is None or out.numel() < max(1, sum(recv)) * words:
            out = torch.empty(max(1, sum(recv)) * words, dtype=torch.int64, device=records.device)
        lo, hi = owned_buckets(nb, self.rank, self.world)
        rc = (ctypes.c_uint64 * max(1, self.world * (hi - lo)))()
        rows = ctypes.c_uint64()
        capi.check(lib.hy_join_exchange_records(self.comm, records.data_ptr(), record_bytes, all_counts, nb,
                                                out.data_ptr(), out.numel() // words, rc, ctypes.byref(rows), stream),
                   "hy_join_exchange_records")
        got = np.frombuffer(rc, dtype=np.uint64)[: self.world * (hi - lo)].reshape(self.world, hi - lo)
        assert np.array_equal(got.astype(np.int64), recv_matrix.astype(np.int64))
        return out[: int(rows.value) * words], recv_matrix


class ExchangeJoin:
    """The two C-ABI steps of the distributed JoinHash on device buffers owned by torch tensors.

    rows=True: row-index records (hy_scan_join_exchange_partition / hy_join_exchange_join_rows) for data-table
    sides, with build_layout / probe_layout the global tables' chunk sizes (global chunk-id order)."""

    def __init__(self, capi, radix_bits, world, hashed_type, mode=0, seed=17, rows=False, build_layout=None,
                 probe_layout=None):
        self.capi = capi
        self.lib = capi.lib
        self.world = world
        self.params = capi.JoinParams(mode, hashed_type, radix_bits, seed)
        self.bits = radix_bits
        self.first_bits = bucket_bits(capi, radix_bits, world)
        self.n_buckets = 1 << self.first_bits
        self.rows = rows
        self.record_bytes = int(capi.lib.hy_join_exchange_row_record_bytes(hashed_type)) if rows else RECORD_BYTES
        self.layouts = [np.ascontiguousarray(np.asarray(x if x is not None else [], dtype=np.uint32))
                        for x in (build_layout, probe_layout)]
        self._ws = {}

    def _workspace(self, key, nbytes, device):
        import torch

        t = self._ws.get(key)
        if t is None or t.numel() < nbytes:
            t = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
            self._ws[key] = t
        return t

    def partition(self, side, n_rows, keep_nulls, stream, device, key="side", filt=None, row_base=0):
        """Step 1 for one side: returns (records int64 tensor, bucket counts np.uint64[B]). Row-index mode: the
        records of the rows taking part (all rows, or the fused scan's matches with filt), payload row_base + row.
        keep_nulls None: from the join mode (NULL keys take part in LEFT / RIGHT joins, join_hash.cpp:468-527)."""
        import torch

        lib, capi = self.lib, self.capi
        if keep_nulls is None:
            keep_nulls = self.params.mode in (capi.HY_JOIN_LEFT, capi.HY_JOIN_RIGHT)
        wsb = ctypes.c_size_t(0)
        fp = ctypes.byref(filt) if filt is not None else None
        if self.rows:
            capi.check(lib.hy_scan_join_exchange_partition_workspace_size(ctypes.byref(side), fp,
                                                                           ctypes.byref(self.params), self.world,
                                                                           ctypes.byref(wsb)), "exchange ws")
        else:
            capi.check(lib.hy_join_exchange_partition_workspace_size(ctypes.byref(side), ctypes.byref(self.params),
                                                                      self.world, ctypes.byref(wsb)), "exchange ws")
        ws = self._workspace(key, wsb.value, device)
        rb = self.record_bytes
        recs = self._workspace(key + ".recs", max(1, n_rows) * rb + 64, device)
        counts = (ctypes.c_uint64 * self.n_buckets)()
        if self.rows:
            capi.check(lib.hy_scan_join_exchange_partition(ctypes.byref(side), fp, ctypes.byref(self.params),
                                                           int(keep_nulls), self.world, row_base, recs.data_ptr(),
                                                           counts, ws.data_ptr(), ws.numel(), stream),
                       "hy_scan_join_exchange_partition")
        else:
            capi.check(lib.hy_join_exchange_partition(ctypes.byref(side), ctypes.byref(self.params), int(keep_nulls),
                                                      self.world, recs.data_ptr(), counts, ws.data_ptr(), ws.numel(),
                                                      stream), "hy_join_exchange_partition")
        counts = np.frombuffer(counts, dtype=np.uint64).copy()
        n_out = int(counts.sum())
        return recs[: n_out * rb].view(torch.int64), counts

    def join(self, build_recs, build_matrix, probe_recs, probe_matrix, rank, stream, device, capacity=None):
        """Step 2: returns (out_build, out_probe, part_begin, part_count, total_pairs) - RowID tensors (int32 pairs)
        and per local partition the output range."""
        import torch

        lib, capi = self.lib, self.capi
        first, last = owned_buckets(self.n_buckets, rank, self.world)
        nb = last - first
        bc = np.ascontiguousarray(build_matrix, dtype=np.uint64)
        pc = np.ascontiguousarray(probe_matrix, dtype=np.uint64)
        bcp = bc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        pcp = pc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        wsb = ctypes.c_size_t(0)
        bl, pl = self.layouts
        if self.rows:
            capi.check(lib.hy_join_exchange_join_rows_workspace_size(bcp, pcp, self.world, nb, ctypes.byref(self.params),
                                                                      bl.ctypes.data, bl.size, pl.ctypes.data, pl.size,
                                                                      ctypes.byref(wsb)), "exchange join ws")
        else:
            capi.check(lib.hy_join_exchange_join_workspace_size(bcp, pcp, self.world, nb, ctypes.byref(self.params),
                                                                 ctypes.byref(wsb)), "exchange join ws")
        ws = self._workspace("join", wsb.value, device)
        n_parts = nb << (self.bits - self.first_bits)
        if capacity is None:
            capacity = int(pc.sum()) + int(bc.sum()) + 16
        out_b = self._workspace("out_b", capacity * 8, device)
        out_p = self._workspace("out_p", capacity * 8, device)
        part_begin = torch.empty(max(1, n_parts), dtype=torch.int64, device=device)
        part_count = torch.empty(max(1, n_parts), dtype=torch.int32, device=device)
        res = capi.JoinResult()
        if self.rows:
            st = lib.hy_join_exchange_join_rows(build_recs.data_ptr(), bcp, probe_recs.data_ptr(), pcp, self.world,
                                                first, nb, ctypes.byref(self.params), bl.ctypes.data, bl.size,
                                                pl.ctypes.data, pl.size, out_b.data_ptr(), out_p.data_ptr(), capacity,
                                                part_begin.data_ptr(), part_count.data_ptr(), ctypes.byref(res),
                                                ws.data_ptr(), ws.numel(), stream)
        else:
            st = lib.hy_join_exchange_join(build_recs.data_ptr(), bcp, probe_recs.data_ptr(), pcp, self.world, first,
                                           nb, ctypes.byref(self.params), out_b.data_ptr(), out_p.data_ptr(),
                                           capacity, part_begin.data_ptr(), part_count.data_ptr(), ctypes.byref(res),
                                           ws.data_ptr(), ws.numel(), stream)
        if st == capi.HY_ERR_CAPACITY:  # more pairs than the first guess (repeated build keys): exact size known
            return self.join(build_recs, build_matrix, probe_recs, probe_matrix, rank, stream, device,
                             capacity=res.capacity_required + 16)
        capi.check(st, "hy_join_exchange_join")
        return out_b, out_p, part_begin[:n_parts], part_count[:n_parts], res.total_pairs
