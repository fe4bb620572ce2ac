"""Streams destroyed while the library still held events recorded on them (round 6, DESIGN.md "Stream lifetime").

Every call that stages host descriptors fences its copies with an event on the caller's stream (the per-thread pinned
ring, capi_common.hpp), and per-kernel timing keeps an event pair per launch until it is collected. hy_stream_destroy
now drops the ring's fences and resolves the pending timings of the stream before the handle dies. Before, a later
ring wrap (or a stats collection) waited on an event whose recording stream was gone; the runtime then read the freed
stream object - "operation not permitted on an event last recorded in a capturing stream" in the full suite - and
could write into it (heap corruption seen later as glibc tcache errors or a device memory fault).

The test stages on short-lived streams, destroys them, and then forces the ring to wrap and the timings to be
collected on this thread: both must succeed, and the scans' PosLists stay exact."""
import ctypes

import numpy as np
import pytest

import device_tables as dt
from helpers import wrap

pytestmark = pytest.mark.gpu


def scan_on(capi, L, col, stream):
    chunks = col.scan_chunks("LessThan", 17)
    for c in range(col.n_chunks):
        chunks[c].out_begin = c * col.chunk  # (chunk c's RowIDs at its own row range)
    sizes = (ctypes.c_uint32 * col.n_chunks)(*[col.chunk_size(c) for c in range(col.n_chunks)])
    ws_bytes = ctypes.c_size_t()
    capi.check(L.hy_table_scan_workspace_size(sizes, col.n_chunks, ctypes.byref(ws_bytes)), "workspace size")
    ws = capi.DeviceArray(np.zeros(max(ws_bytes.value, 16), np.uint8))
    out = capi.DeviceArray(np.zeros(2 * col.values.size, np.uint32))
    counts = capi.DeviceArray(np.zeros(col.n_chunks, np.uint32))
    ids = (ctypes.c_uint32 * col.n_chunks)(*range(col.n_chunks))
    capi.check(L.hy_table_scan_row_ids(chunks, col.n_chunks, 1, None, ids, out.ptr, counts.ptr, ws.ptr, ws_bytes.value,
                                       stream), "hy_table_scan_row_ids")
    capi.check(L.hy_stream_synchronize(stream), "sync")
    n = counts.fetch().astype(np.int64)
    rows = out.fetch().reshape(-1, 2)
    got = np.concatenate([rows[c * col.chunk:c * col.chunk + n[c], 1] + c * col.chunk for c in range(col.n_chunks)])
    return got


def test_ring_wrap_and_timings_after_stream_destroy(hy):
    capi, L = hy.capi, hy.capi.lib
    rng = np.random.default_rng(0x5354)
    vals = rng.integers(0, 50, 200_000).astype(np.int32)
    col = dt.DeviceColumn(capi, vals, None, 20_000, "Dictionary")
    want = np.flatnonzero(vals < 17)
    capi.check(L.hy_kernel_stats_enable(1), "stats on")
    try:
        for _ in range(3):
            streams = []
            for _ in range(6):  # fences and pending timings on streams that are then destroyed
                s = ctypes.c_void_p()
                capi.check(L.hy_stream_create(ctypes.byref(s)), "hy_stream_create")
                streams.append(s)
                assert np.array_equal(scan_on(capi, L, col, s), want)
            for s in streams:
                capi.check(L.hy_stream_destroy(s), "hy_stream_destroy")
            # a 17 MiB constant through the ring on this thread: the ring wraps and waits on its remaining fences
            strings = hy.Table([("s", hy.DataType.String, False)], hy.TableType.Data, 64)
            for i in range(50):
                strings.append([f"s{i}"])
            scan = hy.TableScan(wrap(hy, strings), 0, hy.PredicateCondition.Equals, "x" * (17 << 20))
            scan.execute()
            assert scan.get_output().row_count() == 0
            n = ctypes.c_uint32()
            capi.check(L.hy_kernel_stats_collect(ctypes.byref(n)), "hy_kernel_stats_collect")
            assert n.value >= 1
    finally:
        L.hy_kernel_stats_enable(0)
        L.hy_kernel_stats_reset()
