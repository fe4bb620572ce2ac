"""TPC-H 3 through the distributed JoinHash (bench_q3_dist.py, BASELINE.json configs[4]) with N ranks simulated on one
GPU: customer shard scans + broadcast join with each rank's orders shard, the orders ⋈ lineitem radix shuffle
(hy_scan_join_exchange_partition over a dereferenced reference side and over the lineitem shard with its scan fused,
columns carried with the records, hy_exchange_records_localize, hy_join_exchange_join_rows over the received
records) and the rank-local GROUP BY. The union of the ranks' groups must equal the oracle's TPC-H 3 chain (TableScan
x3, JoinHash x2, Projection, Aggregate; tpch_queries.cpp:101-106) on the whole tables: same groups, and every SUM
exactly (an order's revenue is a sum of <= 7 float products, exact in double, so the oracle's sequential double sum
and the device's exactly rounded sum agree bit for bit)."""
import ctypes
import importlib

import numpy as np
import pytest

from q3_oracle import oracle_q3

pytestmark = pytest.mark.gpu

SF, CHUNK = 0.02, 4_000


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_distributed_q3_equals_oracle(hy, world):
    import torch

    synth = importlib.import_module("hyrise-1_amd.synth")
    q3d = importlib.import_module("bench_q3_dist")
    capi, L = hy.capi, hy.capi.lib
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    capi.check(L.hy_set_device(0), "hy_set_device")
    stream = torch.cuda.current_stream().cuda_stream
    cols = synth.q3_columns(SF, dev)
    cols.pop("l_order_index")
    want, j1_rows, j2_rows = oracle_q3(hy, {k: v.cpu().numpy() for k, v in cols.items()}, CHUNK)
    ranks = q3d.run_in_process(hy, torch, synth, cols, CHUNK, world, dev, stream)
    torch.cuda.synchronize()
    assert sum(r.stats["join1_pairs"] for r in ranks) == j1_rows
    assert sum(r.stats["join2_pairs"] for r in ranks) == j2_rows
    got = {}
    for r in ranks:
        lay = r.stats["layout"]
        w = lay.agg_word[0]
        for row in r.group_records():
            key = tuple(int(np.int32(np.uint32(row[j]))) for j in range(3))
            limbs = (ctypes.c_uint64 * lay.agg_limbs[0])(*[int(x) for x in row[w + 2:w + 2 + lay.agg_limbs[0]]])
            s = ctypes.c_double(0)
            capi.check(L.hy_agg_float_sum(limbs, lay.agg_limbs[0], lay.agg_emin[0], int(row[w + 1]), ctypes.byref(s)))
            assert key not in got, f"group {key} on two ranks"
            got[key] = s.value
    assert set(got) == set(want)
    bad = [k for k in want if got[k] != want[k]]
    assert not bad, f"{len(bad)} sums differ, e.g. {bad[:3]}: {[(got[k], want[k]) for k in bad[:3]]}"
