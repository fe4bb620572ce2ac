"""The distributed JoinHash of SURVEY.md 8(e) as the bench runs it (bench_dist.py), restated on the CPU and run over
gloo with 2 and 3 ranks: every rank takes its chunk-aligned shard (synth.shard_torch), applies the fused TableScan
(l_quantity < 24) and forms 8-byte row-index records {o/l_orderkey, global row} grouped by first-digit bucket of the
GLOBAL radix partition (murmur2 seed 17, join_hash.cpp:640-680; bucket ownership as hy_join_exchange_bucket_bits and
dist.owned_buckets), routes them with dist.exchange_records (all_gather + all_to_all_single), and joins the partitions
it owns (probe rows in the order received, build matches in build order). The ranks' per-partition outputs, in rank
order, must equal the oracle's TableScan -> JoinHash on the whole tables (one chunk per non-empty partition).

This pins the distributed algorithm and the Python plumbing on the host; the same steps on the device
(hy_scan_join_exchange_partition / hy_join_exchange_join_rows) are checked against hy_scan_join_hash in
test_dist_join_gpu.py."""
import importlib
import os
import socket

import numpy as np
import pytest

from helpers import load_oracle, load_pkg

CHUNK = 4_000
SF = 40_000 / 1_500_000  # 40,000 orders


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _partitions(oracle, keys, bits):
    return np.array([oracle.murmur2_int32(int(k), 17) & ((1 << bits) - 1) for k in keys], dtype=np.int64)


def _worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hy = load_pkg()
        oracle = load_oracle()
        synth = importlib.import_module("hyrise-1_amd.synth")
        hd = importlib.import_module("hyrise-1_amd.dist")
        sh = synth.shard_torch(SF, CHUNK, rank, world, "cpu")
        bits = oracle.radix_bits(sum(sh["o_layout"]), 4)
        w0 = int(hy.capi.lib.hy_join_exchange_bucket_bits(bits, world))
        n_buckets = 1 << w0
        sides = {}
        for name, keys, keep, base in (
                ("build", sh["o_orderkey"].numpy(), None, sh["o_row_base"]),
                ("probe", sh["l_orderkey"].numpy(), sh["l_quantity"].numpy() < 24, sh["l_row_base"])):
            rows = np.arange(keys.size, dtype=np.int64) + base
            if keep is not None:  # the fused scan: only matches become records
                keys, rows = keys[keep], rows[keep]
            part = _partitions(oracle, keys, bits)
            bucket = part >> (bits - w0)
            order = np.argsort(bucket, kind="stable")
            words = (rows[order] << 32) | (keys[order].astype(np.int64) & 0xFFFFFFFF)  # {int32 key, u32 row}
            counts = np.bincount(bucket, minlength=n_buckets)
            recv, _ = hd.exchange_records(dist, torch.from_numpy(words), counts, rank, world, record_bytes=8)
            r = recv.numpy()
            sides[name] = ((r & 0xFFFFFFFF).astype(np.uint32).view(np.int32), r >> 32)
        lo, hi = hd.owned_buckets(n_buckets, rank, world)
        bkeys, brows = sides["build"]
        pkeys, prows = sides["probe"]
        bpart, ppart = _partitions(oracle, bkeys, bits), _partitions(oracle, pkeys, bits)
        out = []
        for p in range(lo << (bits - w0), hi << (bits - w0)):
            bsel = np.nonzero(bpart == p)[0]  # received order: sender (= global row) order
            table = {}
            for i in bsel:
                table.setdefault(int(bkeys[i]), []).append(int(brows[i]))
            pairs = [(b, int(prows[i])) for i in np.nonzero(ppart == p)[0] for b in table.get(int(pkeys[i]), [])]
            if pairs:
                out.append(np.array(pairs, dtype=np.int64))
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), *out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_scan_join_equals_single_node(tmp_path, world):
    import torch.multiprocessing as mp

    hy, oracle = load_pkg(), load_oracle()
    synth = importlib.import_module("hyrise-1_amd.synth")
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = []
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        got += [z[f"arr_{i}"] for i in range(len(z.files))]
    full = synth.shard_torch(SF, CHUNK, 0, 1, "cpu")
    orders = hy.Table.from_arrays([("o_orderkey", hy.DataType.Int, False)], [full["o_orderkey"].numpy()], [], CHUNK)
    lineitem = hy.Table.from_arrays([("l_orderkey", hy.DataType.Int, False), ("l_quantity", hy.DataType.Float, False)],
                                    [full["l_orderkey"].numpy(), full["l_quantity"].numpy().astype(np.float32)], [],
                                    CHUNK)
    hy.encode_all_chunks(lineitem, hy.EncodingType.Dictionary)
    scan = oracle.table_scan(lineitem, 1, hy.PredicateCondition.LessThan, 24, [])
    join, bits = oracle.join_hash(orders, scan, hy.JoinMode.Inner, (0, 0))
    assert bits >= 2 and join.chunk_count() == len(got)
    for k, pairs in enumerate(got):
        ch = join.get_chunk(k)
        b, p = ch.get_column(0).pos_list().astype(np.int64), ch.get_column(1).pos_list().astype(np.int64)
        assert np.array_equal(b[:, 0] * CHUNK + b[:, 1], pairs[:, 0]), f"output chunk {k}: build RowIDs"
        assert np.array_equal(p[:, 0] * CHUNK + p[:, 1], pairs[:, 1]), f"output chunk {k}: probe RowIDs"
