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
        out, per_part = [], []
        for p in range(lo << (bits - w0), hi << (bits - w0)):
            bsel = np.nonzero(bpart == p)[0]  # received order: sender (= global row) order
            table = {}
            for i in bsel:
                table.setdefault(int(bkeys[i]), []).append(int(brows[i]))
            pairs = [(b, int(prows[i])) for i in np.nonzero(ppart == p)[0] for b in table.get(int(pkeys[i]), [])]
            per_part.append(np.array(pairs, dtype=np.int64).reshape(-1, 2))
            if pairs:
                out.append(per_part[-1])
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), *out)
        # the bench's per-rank output check (dist.headline_expected / check_partition_output) on this layout, laid out
        # as the device writes it (RowID pairs, partitions placed in an arbitrary order: here reversed), then corrupted
        expected = hd.headline_expected(dist, sh["l_orderkey"], sh["l_quantity"] < 24, sh["l_row_base"], bits)

        def device_layout(parts):
            counts = np.array([len(x) for x in parts], dtype=np.int64)
            begin = np.zeros(len(parts), dtype=np.int64)
            at = 0
            for i in reversed(range(len(parts))):
                begin[i] = at
                at += counts[i]
            rid = np.zeros((2, max(1, at), 2), dtype=np.int32)
            for i, x in enumerate(parts):
                for col in (0, 1):
                    rid[col, begin[i]:begin[i] + counts[i], 0] = x[:, col] // CHUNK
                    rid[col, begin[i]:begin[i] + counts[i], 1] = x[:, col] % CHUNK
            return (torch.from_numpy(rid[0]), torch.from_numpy(rid[1]), torch.from_numpy(begin),
                    torch.from_numpy(counts.astype(np.int32)))

        first_part = lo << (bits - w0)
        checks = {"ok": hd.check_partition_output(expected, *device_layout(per_part), first_part, CHUNK)}
        big = [i for i, x in enumerate(per_part) if len(x) >= 2]
        if len(big) >= 2:
            moved = [x.copy() for x in per_part]
            moved[big[0]][0, 0], moved[big[1]][0, 0] = per_part[big[1]][0, 0], per_part[big[0]][0, 0]
            checks["build_swapped"] = hd.check_partition_output(expected, *device_layout(moved), first_part, CHUNK)
            flipped = [x.copy() for x in per_part]
            flipped[big[0]] = flipped[big[0]][::-1].copy()
            checks["probe_reversed"] = hd.check_partition_output(expected, *device_layout(flipped), first_part, CHUNK)
        import json

        with open(os.path.join(out_dir, f"check{rank}.json"), "w") as f:
            json.dump(checks, f)
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
    # the distributed bench's per-rank output check: passes on the right layout, catches moved and reordered pairs
    import json

    for r in range(world):
        checks = json.load(open(tmp_path / f"check{r}.json"))
        assert all(checks["ok"].values()), checks["ok"]
        if "build_swapped" in checks:
            assert not checks["build_swapped"]["build_row_sums"]
            assert not checks["probe_reversed"]["probe_ascending_within_partitions"]
            assert checks["probe_reversed"]["probe_row_sums"]  # (the same rows, in the wrong order)
