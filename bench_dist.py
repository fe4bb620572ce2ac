"""Headline workload on N GPUs (`torchrun --nproc-per-node N bench.py --gpus N`): the distributed JoinHash of
SURVEY.md 8(e) with the TableScan fused into its exchange partition.

Scaling (--scaling, default strong): strong = the SF100 database split over the N ranks (BASELINE.json's metric:
SF100 on 1/2/4/8 GPUs); weak = an SF x N database, SF per rank. Rank r holds contiguous global chunk ranges of orders
and lineitem (hyrise-1_amd/synth.shard_torch: the union of the shards is exactly the single-GPU database). One step:

    build   hy_scan_join_exchange_partition(orders shard)                    8-byte records {o_orderkey, global row}
    probe   hy_scan_join_exchange_partition(lineitem shard, l_quantity < 24)  the scan runs in the same pass and writes
                                                                             the shard's scan output (chunk offsets)
    exchange  per side: the first-digit bucket counts to every rank, then one all-to-all of the records - by default
              through the library's own RCCL communicator (hy_join_exchange_counts / hy_join_exchange_records, the
              C++ integration's path; --transport torch: torch's all_to_all_single), over xGMI with --dist-backend
              nccl; host-staged gloo rehearsal otherwise
    join    hy_join_exchange_join_rows: remaining radix passes + LDS build/probe of this rank's partitions; output
            RowIDs name global chunks (the ranks' outputs in rank order = the single-GPU output)

The radix bits come from the GLOBAL build size (join_hash.cpp:640-668), so partitions are the single-GPU ones. Timing:
barrier + synchronize around K steps, the max over ranks; value = all ranks' base rows (orders + lineitem) / time.
Check: every rank's output partitions against the single-GPU layout computed from the shards (pairs, probe and build
row sums per partition, probe rows ascending inside each; dist.headline_expected / check_partition_output).
"""
import ctypes
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def main_distributed(args):
    import numpy as np
    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    hy = importlib.import_module("hyrise-1_amd")
    synth = importlib.import_module("hyrise-1_amd.synth")
    hdist = importlib.import_module("hyrise-1_amd.dist")
    capi = hy.capi
    L = capi.lib
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    nccl = args.dist_backend == "nccl"
    if nccl:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group("gloo")
    dev = torch.device("cuda", torch.cuda.current_device())
    xdev = dev if nccl else torch.device("cpu")
    capi.check(L.hy_set_device(dev.index), "hy_set_device")
    stream = torch.cuda.current_stream().cuda_stream
    chunk = args.chunk
    scaling = args.scaling or "strong"
    global_sf = args.sf if scaling == "strong" else args.sf * world

    # ---------------- this rank's shard, resident in HBM ----------------
    sh = synth.shard_torch(global_sf, chunk, rank, world, dev)
    n_ord_g, n_li_g = sum(sh["o_layout"]), sum(sh["l_layout"])
    okey, lkey, qty = sh["o_orderkey"], sh["l_orderkey"], sh["l_quantity"]
    n_ord, n_li = okey.numel(), lkey.numel()
    radix_bits = L.hy_join_radix_bits(n_ord_g, 4)  # global build size (join_hash.cpp:640-668)
    # the single-GPU layout's per-partition pairs / row sums over the whole database (the output check below)
    expected = hdist.headline_expected(dist, lkey, qty < 24, sh["l_row_base"], radix_bits)
    vids, present = synth.dictionary_encode_small_domain(qty, chunk, 50)
    del qty
    present_h = present.cpu().numpy()

    def padded(t, mult=64):
        extra = (-t.numel()) % mult
        return torch.cat([t, torch.zeros(extra + mult, dtype=t.dtype, device=t.device)])

    vids, lkey, okey = padded(vids.contiguous()), padded(lkey.contiguous()), padded(okey.contiguous())
    torch.cuda.synchronize()
    n_lc, n_oc = (n_li + chunk - 1) // chunk, (n_ord + chunk - 1) // chunk

    def data_side(keys, n_rows, n_chunks, chunk_lo):
        arr = (capi.JoinChunk * max(1, n_chunks))()
        for c in range(n_chunks):
            size = min(chunk, n_rows - c * chunk)
            j = arr[c]
            j.column.data = keys.data_ptr() + 4 * c * chunk
            j.column.size = size
            j.column.kind = capi.HY_COL_VALUE
            j.size = size
            j.chunk_id = chunk_lo + c
            j.single_chunk = capi.HY_MIXED_CHUNKS
        side = capi.JoinSide(arr, n_chunks, capi.HY_TYPE_INT32, None, 0, 0, 0)
        side._keep = arr
        return side

    build_side = data_side(okey, n_ord, n_oc, sh["o_chunk_lo"])
    probe_side = data_side(lkey, n_li, n_lc, sh["l_chunk_lo"])
    # l_quantity < 24 on the dictionary chunks (search vid = distinct values < 24 in the chunk)
    scan_chunks = (capi.ScanChunk * max(1, n_lc))()
    for c in range(n_lc):
        size = min(chunk, n_li - c * chunk)
        dsize, svid = int(present_h[c].sum()), int(present_h[c, :23].sum())
        sc = scan_chunks[c]
        sc.column.data = vids.data_ptr() + c * chunk
        sc.column.size = size
        sc.column.dictionary_size = dsize
        sc.column.kind = capi.HY_COL_DICT
        sc.column.vid_width = 1
        sc.search_vid = svid
        sc.op = capi.HY_OP_ALL if svid >= dsize else (capi.HY_OP_NONE if svid == 0 else capi.HY_OP_LT)
    scan_off = torch.empty(n_li + 64, dtype=torch.int32, device=dev)
    scan_begin = torch.zeros(n_lc + 1, dtype=torch.int64, device=dev)
    pfilter = capi.JoinFilter(scan_chunks, capi.HY_TYPE_FLOAT, None, scan_off.data_ptr(), scan_begin.data_ptr())

    xj = hdist.ExchangeJoin(capi, radix_bits, world, capi.HY_TYPE_INT32, capi.HY_JOIN_INNER, 17, rows=True,
                            build_layout=sh["o_layout"], probe_layout=sh["l_layout"])
    rb = xj.record_bytes
    state = {}
    # RCCL transport: the library's own communicator (default) or torch.distributed's all_to_all (--transport torch)
    rx, transport_note, transport = None, "torch all_to_all", "torch"
    transport_error = None
    if args.dist_backend == "nccl" and args.transport == "capi":
        try:
            rx = hdist.RcclExchange(capi, dist, rank, world, dev)
            transport_note = "hy_join_exchange_counts/records (C-ABI RCCL communicator)"
            transport = "capi-rccl"
        except Exception as e:  # noqa: BLE001 - the line says so: "transport": "torch-fallback" + the error
            transport_note = f"torch all_to_all (C-ABI communicator failed: {e})"
            transport, transport_error = "torch-fallback", str(e)
            print(f"bench_dist: rank {rank}: the C-ABI RCCL communicator failed ({e}); this run measures torch's "
                  f"all_to_all instead and its line says \"transport\": \"torch-fallback\"", file=sys.stderr)

    def step():
        brec, bcnt = xj.partition(build_side, n_ord, False, stream, dev, key="build", row_base=sh["o_row_base"])
        precs, pcnt = xj.partition(probe_side, n_li, False, stream, dev, key="probe", filt=pfilter,
                                   row_base=sh["l_row_base"])
        if rx is not None:  # the C-ABI's RCCL exchange (hy_join_exchange_counts / _records)
            brecv, bmat = rx.exchange(brec, bcnt, rb, stream)
            precv, pmat = rx.exchange(precs, pcnt, rb, stream)
        else:
            brecv, bmat = hdist.exchange_records(dist, brec.to(xdev), bcnt, rank, world, device=xdev, record_bytes=rb)
            precv, pmat = hdist.exchange_records(dist, precs.to(xdev), pcnt, rank, world, device=xdev,
                                                 record_bytes=rb)
            brecv, precv = brecv.to(dev), precv.to(dev)
        out = xj.join(brecv, bmat, precv, pmat, rank, stream, dev)
        state["recv_rows"] = (int(bmat.sum()), int(pmat.sum()))
        state["sent_bytes"] = (int(bcnt.sum()) + int(pcnt.sum())) * rb
        state["out"] = out
        return int(pcnt.sum()), out[4]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n_probe, pairs = step()
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    # per-kernel device times: K more steps with HIP events around every launch (kept out of the timed region)
    L.hy_kernel_stats_reset()
    L.hy_kernel_stats_enable(1)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    L.hy_kernel_stats_enable(0)
    # per-rank output check of the last step against the single-GPU layout (dist.check_partition_output)
    out_b, out_p, pbeg, pcnt = state["out"][:4]
    first_bucket, _ = hdist.owned_buckets(xj.n_buckets, rank, world)
    check = hdist.check_partition_output(expected, out_b, out_p, pbeg, pcnt,
                                         first_bucket << (radix_bits - xj.first_bits), chunk)
    bad = torch.tensor([0 if all(check.values()) else 1], dtype=torch.int64, device=xdev)
    dist.all_reduce(bad)
    check["ranks_failing"] = int(bad.item())
    check["status"] = "ok" if check["ranks_failing"] == 0 else "mismatch"
    check["pairs_checked"] = None  # set below from the whole job's pairs
    t = torch.tensor([elapsed], dtype=torch.float64, device=xdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    tot = torch.tensor([n_probe, pairs, state["sent_bytes"]], dtype=torch.int64, device=xdev)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    g_probe, g_pairs, g_sent = (int(x) for x in tot.tolist())
    assert int(scan_begin[n_lc].item()) == n_probe  # the fused scan's output = the probe records
    check["pairs_checked"] = g_pairs
    check["expected_pairs"] = int(expected[0].sum())

    from bench import kernel_stats, HBM_PEAK_GBPS  # noqa: E402  (shared helpers)

    kernels = kernel_stats(L)
    K = args.steps
    step_s = elapsed / K
    # algorithmic bytes, whole job: scan 1 B/row + 4 B/match; JoinHash 4 B/build row + 4 B/probe
    # row + 16 B/pair; per rank its share, against N x the HBM peak
    e2e = n_li_g * 1 + g_probe * 4 + n_ord_g * 4 + g_probe * 4 + g_pairs * 16
    for v in kernels.values():
        v["ms_per_launch"] = v["ms_total"] / max(v["launches"], 1)
    if rank == 0:
        achieved = e2e / step_s / 1e9
        line = {
            "metric": "rows/sec TableScan+JoinHash, TPC-H SF100 lineitem⋈orders, 1/2/4/8 MI355X",
            "value": round((n_li_g + n_ord_g) / step_s, 1),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 3),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded counter-based TPC-H-shaped columns, resident in HBM)",
            "config": {"workload": f"TableScan(l_quantity<24, dictionary u8) fused into the exchange partition -> "
                                   f"distributed JoinHash(orders ⋈ scan, o_orderkey=l_orderkey, "
                                   f"radix_bits={radix_bits})",
                       "path": "hy_scan_join_exchange_partition + " + transport_note + " + hy_join_exchange_join_rows",
                       "transport": transport, "transport_error": transport_error,
                       "sf_total": global_sf, "lineitem_rows": n_li_g, "orders_rows": n_ord_g, "chunk_size": chunk,
                       "scan_matches": g_probe, "join_pairs": g_pairs, "record_bytes": rb,
                       "exchange_bytes_per_step": g_sent,
                       "parallelism": f"chunk-sharded x{world}, {'RCCL' if nccl else 'gloo'} all-to-all radix "
                                      f"exchange"},
            "roofline": {"bound": "hbm", "scope": "end-to-end step, whole job (algorithmic bytes of SURVEY 8(d))",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS * world, "unit": "GB/s",
                         "frac": round(achieved / (HBM_PEAK_GBPS * world), 4), "alg_bytes_per_step": e2e,
                         "traffic": None, "peak_source": f"{world} x the MI355X HBM spec"},
            "kernels_rank0": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                              for k, v in kernels.items()},
            "cpu_baseline": None,
            "check": check,
        }
        print(json.dumps(line))
    if rx is not None:
        rx.close()
    dist.destroy_process_group()
