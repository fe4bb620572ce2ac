"""ctypes view of the C-ABI in include/hyrise_amd.h (libhyrise_amd.so).

Used by bench.py and the multi-GPU shard driver to call the kernels on device buffers that are owned elsewhere
(torch tensors), and by tests to check that the library exports every declared entry point. Structures mirror the
header field for field.
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# HY_AMD_LIB: an alternative build of the same library (kernel-variant experiments); default the in-tree build
LIB_PATH = os.environ.get("HY_AMD_LIB") or os.path.join(_HERE, "_lib", "libhyrise_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "hyrise_amd.h")

lib = ctypes.CDLL(LIB_PATH)

HY_OK, HY_ERR_CAPACITY, HY_ERR_GROUP_BOUND = 0, 6, 8
HY_TYPE_INT32, HY_TYPE_INT64, HY_TYPE_FLOAT, HY_TYPE_DOUBLE = 1, 2, 3, 4
HY_COL_VALUE, HY_COL_DICT = 0, 1
HY_OP_EQ, HY_OP_NE, HY_OP_LT, HY_OP_LE, HY_OP_GT, HY_OP_GE, HY_OP_ALL, HY_OP_NONE, HY_OP_IS_NULL, HY_OP_IS_NOT_NULL, HY_OP_VID_SET = range(11)
HY_JOIN_INNER, HY_JOIN_LEFT, HY_JOIN_RIGHT, HY_JOIN_SEMI, HY_JOIN_ANTI = 0, 1, 2, 5, 6
HY_AGG_MIN, HY_AGG_MAX, HY_AGG_SUM, HY_AGG_AVG, HY_AGG_COUNT, HY_AGG_COUNT_DISTINCT = range(6)
HY_AGG_MAX_AGGREGATES = 16
HY_PROBE_READ, HY_PROBE_COPY = 0, 1
HY_EXPR_COLUMN, HY_EXPR_VALUE, HY_EXPR_ADD, HY_EXPR_SUB, HY_EXPR_MUL, HY_EXPR_DIV, HY_EXPR_MOD = range(7)


class RowID(ctypes.Structure):
    _fields_ = [("chunk_id", ctypes.c_uint32), ("chunk_offset", ctypes.c_uint32)]


class ColumnChunk(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("nulls", ctypes.c_void_p), ("dictionary", ctypes.c_void_p),
                ("size", ctypes.c_uint32), ("dictionary_size", ctypes.c_uint32), ("kind", ctypes.c_int32),
                ("vid_width", ctypes.c_int32)]


class ScanChunk(ctypes.Structure):
    _fields_ = [("column", ColumnChunk), ("op", ctypes.c_int32), ("search_vid", ctypes.c_uint32),
                ("out_begin", ctypes.c_uint64), ("vid_set", ctypes.c_void_p)]


HY_MIXED_CHUNKS = 0xFFFFFFFF


class JoinChunk(ctypes.Structure):
    _fields_ = [("column", ColumnChunk), ("pos_list", ctypes.c_void_p), ("size", ctypes.c_uint32),
                ("chunk_id", ctypes.c_uint32), ("single_chunk", ctypes.c_uint32), ("referenced_offset", ctypes.c_uint32)]


class JoinSide(ctypes.Structure):
    _fields_ = [("chunks", ctypes.POINTER(JoinChunk)), ("n_chunks", ctypes.c_uint32), ("value_type", ctypes.c_int32),
                ("referenced", ctypes.POINTER(ColumnChunk)), ("n_referenced", ctypes.c_uint32),
                ("fuse_dereference", ctypes.c_int32), ("referenced_chunk_base", ctypes.c_uint32)]


class JoinFilter(ctypes.Structure):
    _fields_ = [("chunks", ctypes.POINTER(ScanChunk)), ("value_type", ctypes.c_int32), ("constant", ctypes.c_void_p),
                ("out_offsets", ctypes.c_void_p), ("out_chunk_begin", ctypes.c_void_p), ("n_chunks", ctypes.c_uint32),
                ("out_row_ids", ctypes.c_void_p)]

    def __init__(self, chunks=None, value_type=0, constant=None, out_offsets=None, out_chunk_begin=None,
                 n_chunks=None, out_row_ids=None):
        # n_chunks defaults to the length of a ctypes array of predicate chunks (the side's chunk count)
        if n_chunks is None:
            n_chunks = len(chunks) if chunks is not None and hasattr(chunks, "__len__") else 0
        super().__init__(chunks, value_type, constant, out_offsets, out_chunk_begin, n_chunks, out_row_ids)


class JoinParams(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("hashed_type", ctypes.c_int32), ("radix_bits", ctypes.c_uint32),
                ("seed", ctypes.c_uint32), ("key_hash", ctypes.c_void_p)]


class JoinResult(ctypes.Structure):
    _fields_ = [("total_pairs", ctypes.c_uint64), ("capacity_required", ctypes.c_uint64)]


class ExprNode(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("type", ctypes.c_int32), ("calc_type", ctypes.c_int32),
                ("column", ctypes.c_int32), ("value", ctypes.c_uint64)]


class AggColumn(ctypes.Structure):
    _fields_ = [("value_type", ctypes.c_int32), ("pos_group", ctypes.c_int32), ("chunks", ctypes.POINTER(ColumnChunk)),
                ("n_chunks", ctypes.c_uint32), ("domain", ctypes.c_uint32), ("program", ctypes.POINTER(ExprNode)),
                ("n_nodes", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class AggInput(ctypes.Structure):
    _fields_ = [("n_chunks", ctypes.c_uint32), ("chunk_sizes", ctypes.POINTER(ctypes.c_uint32)),
                ("pos_lists", ctypes.POINTER(ctypes.c_void_p)), ("n_pos_groups", ctypes.c_uint32),
                ("columns", ctypes.POINTER(AggColumn)), ("n_columns", ctypes.c_uint32),
                ("filter", ctypes.POINTER(ScanChunk)), ("filter_value_type", ctypes.c_int32),
                ("filter_constant", ctypes.c_void_p)]


class AggDef(ctypes.Structure):
    _fields_ = [("function", ctypes.c_int32), ("column", ctypes.c_int32)]


class AggParams(ctypes.Structure):
    _fields_ = [("groupby", ctypes.POINTER(ctypes.c_int32)), ("n_groupby", ctypes.c_uint32),
                ("aggregates", ctypes.POINTER(AggDef)), ("n_aggregates", ctypes.c_uint32),
                ("group_bound", ctypes.c_uint64)]


class AggLayout(ctypes.Structure):
    _fields_ = [("words", ctypes.c_uint32), ("dense", ctypes.c_uint32),
                ("agg_word", ctypes.c_uint32 * HY_AGG_MAX_AGGREGATES),
                ("agg_emin", ctypes.c_int32 * HY_AGG_MAX_AGGREGATES),
                ("agg_limbs", ctypes.c_uint32 * HY_AGG_MAX_AGGREGATES)]


class StringPredicate(ctypes.Structure):
    _fields_ = [("value", ctypes.c_char_p), ("value_len", ctypes.c_uint32), ("pattern_regex", ctypes.c_int32),
                ("pattern", ctypes.c_char_p), ("pattern_len", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


_sigs = {
    "hy_get_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "hy_set_device": (ctypes.c_int, [ctypes.c_int]),
    "hy_last_error_message": (ctypes.c_char_p, []),
    "hy_build_info": (ctypes.c_char_p, []),
    "hy_stream_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "hy_stream_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p)]),
    "hy_stream_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "hy_malloc": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]),
    "hy_free": (ctypes.c_int, [ctypes.c_void_p]),
    "hy_memcpy_htod": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "hy_memcpy_dtoh": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "hy_table_scan_workspace_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_size_t)]),
    "hy_table_scan": (ctypes.c_int, [ctypes.POINTER(ScanChunk), ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_void_p]),
    "hy_join_radix_bits": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint32]),
    "hy_murmur2": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                  ctypes.c_void_p]),
    "hy_join_hash_workspace_size": (ctypes.c_int, [ctypes.POINTER(JoinSide), ctypes.POINTER(JoinSide),
                                                   ctypes.POINTER(JoinParams), ctypes.POINTER(ctypes.c_size_t)]),
    "hy_join_hash": (ctypes.c_int, [ctypes.POINTER(JoinSide), ctypes.POINTER(JoinSide), ctypes.POINTER(JoinParams),
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.POINTER(JoinResult), ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_void_p]),
    "hy_scan_join_hash_workspace_size": (ctypes.c_int, [ctypes.POINTER(JoinSide), ctypes.POINTER(JoinFilter),
                                                        ctypes.POINTER(JoinSide), ctypes.POINTER(JoinFilter),
                                                        ctypes.POINTER(JoinParams), ctypes.POINTER(ctypes.c_size_t)]),
    "hy_scan_join_hash": (ctypes.c_int, [ctypes.POINTER(JoinSide), ctypes.POINTER(JoinFilter), ctypes.POINTER(JoinSide),
                                         ctypes.POINTER(JoinFilter), ctypes.POINTER(JoinParams), ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.POINTER(JoinResult), ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_void_p]),
    "hy_stream_bandwidth_probe": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32,
                                                 ctypes.c_void_p]),
    "hy_expand_row_ids": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "hy_table_scan_count": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_size_t, ctypes.c_void_p]),
    "hy_expand_chunk_row_ids": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                               ctypes.c_void_p, ctypes.c_void_p]),
    "hy_aggregate_layout": (ctypes.c_int, [ctypes.POINTER(AggInput), ctypes.POINTER(AggParams),
                                           ctypes.POINTER(AggLayout)]),
    "hy_aggregate_workspace_size": (ctypes.c_int, [ctypes.POINTER(AggInput), ctypes.POINTER(AggParams),
                                                   ctypes.POINTER(ctypes.c_size_t)]),
    "hy_aggregate": (ctypes.c_int, [ctypes.POINTER(AggInput), ctypes.POINTER(AggParams), ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p,
                                    ctypes.c_size_t, ctypes.c_void_p]),
    "hy_projection_workspace_size": (ctypes.c_int, [ctypes.POINTER(AggInput), ctypes.POINTER(ctypes.c_size_t)]),
    "hy_projection": (ctypes.c_int, [ctypes.POINTER(AggInput), ctypes.POINTER(ExprNode), ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_void_p]),
    "hy_projection_multi": (ctypes.c_int, [ctypes.POINTER(AggInput), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_void_p]),
    "hy_agg_float_sum": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, ctypes.c_int32,
                                        ctypes.c_uint64, ctypes.POINTER(ctypes.c_double)]),
    "hy_agg_float_sums": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p]),
    "hy_agg_decode_ordered": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_int32]),
    "hy_join_exchange_bucket_bits": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32]),
    "hy_join_exchange_partition_workspace_size": (ctypes.c_int, [ctypes.POINTER(JoinSide), ctypes.POINTER(JoinParams),
                                                                 ctypes.c_uint32, ctypes.POINTER(ctypes.c_size_t)]),
    "hy_join_exchange_partition": (ctypes.c_int, [ctypes.POINTER(JoinSide), ctypes.POINTER(JoinParams), ctypes.c_int32,
                                                  ctypes.c_uint32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                                  ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "hy_join_exchange_join_workspace_size": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64),
                                                            ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32,
                                                            ctypes.c_uint32, ctypes.POINTER(JoinParams),
                                                            ctypes.POINTER(ctypes.c_size_t)]),
    "hy_join_exchange_join": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p,
                                             ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.POINTER(JoinParams), ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.POINTER(JoinResult), ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_void_p]),
    "hy_join_exchange_row_record_bytes": (ctypes.c_uint32, [ctypes.c_int32]),
    "hy_scan_join_exchange_partition_workspace_size": (ctypes.c_int, [ctypes.POINTER(JoinSide),
                                                                      ctypes.POINTER(JoinFilter),
                                                                      ctypes.POINTER(JoinParams), ctypes.c_uint32,
                                                                      ctypes.POINTER(ctypes.c_size_t)]),
    "hy_scan_join_exchange_partition": (ctypes.c_int, [ctypes.POINTER(JoinSide), ctypes.POINTER(JoinFilter),
                                                       ctypes.POINTER(JoinParams), ctypes.c_int32, ctypes.c_uint32,
                                                       ctypes.c_uint64, ctypes.c_void_p,
                                                       ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p,
                                                       ctypes.c_size_t, ctypes.c_void_p]),
    "hy_join_exchange_join_rows_workspace_size": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64),
                                                                 ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32,
                                                                 ctypes.c_uint32, ctypes.POINTER(JoinParams),
                                                                 ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                                                 ctypes.c_uint32, ctypes.POINTER(ctypes.c_size_t)]),
    "hy_join_exchange_join_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p,
                                                  ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, ctypes.c_uint32,
                                                  ctypes.c_uint32, ctypes.POINTER(JoinParams), ctypes.c_void_p,
                                                  ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.POINTER(JoinResult), ctypes.c_void_p, ctypes.c_size_t,
                                                  ctypes.c_void_p]),
    "hy_aggregate_merge": (ctypes.c_int, [ctypes.POINTER(AggParams), ctypes.POINTER(AggLayout),
                                          ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)),
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64,
                                          ctypes.POINTER(ctypes.c_uint64)]),
    "hy_murmur2_bytes": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32]),
    "hy_comm_get_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "hy_comm_init": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]),
    "hy_comm_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "hy_join_exchange_counts": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32,
                                               ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]),
    "hy_join_exchange_records": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, ctypes.c_void_p,
                                                ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                                ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]),
    "hy_reference_scan_order_workspace_size": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32,
                                                              ctypes.POINTER(ctypes.c_size_t)]),
    "hy_reference_scan_order": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                               ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_size_t, ctypes.c_void_p]),
    "hy_column_compare_scan_workspace_size": (ctypes.c_int, [ctypes.POINTER(JoinSide), ctypes.POINTER(JoinSide),
                                                             ctypes.c_int32, ctypes.POINTER(ctypes.c_size_t)]),
    "hy_column_compare_scan": (ctypes.c_int, [ctypes.POINTER(JoinSide), ctypes.POINTER(JoinSide), ctypes.c_int32,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "hy_validate_workspace_size": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.POINTER(ctypes.c_size_t)]),
    "hy_validate": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_void_p]),
    "hy_validate_pos_list": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "hy_decode_run_length": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p]),
    "hy_decode_frame_of_reference": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "hy_exchange_record_row_ids": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                                  ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "hy_exchange_records_localize": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_void_p]),
    "hy_table_scan_row_ids": (ctypes.c_int, [ctypes.POINTER(ScanChunk), ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_size_t, ctypes.c_void_p]),
    "hy_pos_list_null_positions": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "hy_decode_simd_bp128": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32,
                                             ctypes.c_void_p, ctypes.c_void_p]),
    "hy_scan_join_plan_create": (ctypes.c_int, [ctypes.POINTER(JoinSide), ctypes.POINTER(JoinFilter),
                                                 ctypes.POINTER(JoinSide), ctypes.POINTER(JoinFilter),
                                                 ctypes.POINTER(JoinParams), ctypes.POINTER(ctypes.c_void_p)]),
    "hy_scan_join_plan_execute": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(JoinResult),
                                                  ctypes.c_void_p]),
    "hy_scan_join_plan_rebind": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(JoinFilter), ctypes.POINTER(JoinFilter)]),
    "hy_scan_join_plan_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "hy_string_table_scan_workspace_size": (ctypes.c_int, [ctypes.POINTER(ScanChunk), ctypes.c_uint32,
                                                           ctypes.POINTER(StringPredicate),
                                                           ctypes.POINTER(ctypes.c_size_t)]),
    "hy_string_table_scan": (ctypes.c_int, [ctypes.POINTER(ScanChunk), ctypes.c_uint32, ctypes.POINTER(StringPredicate),
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "hy_string_reference_scan_workspace_size": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32,
                                                               ctypes.POINTER(StringPredicate),
                                                               ctypes.POINTER(ctypes.c_size_t)]),
    "hy_string_reference_scan": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ScanChunk),
                                                ctypes.c_uint32, ctypes.POINTER(StringPredicate), ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
}
HY_COMM_ID_BYTES = 128
for _name, (_res, _args) in _sigs.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


class HyError(RuntimeError):
    pass


def check(status, what=""):
    if status != HY_OK:
        raise HyError(f"{what} failed ({status}): {lib.hy_last_error_message().decode()}")


def declared_symbols():
    """Entry points declared in include/hyrise_amd.h and include/hyrise_amd_trace.h."""
    text = open(HEADER_PATH).read() + open(os.path.join(os.path.dirname(HEADER_PATH), "hyrise_amd_trace.h")).read()
    return sorted(set(re.findall(r"^\s*(?:hy_status|uint32_t|uint64_t|const char\*)\s+(hy_\w+)\s*\(", text, re.M)))


def device_count():
    n = ctypes.c_int(0)
    check(lib.hy_get_device_count(ctypes.byref(n)), "hy_get_device_count")
    return n.value


class DeviceArray:
    """A numpy array mirrored in device memory through the C-ABI's own allocator (tests; no torch involved)."""

    def __init__(self, host):
        import numpy as np

        self.host = np.ascontiguousarray(host)
        self.ptr = ctypes.c_void_p()
        check(lib.hy_malloc(ctypes.byref(self.ptr), max(16, self.host.nbytes)), "hy_malloc")
        check(lib.hy_memcpy_htod(self.ptr, self.host.ctypes.data, self.host.nbytes, None), "hy_memcpy_htod")
        check(lib.hy_stream_synchronize(None), "sync")

    def fetch(self):
        check(lib.hy_memcpy_dtoh(self.host.ctypes.data, self.ptr, self.host.nbytes, None), "hy_memcpy_dtoh")
        check(lib.hy_stream_synchronize(None), "sync")
        return self.host

    def __del__(self):
        if getattr(self, "ptr", None) and self.ptr.value:
            lib.hy_free(self.ptr)
