"""Device mirrors of numpy-built tables for C-ABI tests: per chunk, a ValueColumn (values + optional null flags) or a
DictionaryColumn encoded exactly as the reference's DictionaryEncoder does it (sorted distinct non-NULL values,
value id = rank, NULL value id = dictionary size, FixedSizeByteAligned width from the dictionary size:
dictionary_encoder.hpp:57-130, fixed_size_byte_aligned_compressor.cpp:21-30), plus the host dictionary rewrite of
a scan predicate (single_column_table_scan_impl.cpp:87-205)."""
import ctypes

import numpy as np

INVALID_VALUE_ID = 0xFFFFFFFF


def dict_encode(values, nulls):
    valid = values if nulls is None else values[nulls == 0]
    dictionary = np.unique(valid)
    vids = np.searchsorted(dictionary, values).astype(np.uint32)
    if nulls is not None:
        vids[nulls != 0] = dictionary.size
    width = 1 if dictionary.size <= 0xFF else (2 if dictionary.size <= 0xFFFF else 4)
    return dictionary, vids.astype({1: np.uint8, 2: np.uint16, 4: np.uint32}[width]), width


def lower_bound(dictionary, v):
    i = int(np.searchsorted(dictionary, v, side="left"))
    return INVALID_VALUE_ID if i == dictionary.size else i


def upper_bound(dictionary, v):
    i = int(np.searchsorted(dictionary, v, side="right"))
    return INVALID_VALUE_ID if i == dictionary.size else i


def dictionary_predicate(capi, dictionary, cond, value):
    """(op, search_vid) of operators.cpp dictionary_predicate for cond in {Equals, NotEquals, LessThan,
    LessThanEquals, GreaterThan, GreaterThanEquals}."""
    svid = upper_bound(dictionary, value) if cond in ("LessThanEquals", "GreaterThan") else lower_bound(dictionary, value)
    ub = upper_bound(dictionary, value)
    one = dictionary.size == 1
    if cond == "Equals":
        all_, none = svid != ub and one, svid == ub
    elif cond == "NotEquals":
        all_, none = svid == ub, svid == ub and one
    elif cond in ("LessThan", "LessThanEquals"):
        all_, none = svid == INVALID_VALUE_ID, svid == 0
    else:
        all_, none = svid == 0, svid == INVALID_VALUE_ID
    if all_:
        return capi.HY_OP_ALL, svid
    if none:
        return capi.HY_OP_NONE, svid
    return {"Equals": capi.HY_OP_EQ, "NotEquals": capi.HY_OP_NE, "LessThan": capi.HY_OP_LT,
            "LessThanEquals": capi.HY_OP_LT}.get(cond, capi.HY_OP_GE), svid


VALUE_OPS = {"Equals": 0, "NotEquals": 1, "LessThan": 2, "LessThanEquals": 3, "GreaterThan": 4, "GreaterThanEquals": 5}
HY_TYPES = {np.dtype(np.int32): 1, np.dtype(np.int64): 2, np.dtype(np.float32): 3, np.dtype(np.float64): 4}


class DeviceColumn:
    """One column of a chunked table on the device: chunk c = rows [c * chunk, (c + 1) * chunk)."""

    def __init__(self, capi, values, nulls, chunk, encoding):
        self.capi, self.values, self.nulls, self.chunk, self.encoding = capi, values, nulls, chunk, encoding
        self.n_chunks = (values.size + chunk - 1) // chunk if values.size else 0
        self.dev, self.descs = [], []
        for c in range(self.n_chunks):
            v = np.ascontiguousarray(values[c * chunk:(c + 1) * chunk])
            nl = None if nulls is None else np.ascontiguousarray(nulls[c * chunk:(c + 1) * chunk]).astype(np.uint8)
            d = capi.ColumnChunk()
            d.size = v.size
            keep = []
            if encoding == "Dictionary":
                dictionary, vids, width = dict_encode(v, nl)
                keep += [capi.DeviceArray(vids), capi.DeviceArray(dictionary if dictionary.size else v[:1])]
                d.kind, d.vid_width = capi.HY_COL_DICT, width
                d.data, d.dictionary = keep[0].ptr.value, keep[1].ptr.value
                d.dictionary_size = dictionary.size
                keep.append(dictionary)
            else:
                keep.append(capi.DeviceArray(v))
                d.kind, d.data = capi.HY_COL_VALUE, keep[0].ptr.value
                if nl is not None:
                    keep.append(capi.DeviceArray(nl))
                    d.nulls = keep[1].ptr.value
            self.dev.append(keep)
            self.descs.append(d)

    def chunk_size(self, c):
        return self.descs[c].size

    def scan_chunks(self, cond, value):
        """hy_scan_chunk per chunk for `column cond value` (dictionary rewrite on the host)."""
        capi = self.capi
        arr = (capi.ScanChunk * max(1, self.n_chunks))()
        for c in range(self.n_chunks):
            s = arr[c]
            s.column = self.descs[c]
            if self.encoding == "Dictionary":
                s.op, s.search_vid = dictionary_predicate(capi, self.dev[c][2], cond, value)
            else:
                s.op = VALUE_OPS[cond]
        return arr

    def constant(self, value):
        return np.array([value], dtype=self.values.dtype)


def join_side(capi, col, chunk_ids=None):
    """hy_join_side over the chunks of a data-table column."""
    arr = (capi.JoinChunk * max(1, col.n_chunks))()
    for c in range(col.n_chunks):
        j = arr[c]
        j.column = col.descs[c]
        j.size = col.descs[c].size
        j.chunk_id = c if chunk_ids is None else chunk_ids[c]
        j.single_chunk = capi.HY_MIXED_CHUNKS
    side = capi.JoinSide(arr, col.n_chunks, HY_TYPES[col.values.dtype], None, 0, 0, 0)
    side._keep = arr
    return side
