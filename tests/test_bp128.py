"""SIMD-BP128 attribute vectors (reference src/lib/storage/vector_compression/simd_bp128/): the host packing is
checked word for word against oracle/bp128.py (a restatement of the reference compressor, pinned by the reference's
own simd_bp128_test.cpp sequences), the device decoder hy_decode_simd_bp128 id for id, and scans / joins /
aggregates over SIMD-BP128 dictionary chunks against the oracle."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import bp128  # noqa: E402

from helpers import assert_identical, wrap  # noqa: E402


@pytest.mark.parametrize("bit_size", range(1, 33))
def test_reference_sequences(hy, bit_size):
    """simd_bp128_test.cpp:55-99 (bit sizes 1..32, 4,200 values): restatement round trip, and the product's
    compressor writes exactly the restatement's words."""
    seq = bp128.reference_sequence(bit_size)
    words, meta = bp128.encode(seq)
    assert np.array_equal(bp128.decode(words, meta, len(seq)), seq.astype(np.uint32))
    data, hmeta, back, _ = hy.compress_vector(seq.astype(np.uint32).tolist(), int(seq.max()),
                                              hy.VectorCompressionType.SimdBp128)
    assert data == words.tobytes()
    assert list(hmeta) == meta
    assert np.array_equal(np.array(back, dtype=np.uint32), seq.astype(np.uint32))


@pytest.mark.parametrize("n", [1, 127, 128, 129, 2047, 2048, 2049, 5000])
def test_ragged_and_zero_blocks(hy, n):
    """Partial last blocks / meta blocks and all-zero (width 0) blocks between wide ones."""
    rng = np.random.default_rng(n)
    ids = rng.integers(0, 1 << int(rng.integers(1, 18)), n).astype(np.uint32)
    ids[(np.arange(n) // 128) % 3 == 1] = 0  # every third block is all zeros
    words, meta = bp128.encode(ids)
    data, hmeta, back, width = hy.compress_vector(ids.tolist(), int(ids.max()) + 1, hy.VectorCompressionType.SimdBp128)
    assert data == words.tobytes() and list(hmeta) == meta
    assert np.array_equal(np.array(back, dtype=np.uint32), ids)
    assert width == (1 if ids.max() + 1 <= 0xFF else 2 if ids.max() + 1 <= 0xFFFF else 4)


def bp128_table(hy, rng, n, chunk, distinct, null_frac, compression):
    vals = rng.integers(0, distinct, n).astype(np.int32)
    nulls = (rng.random(n) < null_frac).astype(np.uint8)
    t = hy.Table.from_arrays([("a", hy.DataType.Int, True), ("b", hy.DataType.Int, False)],
                             [vals, np.arange(n, dtype=np.int32)], [nulls, None], chunk)
    hy.encode_all_chunks(t, hy.EncodingType.Dictionary, compression)
    return t


def test_dictionary_columns(hy):
    """A dictionary chunk's ids are the same whichever vector compression holds them."""
    for distinct in (3, 200, 70_000):
        a = bp128_table(hy, np.random.default_rng(distinct), 9_000, 4_001, distinct, 0.05,
                        hy.VectorCompressionType.SimdBp128)
        f = bp128_table(hy, np.random.default_rng(distinct), 9_000, 4_001, distinct, 0.05,
                        hy.VectorCompressionType.FixedSizeByteAligned)
        for c in range(a.chunk_count()):
            ca, cf = a.get_chunk(c).get_column(0), f.get_chunk(c).get_column(0)
            assert ca.attribute_vector_compression() == hy.VectorCompressionType.SimdBp128
            ids = np.array(cf.attribute_vector_ids(), dtype=np.uint32)
            assert np.array_equal(np.array(ca.attribute_vector_ids(), dtype=np.uint32), ids)
            words, _ = bp128.encode(ids)
            assert ca.attribute_vector_bytes() == words.tobytes()
            assert ca.values() == cf.values()


@pytest.mark.gpu
def test_device_decode(hy):
    """hy_decode_simd_bp128 against the restatement, every bit size and output width."""
    capi, L = hy.capi, hy.capi.lib
    for bit_size in range(1, 33):
        seq = bp128.reference_sequence(bit_size, 9_000).astype(np.uint32)
        words, meta = bp128.encode(seq)
        dw = capi.DeviceArray(np.concatenate([words, np.zeros(4, np.uint32)]))
        dm = capi.DeviceArray(np.array(meta, dtype=np.uint32))
        for width, dt in ((1, np.uint8), (2, np.uint16), (4, np.uint32)):
            if bit_size > 8 * width:
                continue
            out = capi.DeviceArray(np.zeros(len(seq), dt))
            capi.check(L.hy_decode_simd_bp128(dw.ptr, dm.ptr, len(seq), width, out.ptr, None), "hy_decode_simd_bp128")
            assert np.array_equal(out.fetch(), seq.astype(dt)), (bit_size, width)


@pytest.mark.gpu
def test_operators_on_bp128_chunks(hy, oracle):
    """TableScan (data + reference input), JoinHash and Aggregate read SIMD-BP128 dictionary chunks (decoded once into
    the HBM id mirror) bit-exactly as the oracle reads them through the host decoder."""
    rng = np.random.default_rng(0x5B1)
    for distinct in (40, 300, 70_000):
        t = bp128_table(hy, rng, 150_000, 65_536, distinct, 0.03, hy.VectorCompressionType.SimdBp128)
        w = wrap(hy, t)
        for cond in ("Equals", "NotEquals", "LessThan", "GreaterThanEquals", "IsNull"):
            s = hy.TableScan(w, 0, getattr(hy.PredicateCondition, cond), None if cond == "IsNull" else distinct // 3)
            s.execute()
            exp = oracle.table_scan(t, 0, getattr(hy.PredicateCondition, cond),
                                    None if cond == "IsNull" else distinct // 3, [])
            assert_identical(s.get_output(), exp)
        s1 = hy.TableScan(w, 1, hy.PredicateCondition.LessThan, 100_000)
        s1.execute()
        s2 = hy.TableScan(s1, 0, hy.PredicateCondition.GreaterThan, distinct // 2)
        s2.execute()
        assert_identical(s2.get_output(),
                         oracle.table_scan(s1.get_output(), 0, hy.PredicateCondition.GreaterThan, distinct // 2, []))
    small = bp128_table(hy, rng, 40_000, 10_000, 500, 0.0, hy.VectorCompressionType.SimdBp128)
    other = bp128_table(hy, rng, 30_000, 7_000, 500, 0.02, hy.VectorCompressionType.SimdBp128)
    j = hy.JoinHash(wrap(hy, small), wrap(hy, other), hy.JoinMode.Inner, (0, 0), hy.PredicateCondition.Equals)
    j.execute()
    assert_identical(j.get_output(), oracle.join_hash(small, other, hy.JoinMode.Inner, (0, 0))[0])
    agg = hy.Aggregate(wrap(hy, other), [hy.AggregateColumnDefinition(1, hy.AggregateFunction.Sum)], [0])
    agg.execute()
    exp = oracle.aggregate(other, [hy.AggregateColumnDefinition(1, hy.AggregateFunction.Sum)], [0])
    assert_identical(agg.get_output(), exp)
