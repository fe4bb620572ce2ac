"""Binary table files (reference ImportBinary / ExportBinary, import_binary.cpp / export_binary.cpp; the loader that
feeds encoded chunks to HBM): every case of the reference's import_binary_test.cpp and export_binary_test.cpp against
the reference's own fixtures (src/test/binary/*.bin, copied as data into tests/golden/binary/). Import: the table each
file decodes to, chunk layout and encodings included; export: the exact bytes of the fixture. Host-only."""
import os

import pytest

from helpers import ROOT, assert_table_eq_unordered, tbl

BIN = os.path.join(ROOT, "tests", "golden", "binary")
ALL5 = [("a", "String"), ("b", "Int"), ("c", "Long"), ("d", "Float"), ("e", "Double")]
ROWS5 = [["AAAAA", 1, 100, 1.1, 11.1], ["BBBBBBBBBB", 2, 200, 2.2, 22.2],
         ["CCCCCCCCCCCCCCC", 3, 300, 3.3, 33.3], ["DDDDDDDDDDDDDDDDDDDD", 4, 400, 4.4, 44.4]]
NULL5 = [[None, 1.1, 100, "one", 1.11], [2, None, 200, "two", 2.22], [3, 3.3, None, "three", 3.33],
         [4, 4.4, 400, None, 4.44], [5, 5.5, 500, "five", None]]


def make(hy, defs, rows, chunk, nullable=False):
    t = hy.Table([(n, getattr(hy.DataType, ty), nullable) for n, ty in defs], hy.TableType.Data, chunk)
    for r in rows:
        t.append(r)
    return t


def assert_ordered(actual, expected):
    """EXPECT_TABLE_EQ_ORDERED: schema, then rows in order."""
    assert_table_eq_unordered(actual, expected)
    assert [list(map(_round, r)) for r in actual.rows()] == [list(map(_round, r)) for r in expected.rows()]


def _round(v):
    return round(v, 4) if isinstance(v, float) else v


def cases(hy):
    """(fixture, expected table) of import_binary_test.cpp / export_binary_test.cpp."""
    f = [("a", "Float")]
    s = [("a", "String")]
    strs = [["This"], ["is"], ["a"], ["test"]]
    dict_s = make(hy, s, strs, 10)
    hy.encode_all_chunks(dict_s, hy.EncodingType.Dictionary)
    dict5 = make(hy, ALL5, ROWS5, 2)
    hy.encode_all_chunks(dict5, hy.EncodingType.Dictionary)
    mix5 = make(hy, ALL5, ROWS5, 2)
    hy.encode_chunks(mix5, [0], hy.EncodingType.Dictionary)
    return {
        "SingleChunkSingleFloatColumn": make(hy, f, [[5.5], [13.0], [16.2]], 5),
        "MultipleChunkSingleFloatColumn": make(hy, f, [[5.5], [13.0], [16.2]], 2),
        "StringValueColumn": make(hy, s, strs, 5),
        "StringDictionaryColumn": dict_s,
        "AllTypesValueColumn": make(hy, ALL5, ROWS5, 2),
        "AllTypesDictionaryColumn": dict5,
        "AllTypesMixColumn": mix5,
        "TwoColumnsNoValues": make(hy, [("FirstColumn", "Int"), ("SecondColumn", "String")], [], 30000),
        "EmptyStringsValueColumn": make(hy, s, [[""]] * 5, 10),
    }


@pytest.mark.parametrize("name", ["SingleChunkSingleFloatColumn", "MultipleChunkSingleFloatColumn",
                                  "StringValueColumn", "StringDictionaryColumn", "AllTypesValueColumn",
                                  "AllTypesDictionaryColumn", "AllTypesMixColumn", "TwoColumnsNoValues",
                                  "EmptyStringsValueColumn"])
def test_import_matches_reference_fixture(hy, name):
    expected = cases(hy)[name]
    got = hy.import_binary(os.path.join(BIN, name + ".bin"))
    assert_ordered(got, expected)
    assert got.chunk_count() == expected.chunk_count()
    assert got.max_chunk_size() == expected.max_chunk_size()
    for c in range(expected.chunk_count()):  # each chunk keeps its stored encoding
        for col in range(expected.column_count()):
            assert (got.get_chunk(c).get_column(col).encoding_type() ==
                    expected.get_chunk(c).get_column(col).encoding_type())


@pytest.mark.parametrize("name", ["SingleChunkSingleFloatColumn", "MultipleChunkSingleFloatColumn",
                                  "StringValueColumn", "StringDictionaryColumn", "AllTypesValueColumn",
                                  "AllTypesDictionaryColumn", "AllTypesMixColumn", "TwoColumnsNoValues",
                                  "EmptyStringsValueColumn"])
def test_export_writes_reference_bytes(hy, tmp_path, name):
    out = tmp_path / "export_test.bin"
    hy.export_binary(cases(hy)[name], str(out))
    with open(os.path.join(BIN, name + ".bin"), "rb") as fx:
        assert out.read_bytes() == fx.read()


@pytest.mark.parametrize("name", ["AllTypesNullValues", "AllTypesDictionaryNullValues"])
def test_import_null_values(hy, name):
    cols = [("a", "Int"), ("b", "Float"), ("c", "Long"), ("d", "String"), ("e", "Double")]
    assert_ordered(hy.import_binary(os.path.join(BIN, name + ".bin")), make(hy, cols, NULL5, 100_000, True))


def test_import_empty_strings_dictionary_and_float_table(hy):
    got = hy.import_binary(os.path.join(BIN, "EmptyStringsDictionaryColumn.bin"))
    assert [r[0] for r in got.rows()] == [""] * 5
    assert_ordered(hy.import_binary(os.path.join(BIN, "float.bin")), hy.load_table(tbl("float.tbl"), 5))


@pytest.mark.parametrize("name", ["InvalidColumnType", "InvalidAttributeVectorWidth", "DoesNotExist"])
def test_import_rejects(hy, name):
    with pytest.raises(Exception):
        hy.import_binary(os.path.join(BIN, name + ".bin"))


def test_round_trip_keeps_dictionary_bytes(hy, tmp_path):
    """Export -> import of a dictionary-encoded numeric table reproduces every attribute-vector byte (what
    load_to_device uploads to HBM) and every value."""
    import numpy as np

    rng = np.random.default_rng(4)
    q = rng.integers(1, 51, 70_000).astype(np.int32)
    k = rng.integers(0, 1 << 20, 70_000).astype(np.int32)
    t = hy.Table.from_arrays([("q", hy.DataType.Int, False), ("k", hy.DataType.Int, False)], [q, k], [], 30_000)
    hy.encode_columns(t, [0], hy.EncodingType.Dictionary)
    out = tmp_path / "rt.bin"
    hy.export_binary(t, str(out))
    back = hy.import_binary(str(out))
    assert back.chunk_count() == 3 and back.row_count() == 70_000
    assert [r for r in back.rows()] == [r for r in t.rows()]
    hy.export_binary(back, str(tmp_path / "rt2.bin"))
    assert (tmp_path / "rt2.bin").read_bytes() == out.read_bytes()


@pytest.mark.gpu
def test_imported_table_on_device(hy, oracle, tmp_path):
    """A table read from a binary file goes to HBM as stored (load_to_device: the attribute vectors are the file's
    bytes) and the device TableScan over it equals the oracle's scan of the original table."""
    import numpy as np

    from helpers import assert_identical, wrap

    rng = np.random.default_rng(9)
    q = rng.integers(1, 51, 90_000).astype(np.int32)
    k = rng.integers(-1000, 1000, 90_000).astype(np.int32)
    t = hy.Table.from_arrays([("q", hy.DataType.Int, False), ("k", hy.DataType.Int, False)], [q, k], [], 20_000)
    hy.encode_columns(t, [0], hy.EncodingType.Dictionary)
    hy.export_binary(t, str(tmp_path / "t.bin"))
    back = hy.import_binary(str(tmp_path / "t.bin"))
    hy.load_to_device(back)
    s = hy.TableScan(wrap(hy, back), 0, hy.PredicateCondition.LessThan, 24)
    s.execute()
    assert [r for r in back.rows()] == [r for r in t.rows()]
    assert_identical(s.get_output(), oracle.table_scan(back, 0, hy.PredicateCondition.LessThan, 24, []))
