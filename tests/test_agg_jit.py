"""The plan-compiled aggregation kernel (hyrise_amd_agg_jit.cpp) on the CPU: its generated source for a TPC-H-1
shaped plan compiles with hiprtc for gfx950 (no GPU needed). Its results are checked on the GPU against the oracle by
tests/test_aggregate_lanes_gpu.py (stream mode "j", the default) and tests/test_tpch_queries.py."""
import ctypes
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _lib():
    return importlib.import_module("hyrise-1_amd").capi.lib


def test_generated_source_is_straight_line():
    L = _lib()
    buf = ctypes.create_string_buffer(1 << 20)
    assert L.hy_internal_agg_jit_selftest(1, buf, len(buf)) == 0
    src = buf.value.decode()
    assert 'extern "C" __global__' in src and "agg_jit(JitArgs a)" in src
    # plan constants are literals: no plan tables are read, every column has its own width-specialised load
    assert "load_column<1>(d0" in src and "load_column<4>(d3" in src and "load_column<2>(fdata" in src
    assert "__uint_as_float(0xbf800000u)" in src  # the -1 of 1 - l_discount
    assert src.count("acc[j][") >= 10


def test_generated_kernel_compiles_for_gfx950():
    L = _lib()
    buf = ctypes.create_string_buffer(1 << 16)
    rc = L.hy_internal_agg_jit_selftest(0, buf, len(buf))
    assert rc == 0, buf.value.decode()
