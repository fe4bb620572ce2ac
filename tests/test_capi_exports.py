"""The C-ABI library loads without a GPU and exports every entry point include/hyrise_amd.h declares."""
import ctypes


def test_library_exports_all_declared_symbols(hy):
    declared = hy.capi.declared_symbols()
    assert len(declared) >= 20
    missing = [s for s in declared if not hasattr(hy.capi.lib, s)]
    assert not missing, missing


def test_build_info_names_gfx950(hy):
    assert b"gfx950" in hy.capi.lib.hy_build_info()


def test_radix_bits_formula(hy):
    # reference join_hash.cpp:640-668 evaluated in float arithmetic (15M -> 13, 150M -> 16)
    assert hy.join_radix_bits(15_000_000, 4) == 13
    assert hy.join_radix_bits(150_000_000, 4) == 16
    assert hy.join_radix_bits(1_500_000, 4) == 9
    assert hy.join_radix_bits(15_000, 4) == 3
    assert hy.join_radix_bits(0, 4) == 0
    assert hy.capi.lib.hy_join_radix_bits(15_000_000, 4) == 13


def test_device_count_without_gpu_is_a_number(hy):
    n = hy.capi.device_count()
    assert n >= 0
