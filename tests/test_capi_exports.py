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


def test_projection_multi_checks_its_programs_without_a_device(hy):
    """hy_projection_multi validates every program against the input (program count, column index, node types, stack
    depth) before any device work, and an input without rows returns HY_OK without touching the device."""
    capi = hy.capi
    L = capi.lib
    L.hy_projection_multi.restype = ctypes.c_int
    col = (capi.AggColumn * 1)()
    col[0].value_type, col[0].pos_group, col[0].n_chunks = capi.HY_TYPE_INT32, -1, 0
    inp = capi.AggInput(0, None, None, 0, col, 1)

    def call(progs, outs=None):
        arrs = [(capi.ExprNode * len(p))(*p) for p in progs]
        ptrs = (ctypes.c_void_p * max(1, len(arrs)))(*[ctypes.addressof(a) for a in arrs])
        lens = (ctypes.c_uint32 * max(1, len(arrs)))(*[len(p) for p in progs])
        out = (ctypes.c_void_p * max(1, len(arrs)))(*([0x1000] * len(arrs) if outs is None else outs))
        return L.hy_projection_multi(ctypes.byref(inp), ptrs, lens, len(arrs), out, None, None, 0, None)

    column = capi.ExprNode(capi.HY_EXPR_COLUMN, capi.HY_TYPE_INT32, 0, 0, 0)
    one = capi.ExprNode(capi.HY_EXPR_VALUE, capi.HY_TYPE_INT32, 0, 0, 1)
    add = capi.ExprNode(capi.HY_EXPR_ADD, capi.HY_TYPE_INT32, capi.HY_TYPE_INT32, 0, 0)
    assert call([]) == 1                                                  # no program
    assert call([[column]] * 17) == 1                                     # more than HY_PROJ_MAX_OUTPUTS
    assert call([[column], [capi.ExprNode(capi.HY_EXPR_COLUMN, capi.HY_TYPE_INT32, 0, 3, 0)]]) == 1  # column index
    assert call([[capi.ExprNode(capi.HY_EXPR_COLUMN, capi.HY_TYPE_FLOAT, 0, 0, 0)]]) == 1            # column type
    assert call([[column, add]]) == 1                                     # stack underflow
    assert call([[column, one]]) == 1                                     # two values left
    assert call([[column, one, add], [column]]) == 0                      # valid, no rows: nothing to do
