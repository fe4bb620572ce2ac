"""hyrise-1_amd — MI355X (gfx950) execution layer for Hyrise's TableScan / JoinHash / Aggregate hot path.

The package directory name contains a hyphen, so import it with ``importlib.import_module("hyrise-1_amd")``.
It loads the in-tree native libraries built by ``make`` (``_lib/``):

* ``libhyrise_amd.so``   — hand-written HIP kernels + the C-ABI of ``include/hyrise_amd.h``
* ``libhyrise_host.so``  — host operator layer (Table/Chunk/columns, TableScan/JoinHash/Aggregate drop-ins)
* ``_hyrise_host*.so``   — Python bindings of the host layer

There is no CPU fallback: operators raise if the HIP library reports no device.
"""
import glob
import importlib.machinery
import importlib.util
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "_lib")


def _load_extension(name):
    cands = glob.glob(os.path.join(LIB_DIR, name + "*.so"))
    if not cands:
        raise ImportError(f"hyrise-1_amd: native module {name} not built (run `make` at the repo root)")
    if name in sys.modules:
        return sys.modules[name]
    loader = importlib.machinery.ExtensionFileLoader(name, cands[0])
    spec = importlib.util.spec_from_file_location(name, cands[0], loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    sys.modules[name] = mod
    return mod


_host = _load_extension("_hyrise_host")

# Re-export the reference vocabulary.
DataType = _host.DataType
PredicateCondition = _host.PredicateCondition
JoinMode = _host.JoinMode
TableType = _host.TableType
EncodingType = _host.EncodingType
AggregateFunction = _host.AggregateFunction
Table = _host.Table
Chunk = _host.Chunk
BaseColumn = _host.BaseColumn
ReferenceColumn = _host.ReferenceColumn
AbstractOperator = _host.AbstractOperator
TableWrapper = _host.TableWrapper
TableScan = _host.TableScan
ColumnParameter = _host.ColumnParameter
ParameterID = _host.ParameterID
Validate = _host.Validate
TransactionContext = _host.TransactionContext
MAX_COMMIT_ID = _host.MAX_COMMIT_ID
JoinHash = _host.JoinHash
Aggregate = _host.Aggregate
AggregateColumnDefinition = _host.AggregateColumnDefinition
Projection = _host.Projection
ArithmeticOperator = _host.ArithmeticOperator
AbstractExpression = _host.AbstractExpression
PQPColumnExpression = _host.PQPColumnExpression
ValueExpression = _host.ValueExpression
ParameterExpression = _host.ParameterExpression
ArithmeticExpression = _host.ArithmeticExpression
expression_common_type = _host.expression_common_type
LogicError = _host.LogicError
load_table = _host.load_table
import_binary = _host.import_binary
export_binary = _host.export_binary
load_to_device = _host.load_to_device
VectorCompressionType = _host.VectorCompressionType
compress_vector = _host.compress_vector
encode_chunks = _host.encode_chunks
encode_all_chunks = _host.encode_all_chunks
encode_columns = _host.encode_columns
synchronize = _host.synchronize
join_hashed_type = _host.join_hashed_type
join_radix_bits = _host.join_radix_bits
device_count = _host.device_count
build_info = _host.build_info
op_trace_enable = _host.op_trace_enable
op_trace_take = _host.op_trace_take
join_plan_cache_stats = _host.join_plan_cache_stats
join_plan_cache_clear = _host.join_plan_cache_clear
join_plan_cache_set_capacity = _host.join_plan_cache_set_capacity
pool_stats = _host.pool_stats
device_memory = _host.device_memory
host_cpu_share = _host.host_cpu_share
release_drain = _host.release_drain
set_job_scheduler = _host.set_job_scheduler
DescriptionMode = _host.DescriptionMode

from . import capi  # noqa: E402  (ctypes view of the C-ABI)
