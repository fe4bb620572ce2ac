#!/bin/bash
# round-3 GPU check P: JoinHash output chunks built by per-thread arenas in parallel: join / operator tests, the
# operator-path bench with its phase trace
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_join_gpu.py tests/test_scan_join_gpu.py tests/test_tpch_queries.py tests/test_validate.py tests/test_string_scan_gpu.py tests/test_bp128.py tests/test_scan_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r3p_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit 1;; esac
HY_OP_TRACE=1 timeout -k 10 400 python -u bench.py --through-operators --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3p_ops.json 2> gpurun_out/r3p_ops.err || exit 2
