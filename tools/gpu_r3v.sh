#!/bin/bash
# round-3 GPU check V: batched LIKE id sets: scan / string / TPC-H tests, widening-row bench
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_scan_gpu.py tests/test_string_scan_gpu.py tests/test_tpch_queries.py tests/test_tpch_sf001.py tests/test_bp128.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3v_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 500 python -u tools/bench_widen.py --steps 3 > gpurun_out/r3v_widen_ops.jsonl 2> gpurun_out/r3v_widen.err || exit 2
