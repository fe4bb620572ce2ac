set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
HY_DEBUG_RING=1 timeout -k 10 600 python -u -m pytest tests/test_join_direct_gpu.py tests/test_scan_join_gpu.py tests/test_string_scan_gpu.py -x -q --capture=sys --timeout 300 --timeout-method thread -k "prepared or string_synthetic" > $O/tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
echo ok
