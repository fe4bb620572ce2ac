set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_join_direct_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r6_b_direct.txt 2>&1 || { echo DIRECT_FAILED; tail -40 $O/r6_b_direct.txt; exit 1; }
tail -2 $O/r6_b_direct.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --op-kernel-stats > $O/r6_b_bench.json 2> $O/r6_b_bench.err || { echo BENCH_FAILED; tail -30 $O/r6_b_bench.err; exit 1; }
timeout -k 10 500 python -u -m pytest tests/test_scan_join_gpu.py tests/test_join_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r6_b_tests.txt 2>&1 || { echo TESTS_FAILED; tail -40 $O/r6_b_tests.txt; exit 1; }
tail -2 $O/r6_b_tests.txt
