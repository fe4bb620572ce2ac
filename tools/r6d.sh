set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_join_direct_gpu.py tests/test_string_scan_gpu.py tests/test_scan_gpu.py tests/test_operator_surface_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python bench.py --workload scan --steps 20 --warmup 5 --op-kernel-stats > $O/scan.json 2> $O/scan.err || { echo SCAN_FAILED; tail -20 $O/scan.err; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --op-kernel-stats > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -20 $O/bench.err; exit 1; }
echo ok
