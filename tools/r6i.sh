set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_join_gpu.py tests/test_scan_join_gpu.py tests/test_join_direct_gpu.py -x -q --capture=sys --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python bench.py --workload join-only --steps 10 --warmup 3 --op-kernel-stats > $O/joinonly.json 2> $O/joinonly.err || { echo JO_FAILED; tail -20 $O/joinonly.err; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -20 $O/bench.err; exit 1; }
echo ok
