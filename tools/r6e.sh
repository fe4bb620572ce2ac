set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
HY_DEBUG_RING=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --capture=sys --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 120 ./tools/scan_probe > $O/scan_probe.jsonl 2>&1 || { echo PROBE_FAILED; exit 1; }
timeout -k 10 300 python bench.py --workload scan --steps 20 --warmup 5 --no-cpu-baseline --op-kernel-stats > $O/scan.json 2> $O/scan.err || { echo SCAN_FAILED; tail -20 $O/scan.err; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --op-kernel-stats > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -20 $O/bench.err; exit 1; }
echo ok
