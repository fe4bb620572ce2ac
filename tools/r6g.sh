set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_stream_lifetime_gpu.py tests/test_scan_gpu.py tests/test_string_scan_gpu.py tests/test_operator_surface_gpu.py tests/test_scan_join_gpu.py -x -q --capture=sys --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python bench.py --workload scan --steps 20 --warmup 5 --op-kernel-stats > $O/scan.json 2> $O/scan.err || { echo SCAN_FAILED; tail -20 $O/scan.err; exit 1; }
HY_SCAN_TWO_PASS=0 timeout -k 10 300 python bench.py --workload scan --steps 20 --warmup 5 --no-cpu-baseline --op-kernel-stats > $O/scan_1pass.json 2> $O/scan_1pass.err || { echo SCAN1_FAILED; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- python bench.py --workload scan --steps 20 --warmup 5 --no-cpu-baseline > $O/scan_prof.json 2> $O/scan_prof.err || { echo PROF_FAILED; exit 1; }
echo ok
