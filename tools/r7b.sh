set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_join_gpu.py tests/test_scan_join_gpu.py tests/test_join_direct_gpu.py tests/test_sizes_gpu.py -x -q --timeout 120 --timeout-method thread > $O/b_join.txt 2>&1 || { tail -30 $O/b_join.txt; exit 1; }
timeout -k 10 200 python bench.py --workload join-only --no-cpu-baseline > $O/b_joinonly.json 2> $O/b_bench.err
HY_JOIN_STASH=0 timeout -k 10 200 python bench.py --workload join-only --no-cpu-baseline > $O/b_joinonly_nostash.json 2>> $O/b_bench.err
timeout -k 10 200 python bench.py --workload join-only --no-cpu-baseline > $O/b_joinonly2.json 2>> $O/b_bench.err
timeout -k 10 300 python -u bench.py --through-operators --steps 5 --warmup 2 --no-cpu-baseline > $O/b_ops.json 2> $O/b_ops.err
