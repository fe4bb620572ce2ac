set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_scan_join_gpu.py tests/test_join_gpu.py -k "row_ids or plan_cache or deferred_scan" -x -q --timeout 120 --timeout-method thread > $O/a_rowids.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/a_pytest.txt 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/a_bench.json 2> $O/a_bench.err
HY_PLAN_GRAPH=0 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/a_bench_eager.json 2>> $O/a_bench.err
timeout -k 10 300 python -u bench.py --through-operators --steps 5 --warmup 2 --no-cpu-baseline > $O/a_ops.json 2> $O/a_ops.err
