set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/f_pytest.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/f_smoke.txt 2>&1
timeout -k 10 240 python bench.py > $O/f_bench.json 2> $O/f_bench.err
timeout -k 10 200 python bench.py --workload scan > $O/f_scan.json 2>> $O/f_bench.err
timeout -k 10 200 python bench.py --workload join-only > $O/f_joinonly.json 2>> $O/f_bench.err
timeout -k 10 300 python bench.py --workload q1 --no-cpu-baseline > $O/f_q1.json 2>> $O/f_bench.err
timeout -k 10 300 python bench.py --workload q3 --no-cpu-baseline > $O/f_q3.json 2>> $O/f_bench.err
timeout -k 10 300 python -u bench.py --through-operators --steps 5 --warmup 2 --no-cpu-baseline > $O/f_ops.json 2>> $O/f_bench.err
