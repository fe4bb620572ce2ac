set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/i_smoke.txt 2>&1
timeout -k 10 240 python bench.py > $O/i_bench.json 2> $O/i_bench.err
timeout -k 10 200 python bench.py --workload scan > $O/i_scan.json 2>> $O/i_bench.err
timeout -k 10 200 python bench.py --workload join-only > $O/i_joinonly.json 2>> $O/i_bench.err
timeout -k 10 300 python bench.py --workload q1 --no-cpu-baseline > $O/i_q1.json 2>> $O/i_bench.err
timeout -k 10 300 python bench.py --workload q3 --no-cpu-baseline > $O/i_q3.json 2>> $O/i_bench.err
timeout -k 10 300 python -u bench.py --through-operators --steps 5 --warmup 2 --no-cpu-baseline > $O/i_ops.json 2>> $O/i_bench.err
