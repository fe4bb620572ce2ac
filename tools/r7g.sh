set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
bash tools/r7f.sh default 10
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/h_pytest.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/h_smoke.txt 2>&1
timeout -k 10 300 python -u bench.py --through-operators --steps 5 --warmup 2 --no-cpu-baseline > $O/h_ops.json 2> $O/h_ops.err
timeout -k 10 240 python bench.py > $O/h_bench.json 2> $O/h_bench.err
