set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/j_pytest1.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/j_pytest2.txt 2>&1
timeout -k 10 300 python -u bench.py --through-operators --steps 5 --warmup 2 --no-cpu-baseline > $O/j_ops.json 2> $O/j_ops.err
