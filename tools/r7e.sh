set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
HY_JOIN_STASH=0 timeout -k 10 300 python -u -m pytest tests/test_operator_surface_gpu.py -x -q -k "concurrent" > $O/e1.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_join_gpu.py tests/test_operator_surface_gpu.py -x -q -k "probe_skew or concurrent" > $O/e2.txt 2>&1
