set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_operator_surface_gpu.py tests/test_join_gpu.py tests/test_stream_lifetime_gpu.py -x -q --timeout 120 --timeout-method thread > $O/d_ops_tests.txt 2>&1 || { tail -30 $O/d_ops_tests.txt; exit 1; }
timeout -k 10 300 python -u bench.py --through-operators --steps 5 --warmup 2 --no-cpu-baseline > $O/d_ops.json 2> $O/d_ops.err
for g in 1 0; do for ov in 1 0; do
HY_PLAN_GRAPH=$g HY_JOIN_OVERLAP=$ov timeout -k 10 200 python bench.py --no-cpu-baseline > $O/d_bench_g${g}_ov${ov}.json 2>> $O/d_bench.err
done; done
export TMPDIR=/tmp
cd /tmp
HY_PLAN_GRAPH=0 timeout -s KILL 300 rocprofv3 --kernel-trace -d $O/d_trace -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/d_bench_tr.json 2> $O/d_trace.err
python3 $R/tools/trace_step.py $O/d_trace/run_kernel_trace.csv > $O/d_step_eager.txt 2>&1 || true
find $O/d_trace -name "*.csv" -size +5M -delete
