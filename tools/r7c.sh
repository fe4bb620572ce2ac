set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace -d $O/c_trace -o run -f csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/c_bench.json 2> $O/c_trace.err
python3 $R/tools/trace_step.py $O/c_trace/run_kernel_trace.csv > $O/c_step.txt 2>&1 || true
find $O/c_trace -name "*.csv" -size +5M -delete
