#!/bin/bash
# round-3 GPU check A: full GPU suite (test failures do not stop the benches; crashes / timeouts do), headline
# variants (plan + graph default, plan without graph, per-call path, compact pass)
mkdir -p gpurun_out
timeout -k 10 660 python -u -m pytest tests -m gpu -q --maxfail 30 --timeout 300 --timeout-method thread > gpurun_out/r3e_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3e_bench.json 2> gpurun_out/r3e_bench.err || exit 2
HY_PLAN_GRAPH=0 timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3e_bench_nograph.json 2> gpurun_out/r3e_bench_nograph.err || exit 3
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-plan > gpurun_out/r3e_bench_noplan.json 2> gpurun_out/r3e_bench_noplan.err || exit 4
HY_FILTER_COMPACT=1 timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3e_bench_compact.json 2> gpurun_out/r3e_bench_compact.err || exit 5
