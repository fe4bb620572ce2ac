#!/bin/bash
# round-3 GPU check T: agg_dense_vec with the next step's loads pipelined: aggregate tests + TPC-H 1 (both instances)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_aggregate_lanes_gpu.py tests/test_aggregate_expr_gpu.py tests/test_aggregate_gpu.py tests/test_tpch_queries.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3t_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 240 python -u bench.py --workload q1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3t_q1.json 2> gpurun_out/r3t_q1.err || exit 3
HY_VEC_ALLF=0 timeout -k 10 240 python -u bench.py --workload q1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3t_q1_generic.json 2> gpurun_out/r3t_q1_generic.err || exit 4
