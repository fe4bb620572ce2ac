#!/bin/bash
# round-3 GPU check M: build side overlapped on a second stream: join tests, headline (overlap on / off), Q3, Q1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_join_gpu.py tests/test_scan_join_gpu.py tests/test_dist_join_gpu.py tests/test_sizes_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r3m_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3m_bench.json 2> gpurun_out/r3m_bench.err || exit 2
HY_JOIN_OVERLAP=0 timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3m_bench_seq.json 2> gpurun_out/r3m_bench_seq.err || exit 3
HY_PLAN_GRAPH=0 timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3m_bench_nograph.json 2> gpurun_out/r3m_bench_nograph.err || exit 4
timeout -k 10 240 python -u bench.py --workload q3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3m_q3.json 2> gpurun_out/r3m_q3.err || exit 5
