#!/bin/bash
# round-3 GPU check: full GPU suite (test failures do not stop the benches; crashes / timeouts do), headline A/B
# (mask sub 2 / sub 1 / compact), TPC-H 1 with and without the RowID prefetch, operator path, distributed Q3 2-rank
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 300 --timeout-method thread > gpurun_out/r3d_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_bench.err || exit 2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-plan > gpurun_out/r3d_bench_noplan.json 2> gpurun_out/r3d_bench_noplan.err || exit 9
HY_PART_SUB_FILTERED=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3d_bench_sub1.json 2> gpurun_out/r3d_bench_sub1.err || exit 3
HY_FILTER_COMPACT=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3d_bench_compact.json 2> gpurun_out/r3d_bench_compact.err || exit 4
timeout -k 10 300 python -u bench.py --workload q1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3d_q1.json 2> gpurun_out/r3d_q1.err || exit 5
HY_AGG_PREFETCH=1 timeout -k 10 300 python -u bench.py --workload q1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3d_q1_pf.json 2> gpurun_out/r3d_q1_pf.err || exit 6
timeout -k 10 400 python -u bench.py --through-operators --steps 5 --warmup 2 > gpurun_out/r3d_ops.json 2> gpurun_out/r3d_ops.err || exit 7
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --workload q3 --dist-backend gloo --sf 10 --steps 3 --warmup 1 > gpurun_out/r3d_q3n2.json 2> gpurun_out/r3d_q3n2.err || exit 8
