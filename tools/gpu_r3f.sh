#!/bin/bash
# round-3 GPU check B: TPC-H 1 (default / RowID prefetch / fused scan) + PMC of agg_dense_lanes, operator path,
# distributed Q3 2-rank rehearsal
mkdir -p gpurun_out
timeout -k 10 240 python -u bench.py --workload q1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3f_q1.json 2> gpurun_out/r3f_q1.err || exit 1
HY_AGG_PREFETCH=1 timeout -k 10 240 python -u bench.py --workload q1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3f_q1_pf.json 2> gpurun_out/r3f_q1_pf.err || exit 2
timeout -k 10 240 python -u bench.py --workload q1 --q1-fused --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3f_q1_fused.json 2> gpurun_out/r3f_q1_fused.err || exit 3
bash tools/pmc_lanes.sh > gpurun_out/r3f_pmc_lanes.txt 2>&1 || exit 4
timeout -k 10 400 python -u bench.py --through-operators --steps 5 --warmup 2 > gpurun_out/r3f_ops.json 2> gpurun_out/r3f_ops.err || exit 5
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --workload q3 --dist-backend gloo --sf 10 --steps 3 --warmup 1 > gpurun_out/r3f_q3n2.json 2> gpurun_out/r3f_q3n2.err || exit 6
