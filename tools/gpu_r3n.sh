#!/bin/bash
# round-3 GPU check N: TPC-H 3 + widening-row profiles, the operator path (--through-operators), config-5 rehearsal
# (2 ranks on one GPU, gloo, SF10)
mkdir -p gpurun_out
bash tools/profile_r03.sh r03 q3 widen > gpurun_out/r3n_prof.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --through-operators --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3n_ops.json 2> gpurun_out/r3n_ops.err || exit 2
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --workload q3 --dist-backend gloo --sf 10 --steps 3 --warmup 1 > gpurun_out/r3n_q3n2.json 2> gpurun_out/r3n_q3n2.err || exit 3
