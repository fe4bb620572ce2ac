#!/bin/bash
# round-3 GPU check: size tests + distributed Q3 test, headline bench with its output check, 2-rank Q3 rehearsal
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist_q3_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3b_pytest.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r3b_bench.json 2> gpurun_out/r3b_bench.err || exit 2
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --workload q3 --dist-backend gloo --sf 10 --steps 3 --warmup 1 > gpurun_out/r3b_q3n2.json 2> gpurun_out/r3b_q3n2.err || exit 3
