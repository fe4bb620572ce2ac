#!/bin/bash
# round-3 GPU check S: the multi-GPU headline at its real per-rank size, rehearsed as 2 ranks on one GPU (gloo
# transport), strong scaling SF100: the distributed JoinHash's step 1 / exchange / step 2 at 300M lineitem rows per rank
mkdir -p gpurun_out
timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --dist-backend gloo --steps 2 --warmup 1 > gpurun_out/r3s_n2.json 2> gpurun_out/r3s_n2.err || exit 1
