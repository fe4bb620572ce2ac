#!/bin/bash
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_lanes
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_WAVES --kernel-include-regex 'agg_dense_lanes' -d $R/gpurun_out/pmc_lanes/a -o run -f csv -- python3 $R/bench.py --workload q1 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_lanes/a.json 2> $R/gpurun_out/pmc_lanes/a.err
timeout -s KILL 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex 'agg_dense_lanes' -d $R/gpurun_out/pmc_lanes/b -o run -f csv -- python3 $R/bench.py --workload q1 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_lanes/b.json 2> $R/gpurun_out/pmc_lanes/b.err
echo done
