#!/bin/bash
# SQ counters of agg_dense_lanes (two passes, each within the per-block counter limits) over one TPC-H 1 step.
# usage: tools/pmc_lanes.sh <tag> [extra bench.py args]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-q1}
shift || true
export TMPDIR=/tmp
O=$R/gpurun_out/pmc_lanes_$TAG
mkdir -p $O
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_WAVES --kernel-include-regex 'agg_dense' -d $O/a -o run -f csv -- python3 $R/bench.py --workload q1 --steps 1 --warmup 0 --no-cpu-baseline "$@" > $O/a.json 2> $O/a.err
timeout -s KILL 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex 'agg_dense' -d $O/b -o run -f csv -- python3 $R/bench.py --workload q1 --steps 1 --warmup 0 --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err
echo done
